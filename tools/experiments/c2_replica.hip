// Data-movement replica of 2^20 c2c (BASELINE config 2, 4096 x 2^20 complex f64): the loads,
// stores and in-launch hand-off of the two-launch path and of the best one-launch schedule
// (round 2's fixed-role launch: pass-A items of 4 columns x 2048 points, pass-B tiles of 8
// q-columns x 512 points, per-row counters, bounded throttle), with NO arithmetic and no LDS
// exchange.  What it measures is the floor the data movement alone sets -- a one-launch
// schedule cannot run faster than its replica.  Timing only (results are copies).
//   hipcc -O3 --offload-arch=gfx950 -o tools/experiments/c2_replica tools/experiments/c2_replica.hip
// Usage: c2_replica [rows=4096]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr unsigned N = 1u << 20;  /* points per row */
constexpr unsigned MA = 512;      /* pass-A columns (t < 2048 points each, stride 512) */
constexpr unsigned QB = 2048;     /* pass-B columns (m < 512 points each, stride 2048) */
constexpr unsigned ITEMS = 128;   /* pass-A items per row: 4 columns each */
constexpr unsigned TILES = 256;   /* pass-B tiles per row: 8 columns each */
constexpr unsigned CS = 32;       /* counter stride: one 128-B line per counter */
constexpr unsigned long long T_LIMIT = 1ull << 28; /* bounded waits: ~2.7 s of the 100 MHz clock */

typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned xcd_remap(unsigned blk)
{
    const unsigned nwg = gridDim.x, q8 = nwg / 8, r8_ = nwg % 8, xcd = blk % 8;
    return (xcd < r8_ ? xcd * (q8 + 1) : r8_ * (q8 + 1) + (xcd - r8_) * q8) + blk / 8;
}

/* pass-A item movement: 4 adjacent columns m0..m0+3 of one row, 2048 points each, read as
 * 64-B row segments (4 lanes per segment, like pf::k_firstq's paired loads), written as the
 * four contiguous 32-KiB output columns [m][u] (k_firstq's store pattern) */
template <bool SC1>
__device__ __forceinline__ void a_item(const double2 *in, double2 *out, unsigned m0)
{
    const unsigned c = threadIdx.x & 3, tq = threadIdx.x >> 2; /* tq < 128 */
    u4 v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const unsigned t = tq + 128 * i;
        const double2 x = in[(size_t)t * MA + m0 + c];
        __builtin_memcpy(&v[i], &x, 16);
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)(N * 16u), 0x00020000);
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const unsigned t = tq + 128 * i;
        __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, ((m0 + c) * 2048u + t) * 16u, 0, SC1 ? 16 : 0);
    }
}

/* pass-B tile movement: 8 adjacent q-columns of one row, 512 points each (128-B segments at
 * a 32-KiB stride, like pf::k_b512), written back in place */
template <bool SC1>
__device__ __forceinline__ void b_tile(double2 *row, unsigned q0)
{
    const unsigned g = threadIdx.x & 7, jt = threadIdx.x >> 3; /* jt < 64 */
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, (int)(N * 16u), 0x00020000);
    u4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((jt + 64 * i) * QB + q0 + g) * 16u, 0, SC1 ? 16 : 0);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; i++) __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, ((jt + 64 * i) * QB + q0 + g) * 16u, 0, 0);
}

template <bool SC1>
__device__ __forceinline__ void b_load(const double2 *row, unsigned q0, u4 (&v)[8])
{
    const unsigned g = threadIdx.x & 7, jt = threadIdx.x >> 3;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)row, 0, (int)(N * 16u), 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((jt + 64 * i) * QB + q0 + g) * 16u, 0, SC1 ? 16 : 0);
}

__device__ __forceinline__ void b_store(double2 *row, unsigned q0, const u4 (&v)[8])
{
    const unsigned g = threadIdx.x & 7, jt = threadIdx.x >> 3;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, (int)(N * 16u), 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; i++) __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, ((jt + 64 * i) * QB + q0 + g) * 16u, 0, 0);
}

/* two-launch replica: pass A (grid = rows x 128 items), pass B (rows x 256 tiles) */
__global__ __launch_bounds__(512) void k_pass_a(const double2 *in, double2 *out)
{
    const unsigned blk = xcd_remap(blockIdx.x), row = blk / ITEMS, it = blk % ITEMS;
    a_item<false>(in + (size_t)row * N, out + (size_t)row * N, it * 4);
}

__global__ __launch_bounds__(512) void k_pass_b(double2 *out)
{
    const unsigned blk = xcd_remap(blockIdx.x), row = blk / TILES, tile = blk % TILES;
    b_tile<false>(out + (size_t)row * N, tile * 8);
}

struct OArgs {
    const double2 *in;
    double2 *out;
    unsigned *adone, *bdone, *err;
    unsigned rows, na, nb, lag, pref;
};

/* B poller: wait until row `row` has all its pass-A items, then one agent acquire; false on
 * timeout */
__device__ __forceinline__ bool b_wait(const OArgs &a, unsigned row, unsigned long long t0, unsigned *flag)
{
    if (threadIdx.x == 0) {
        unsigned bad = 0;
        while (__hip_atomic_load(&a.adone[row * CS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ITEMS) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > T_LIMIT) {
                __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                bad = 1;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *flag = bad;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*flag) == 0;
}

/* one-launch replica (fixed roles): A workgroups take items it = a, a + na, ... in row order
 * and stay at most `lag` rows ahead of the pass-B tiles; B workgroups own tiles b, b + nb, ...
 * and walk the rows.  Hand-off per row: sc1 item stores, every wave's vmcnt(0), barrier, one
 * lane's agent add; the B poller's relaxed poll, agent acquire, barrier, sc1 loads
 * (Guideline 16 R1). */
__global__ __launch_bounds__(512) void k_one(OArgs a)
{
    __shared__ unsigned flag;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (blockIdx.x < a.na) {
        const unsigned total = a.rows * ITEMS;
        for (unsigned it = blockIdx.x; it < total; it += a.na) {
            const unsigned row = it / ITEMS, m0 = (it % ITEMS) * 4;
            if (row >= a.lag && threadIdx.x == 0) { /* throttle (bounded: gives up, not a dependency) */
                while (__hip_atomic_load(&a.bdone[(row - a.lag) * CS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < TILES &&
                       __builtin_amdgcn_s_memrealtime() - t0 < T_LIMIT)
                    __builtin_amdgcn_s_sleep(2);
            }
            __syncthreads();
            a_item<true>(a.in + (size_t)row * N, a.out + (size_t)row * N, m0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add(&a.adone[row * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    const unsigned b = blockIdx.x - a.na;
    for (unsigned tile = b; tile < TILES; tile += a.nb) {
        if (a.pref) { /* the next row's tile loads while this row's tile is stored */
            u4 v0[8], v1[8];
            if (!b_wait(a, 0, t0, &flag)) return;
            b_load<true>(a.out, tile * 8, v0);
            for (unsigned row = 0; row < a.rows; row += 2) {
                const bool more = row + 1 < a.rows;
                if (more) {
                    if (!b_wait(a, row + 1, t0, &flag)) return;
                    b_load<true>(a.out + (size_t)(row + 1) * N, tile * 8, v1);
                }
                b_store(a.out + (size_t)row * N, tile * 8, v0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) __hip_atomic_fetch_add(&a.bdone[row * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!more) break;
                const bool more2 = row + 2 < a.rows;
                if (more2) {
                    if (!b_wait(a, row + 2, t0, &flag)) return;
                    b_load<true>(a.out + (size_t)(row + 2) * N, tile * 8, v0);
                }
                b_store(a.out + (size_t)(row + 1) * N, tile * 8, v1);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0) __hip_atomic_fetch_add(&a.bdone[(row + 1) * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            continue;
        }
        for (unsigned row = 0; row < a.rows; row++) {
            if (!b_wait(a, row, t0, &flag)) return;
            b_tile<true>(a.out + (size_t)row * N, tile * 8);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add(&a.bdone[row * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

__global__ __launch_bounds__(256) void k_copy(const u4 *a, u4 *b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

static float timed(hipEvent_t e0, hipEvent_t e1, void (*launch)(void *), void *ctx, int reps)
{
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
        CK(hipEventRecord(e0));
        launch(ctx);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

struct Ctx {
    double2 *in, *out;
    unsigned *ctr, *err;
    size_t ctr_bytes;
    unsigned rows, na, nb, lag, pref;
};

int main(int argc, char **argv)
{
    const unsigned rows = argc > 1 ? (unsigned)atoi(argv[1]) : 4096;
    const size_t bytes = (size_t)rows * N * 16;
    Ctx c;
    c.rows = rows;
    CK(hipMalloc(&c.in, bytes));
    CK(hipMalloc(&c.out, bytes));
    c.ctr_bytes = (size_t)2 * rows * CS * sizeof(unsigned) + 64;
    CK(hipMalloc(&c.ctr, c.ctr_bytes));
    c.err = c.ctr + 2 * rows * CS;
    CK(hipMemset(c.in, 0, bytes));
    CK(hipMemset(c.out, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double gs = (double)rows * N / 1e9, alg = (double)rows * N * 32.0;
    auto report = [&](const char *what, float ms) {
        printf("%-58s %8.2f ms  %7.1f GSamples/s-equivalent  %6.0f GB/s algorithmic (32 B/sample)\n", what, ms, gs / (ms / 1e3),
               alg / (ms / 1e3) / 1e9);
        fflush(stdout);
    };
    report("stream copy in -> out (16 B per lane)", timed(e0, e1, [](void *p) {
               Ctx *c = (Ctx *)p;
               hipLaunchKernelGGL(k_copy, dim3(65536), dim3(256), 0, 0, (const u4 *)c->in, (u4 *)c->out, (size_t)c->rows * N);
           }, &c, 3));
    float ta = timed(e0, e1, [](void *p) {
        Ctx *c = (Ctx *)p;
        hipLaunchKernelGGL(k_pass_a, dim3(c->rows * ITEMS), dim3(512), 0, 0, c->in, c->out);
    }, &c, 3);
    float tb = timed(e0, e1, [](void *p) {
        Ctx *c = (Ctx *)p;
        hipLaunchKernelGGL(k_pass_b, dim3(c->rows * TILES), dim3(512), 0, 0, c->out);
    }, &c, 3);
    report("two-launch replica: pass A movement", ta);
    report("two-launch replica: pass B movement", tb);
    report("two-launch replica: A + B", ta + tb);
    const unsigned cfg[][4] = {{256, 256, 8, 0}, {256, 256, 100000, 0}, {128, 384, 4, 0}, {256, 256, 4, 1}, {256, 256, 8, 1},
                               {256, 256, 16, 1}, {256, 256, 100000, 1}, {128, 384, 8, 1}, {192, 320, 8, 1}};
    for (auto &g : cfg) {
        c.na = g[0];
        c.nb = g[1];
        c.lag = g[2];
        c.pref = g[3];
        float t = timed(e0, e1, [](void *p) {
            Ctx *c = (Ctx *)p;
            CK(hipMemsetAsync(c->ctr, 0, c->ctr_bytes, 0));
            OArgs a;
            a.in = c->in;
            a.out = c->out;
            a.adone = c->ctr;
            a.bdone = c->ctr + c->rows * CS;
            a.err = c->err;
            a.rows = c->rows;
            a.na = c->na;
            a.nb = c->nb;
            a.lag = c->lag;
            a.pref = c->pref;
            hipLaunchKernelGGL(k_one, dim3(c->na + c->nb), dim3(512), 0, 0, a);
        }, &c, 3);
        unsigned err = 0;
        CK(hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
        char name[96];
        snprintf(name, sizeof name, "one-launch replica: %u A + %u B wgs, lag %u rows%s%s", g[0], g[1], g[2],
                 g[3] ? ", B prefetch" : "", err ? " [WAIT TIMED OUT]" : "");
        report(name, t);
    }
    return 0;
}
