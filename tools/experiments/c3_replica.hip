// Replica of the 12600-point row kernel (BASELINE config 3, 65536 x 12600 complex f64) with a
// synthetic arithmetic load, to decide between one row per CU (mr::k_row2's geometry: one
// 512-thread workgroup per CU, 98 KiB split exchange image), TWO rows per CU (two 512-thread
// workgroups of <= 128 VGPRs, each exchanging through a half-row image in two rounds) and HALF a
// row per workgroup (two workgroups per row, the transpose between them through global memory)
// before building either (round-4 verdict item 3).  The two-rows-per-CU variant does not fit:
// its 25 points per thread (100 VGPRs) plus the exchange stash spill 132 dwords at the 128-VGPR
// bound even with no butterfly temporaries, so it is compiled but not timed.  Each workgroup walks rows: loads its row
// (25 points per thread, 16-B coalesced), runs S "stages" of K complex multiply-adds per point,
// X exchanges through LDS (a fixed permutation of the row), and stores the row.  Timing only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/experiments/c3_replica tools/experiments/c3_replica.hip
// Usage: c3_replica [rows=65536]   (prints ms per launch for a grid of variants)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

constexpr int N = 12600, T = 512, PPT = 25; /* points per thread (25 * 512 = 12800 >= N) */
constexpr int HALF = 13 * T; /* the two-row variant's image: slots 0..12 of every thread */

__device__ __forceinline__ unsigned perm(unsigned p) { return (p * 41u) % (unsigned)N; }

/* the synthetic stage: K complex multiply-adds per point (a twiddle multiply plus butterfly
 * additions cost ~ 5-7 such per point per radix stage in the real kernel) */
__device__ __forceinline__ void alu(double2 (&x)[PPT], int K, double2 w)
{
#pragma unroll 1
    for (int k = 0; k < K; k++) {
#pragma unroll
        for (int i = 0; i < PPT; i++) {
            const double r = x[i].x * w.x - x[i].y * w.y + 0.5, m = x[i].x * w.y + x[i].y * w.x - 0.25;
            x[i] = make_double2(r, m);
        }
    }
}

/* TWO = 0: one workgroup per CU, full-row split image (12600 doubles); TWO = 1: two per CU,
 * half-row image (6300 doubles), every exchange in two rounds per part */
template <int TWO>
__global__ __launch_bounds__(512, TWO ? 4 : 2) void k_row_rep(const double2 *in, double2 *out, int rows, int S, int K,
                                                              int X)
{
    extern __shared__ double img[];
    const unsigned tid0 = threadIdx.x;
    const double2 w = make_double2(0.9999, 0.0001 * (double)(tid0 & 7));
#pragma unroll 1
    for (int r = blockIdx.x; r < rows; r += gridDim.x) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid)); /* no per-element index hoisted out of the row loop (spills) */
        const double2 *row = in + (size_t)r * N;
        double2 x[PPT];
#pragma unroll
        for (int i = 0; i < PPT; i++) {
            const unsigned p = tid + T * i;
            x[i] = row[p < (unsigned)N ? p : 0];
        }
        int xdone = 0;
#pragma unroll 1
        for (int s = 0; s < S; s++) {
            asm volatile("" : "+v"(tid));
            alu(x, K, w);
            if (xdone < X && s < S - 1) { /* exchange: new point q takes old point perm(q) */
                xdone++;
#pragma unroll 1
                for (int part = 0; part < 2; part++) {
                    asm volatile("" : "+v"(tid));
                    if (!TWO) {
#pragma unroll
                        for (int i = 0; i < PPT; i++) {
                            const unsigned p = tid + T * i;
                            if (p < (unsigned)N) img[p] = part ? x[i].y : x[i].x;
                        }
                        __syncthreads();
#pragma unroll
                        for (int i = 0; i < PPT; i++) {
                            const unsigned q = tid + T * i;
                            const double v = img[perm(q < (unsigned)N ? q : 0)];
                            if (part) x[i].y = v;
                            else x[i].x = v;
                        }
                        __syncthreads();
                    } else { /* half 0 = slots 0..12, half 1 = slots 13..24: a slot whose new
                              * value comes from half 0 but whose old value is written in round 1
                              * waits in a stash (12 doubles) */
                        constexpr int H0 = 13;
                        double stash[PPT - H0];
#pragma unroll
                        for (int i = 0; i < H0; i++) img[tid + T * i] = part ? x[i].y : x[i].x;
                        __syncthreads();
#pragma unroll
                        for (int i = 0; i < PPT; i++) {
                            const unsigned q = tid + T * i, src = perm(q < (unsigned)N ? q : 0);
                            const double v = img[src < (unsigned)(T * H0) ? src : 0];
                            if (i < H0) {
                                if (src < (unsigned)(T * H0)) {
                                    if (part) x[i].y = v;
                                    else x[i].x = v;
                                }
                            } else {
                                stash[i - H0] = v;
                            }
                        }
                        __syncthreads();
#pragma unroll
                        for (int i = H0; i < PPT; i++) {
                            const unsigned p = tid + T * i;
                            if (p < (unsigned)N) img[p - T * H0] = part ? x[i].y : x[i].x;
                        }
                        __syncthreads();
#pragma unroll
                        for (int i = 0; i < PPT; i++) {
                            const unsigned q = tid + T * i, src = perm(q < (unsigned)N ? q : 0);
                            const bool hi = src >= (unsigned)(T * H0);
                            const double v = img[hi ? src - T * H0 : 0];
                            double nv = v;
                            if (i >= H0 && !hi) nv = stash[i - H0];
                            if (i >= H0 || hi) {
                                if (part) x[i].y = nv;
                                else x[i].x = nv;
                            }
                        }
                        __syncthreads();
                    }
                }
            }
        }
        double2 *orow = out + (size_t)r * N;
#pragma unroll
        for (int i = 0; i < PPT; i++) {
            const unsigned p = tid + T * i;
            if (p < (unsigned)N) orow[p] = x[i];
        }
    }
}

/* HALF-ROW design: two workgroups per row, one per half (6300 points, 13 per thread), each with
 * its own half image; the row's transpose between the two halves of the stage list goes through
 * a scratch slot in global memory with the agent-scope hand-off (plain stores, workgroup
 * barrier, one lane's release fence + counter add; partner: relaxed poll, acquire, barrier,
 * loads -- MI355X_MICROARCH.md Valid forms).  Partners are blocks b and b ^ 8 (the same XCD under
 * round-robin dispatch: speed only).  Slots double-buffered by row parity; a workgroup writes the
 * slot of row k+2 only after the partner counted row k+1 in, i.e. after it read row k. */
constexpr int HP = 6300, HPPT = 13;

__global__ __launch_bounds__(512, 4) void k_half_rep(const double2 *in, double2 *out, double2 *scr, unsigned *cnt,
                                                     int rows, int S, int K, int X)
{
    extern __shared__ double img[];
    const unsigned tid0 = threadIdx.x, b = blockIdx.x, h = (b >> 3) & 1, partner = b ^ 8u;
    const unsigned pair = (b >> 4) * 8 + (b & 7), npairs = gridDim.x / 2;
    const double2 w = make_double2(0.9999, 0.0001 * (double)(tid0 & 7));
    __shared__ unsigned ok;
    unsigned k = 0;
#pragma unroll 1
    for (int r = pair; r < rows; r += npairs, k++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid)); /* no per-element index hoisted out of the row loop (spills) */
        const double2 *row = in + (size_t)r * N + h * HP;
        double2 x[HPPT];
#pragma unroll
        for (int i = 0; i < HPPT; i++) {
            const unsigned p = tid + T * i;
            x[i] = row[p < (unsigned)HP ? p : 0];
        }
        int xdone = 0;
#pragma unroll 1
        for (int s = 0; s < S; s++) {
            asm volatile("" : "+v"(tid));
#pragma unroll 1
            for (int kk = 0; kk < K; kk++) {
#pragma unroll
                for (int i = 0; i < HPPT; i++) {
                    const double rr = x[i].x * w.x - x[i].y * w.y + 0.5, m = x[i].x * w.y + x[i].y * w.x - 0.25;
                    x[i] = make_double2(rr, m);
                }
            }
            if (s == S / 2 - 1) { /* the row's transpose: through the global slots */
                double2 *mine = scr + ((size_t)pair * 4 + (k & 1) * 2 + h) * HP;
#pragma unroll
                for (int i = 0; i < HPPT; i++) {
                    const unsigned p = tid + T * i;
                    if (p < (unsigned)HP) mine[p] = x[i];
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __hip_atomic_fetch_add(cnt + b * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    unsigned spins = 0;
                    while (__hip_atomic_load(cnt + partner * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k + 1 &&
                           ++spins < (1u << 26))
                        __builtin_amdgcn_s_sleep(1);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    ok = spins < (1u << 26);
                }
                __syncthreads();
                /* new point q of this half: half from the own slot, half from the partner's
                 * (one base, 32-bit offsets: the two slots of a row parity are adjacent) */
                const char *pb = (const char *)(scr + ((size_t)pair * 4 + (k & 1) * 2) * HP);
                unsigned src = (tid * 41u) % (unsigned)(2 * HP);
#pragma unroll
                for (int i = 0; i < HPPT; i++) {
                    const unsigned off = src < (unsigned)HP ? h * HP + src : (1 - h) * HP + src - HP;
                    x[i] = *(const double2 *)(pb + off * 16u);
                    src += (T * 41u) % (unsigned)(2 * HP);
                    src = src >= (unsigned)(2 * HP) ? src - 2 * HP : src;
                }
            } else if (xdone < X - 1 && s < S - 1) { /* local exchange through the half image (X - 1 of them: the transpose is the X-th) */
                xdone++;
#pragma unroll 1
                for (int part = 0; part < 2; part++) {
                    asm volatile("" : "+v"(tid));
#pragma unroll
                    for (int i = 0; i < HPPT; i++) {
                        const unsigned p = tid + T * i;
                        if (p < (unsigned)HP) img[p] = part ? x[i].y : x[i].x;
                    }
                    __syncthreads();
#pragma unroll
                    for (int i = 0; i < HPPT; i++) {
                        const unsigned q = tid + T * i;
                        const double v = img[(q < (unsigned)HP ? q : 0) * 37u % (unsigned)HP];
                        if (part) x[i].y = v;
                        else x[i].x = v;
                    }
                    __syncthreads();
                }
            }
        }
        double2 *orow = out + (size_t)r * N + h * HP;
#pragma unroll
        for (int i = 0; i < HPPT; i++) {
            const unsigned p = tid + T * i;
            if (p < (unsigned)HP) orow[p] = x[i];
        }
    }
}

int main(int argc, char **argv)
{
    const int rows = argc > 1 ? atoi(argv[1]) : 65536;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t bytes = (size_t)rows * N * 16;
    double2 *in, *out;
    CK(hipMalloc((void **)&in, bytes));
    CK(hipMalloc((void **)&out, bytes));
    CK(hipMemset(in, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds1 = N * 8, lds2 = HALF * 8;
    CK(hipFuncSetAttribute((const void *)k_row_rep<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1));
    CK(hipFuncSetAttribute((const void *)k_row_rep<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2));
    int occ0 = 0, occ1 = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, (const void *)k_row_rep<0>, 512, lds1));
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, (const void *)k_row_rep<1>, 512, lds2));
    printf("c3 replica: %d rows of %d points, %d CUs, workgroups per CU: one-row %d, two-row %d\n", rows, N, cus, occ0,
           occ1);
    printf("copy-equivalent: %.1f GB moved per launch\n", 2.0 * bytes / 1e9);
    const int S = 6;
    double2 *scr;
    unsigned *cnt;
    const int g2 = cus * 2;
    CK(hipMalloc((void **)&scr, (size_t)g2 * 2 * HP * 16 * 2));
    CK(hipMalloc((void **)&cnt, (size_t)g2 * 32 * 4));
    const size_t ldsh = HP * 8;
    CK(hipFuncSetAttribute((const void *)k_half_rep, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsh));
    int occh = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occh, (const void *)k_half_rep, 512, ldsh));
    printf("half-row workgroups per CU %d\n", occh);
    const int Ks[] = {0, 2, 4, 6, 8};
    for (int ki = 0; ki < 5; ki++)
        for (int v = 0; v < 3; v++) {
            if (v == 1) continue; /* the two-row variant spills at 128 VGPRs (see the header) */
            const int X = 3, K = Ks[ki];
            auto go = [&]() {
                if (v == 2) {
                    CK(hipMemsetAsync(cnt, 0, (size_t)g2 * 32 * 4, 0));
                    hipLaunchKernelGGL(k_half_rep, dim3(g2), dim3(512), ldsh, 0, in, out, scr, cnt, rows, S, K, X);
                } else {
                    hipLaunchKernelGGL(k_row_rep<0>, dim3(cus), dim3(512), lds1, 0, in, out, rows, S, K, X);
                }
            };
            go();
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            float tot = 0;
            for (int it = 0; it < 3; it++) {
                CK(hipEventRecord(e0, 0));
                go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                tot += ms;
            }
            printf("alu K %d  %s  %.3f ms  (%.1f GSamples/s)\n", K,
                   v == 2 ? "half row per workgroup (2 per CU, global transpose)" : "one row per CU (full image)     ",
                   tot / 3, (double)rows * N / (tot / 3 / 1e3) / 1e9);
            fflush(stdout);
        }
    return 0;
}
