// Occupancy replica for the r2c split walk (k_r2c_walk1, csrc/hsfft_pass_pf.h), VERDICT r5 item 2:
// would a walk with more workgroups per CU (or a loader wave feeding the compute waves) move the
// walk's bytes faster?  The replica moves exactly the walk's byte stream in the walk's order --
// per tile pair: the hi and lo tiles' 512 rows x 128 B (rows B = 4096 entries apart), the
// twiddle2 entries w2t[k] / w2t[h-k] of the pairs phase, and the four output streams X[k], X[h+k],
// X[N-k], X[h-k] on whole 128-B lines -- with NBAR workgroup barriers per tile pair (the walk has
// 6) and no FFT arithmetic, at
//   OCC workgroups of 512 threads per CU (LDS sized so that exactly OCC fit; launch bounds
//   asking for 2*OCC waves per SIMD, i.e. <= 256 / 128 / 85 / 64 VGPRs for OCC 1 / 2 / 3 / 4),
//   walks of T tile pairs,
//   LOADER 1: one extra wave per workgroup loads the NEXT tile pair's rows into LDS with
//   global_load_lds (16 B per lane) while the 8 compute waves store the current one from LDS.
// Timing only (results are meaningless); the walk itself takes 13.65 ms per 512 rows at HEAD.
//   hipcc -O3 --offload-arch=gfx950 -o tools/experiments/r2c_occ tools/experiments/r2c_occ.hip
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

constexpr unsigned B = 4096, P = 512, H = B * P, N = 2 * H, TILES = B / 16;

__device__ __forceinline__ unsigned xcd_remap(unsigned blk)
{
    const unsigned nwg = gridDim.x, q8 = nwg / 8, r8_ = nwg % 8, xcd = blk % 8;
    return (xcd < r8_ ? xcd * (q8 + 1) : r8_ * (q8 + 1) + (xcd - r8_) * q8) + blk / 8;
}

// register-path replica: every thread loads its 8 hi + 8 lo entries, NBAR barriers, then the
// pairs phase loads 16 twiddle2 entries and stores 32 entries (4 streams x 8)
template <int OCC, int T, int NBAR, bool LATE_LO>
__global__ __launch_bounds__(512, 2 * OCC) void k_occ(const double2 *Z, const double2 *w2t, double2 *X, unsigned sink)
{
    extern __shared__ double2 lds[];
    constexpr unsigned W = TILES / T;
    const unsigned blk = xcd_remap(blockIdx.x), b = blk / W, s = blk % W;
    const unsigned t = threadIdx.x, g = t & 7, jt = t >> 3;
    const double2 *row = Z + (size_t)b * H;
    double2 *Xr = X + (size_t)b * N;
    const unsigned j0 = s * T, o = ((b % 8) * T) / 8;
    double acc = 0;
#pragma unroll 1
    for (unsigned jr = 0; jr < T; jr++) {
        const unsigned j = j0 + (o + jr) % T, qlo = 8 * j + 1, qhi = B - 8 * j - 8;
        /* LATE_LO (needed at OCC >= 3, <= 85 VGPRs: holding both tiles' 16 entries spills): the lo
         * entries are loaded in the pairs loop, one per output group (same addresses, issued later) */
        double2 hv[8], lv[8];
#pragma unroll
        for (int i = 0; i < 8; i++) hv[i] = row[(size_t)(jt + 64 * i) * B + qhi + g];
        lds[t] = make_double2(hv[0].x + hv[7].x, hv[3].y);
        __syncthreads();
        if (!LATE_LO) {
#pragma unroll
            for (int i = 0; i < 8; i++) lv[i] = row[(size_t)(jt + 64 * i) * B + qlo + g];
        }
#pragma unroll
        for (int k = 1; k < NBAR; k++) {
            const double2 z = lds[t ^ k];
            __syncthreads();
            lds[t] = make_double2(z.x + (LATE_LO ? 1.0 : lv[k & 7].x), z.y + hv[k & 7].y);
            __syncthreads();
        }
        const double2 z = lds[t ^ 1];
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * 64, k = u * B + qlo + g, hk = H - k;
            if (LATE_LO) lv[jj] = row[(size_t)u * B + qlo + g];
            const double2 wk = w2t[k], whk = w2t[hk];
            const unsigned p = u * B + 8 * j + g, m = (P - 1 - u) * B + (B - 8 * j - 8) + g;
            Xr[p] = make_double2(hv[jj].x + wk.x, lv[jj].y + z.x);
            Xr[(size_t)H + p] = make_double2(hv[jj].y, lv[jj].x + whk.y);
            Xr[N - 1 - (size_t)p] = make_double2(lv[jj].x + wk.y, hv[jj].x);
            Xr[m] = make_double2(lv[jj].y, hv[jj].y + whk.x);
        }
        acc += z.x;
    }
    if (acc == (double)sink) X[t] = make_double2(acc, 1.0); /* never true */
}

// loader-wave replica: waves 0-7 store tile pair k from LDS (hi / lo rows staged there) while
// wave 8 issues global_load_lds of tile pair k+1 into the other half; one workgroup per CU
// (2 x 128 KiB would not fit: the staged pair is 64 KiB per tile, so ONE tile pair is staged,
// double-buffered by tile: hi(k+1) loads while lo(k) is stored, lo(k+1) while hi(k+1) is)
template <int T>
__global__ __launch_bounds__(576, 1) void k_occ_loader(const double2 *Z, const double2 *w2t, double2 *X, unsigned sink)
{
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    constexpr unsigned W = TILES / T;
    const unsigned blk = xcd_remap(blockIdx.x), b = blk / W, s = blk % W;
    const unsigned t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const double2 *row = Z + (size_t)b * H;
    double2 *Xr = X + (size_t)b * N;
    const unsigned j0 = s * T, o = ((b % 8) * T) / 8;
    /* buffer: [2][512 rows][8] double2 = 2 x 64 KiB */
    double acc = 0;
    auto tile_q = [&](unsigned step) -> unsigned { /* step 2k: hi of pair k, 2k+1: lo */
        const unsigned j = j0 + (o + step / 2) % T;
        return (step & 1) ? 8 * j + 1 : B - 8 * j - 8;
    };
    auto load_tile = [&](unsigned step) { /* wave 8: 512 rows x 8 entries = 4096 x 16 B, 64 per instruction */
        const unsigned q = tile_q(step);
        double2 *dst = lds + (step & 1) * 4096;
        for (unsigned it = 0; it < 64; it++) {
            const unsigned e = it * 64 + lane, r = e >> 3, c = e & 7;
            const double2 *src = row + (size_t)r * B + q + c;
            __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)(dst + it * 64),
                                             16, 0, 0);
        }
    };
    if (wave == 8) load_tile(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (unsigned step = 0; step < 2 * T; step++) {
        if (wave == 8) {
            if (step + 1 < 2 * T) load_tile(step + 1);
        } else {
            const unsigned q = tile_q(step), g = t & 7, jt = t >> 3;
            const double2 *src = lds + (step & 1) * 4096;
#pragma unroll
            for (int jj = 0; jj < 8; jj++) {
                const unsigned u = jt + jj * 64, k = u * B + q + g;
                const double2 v = src[u * 8 + g], wk = w2t[k < H ? k : k - H];
                if (step & 1) {
                    Xr[k] = make_double2(v.x + wk.x, v.y);
                    Xr[(size_t)H + k] = make_double2(v.y, v.x + wk.y);
                } else {
                    Xr[N - 1 - (size_t)k] = make_double2(v.x, v.y + wk.x);
                    Xr[H - 1 - (size_t)k] = make_double2(v.y + wk.y, v.x);
                }
                acc += v.x;
            }
        }
        /* the loader wave's DMA has landed; the store waves do NOT wait for their stores (raw
         * barrier: __syncthreads would drain every wave's vmcnt) */
        if (wave == 8) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    if (acc == (double)sink) X[t] = make_double2(acc, 1.0); /* never true */
}

template <int OCC, int T, int NBAR, bool LATE_LO = (OCC >= 3)>
float run(const double2 *Z, const double2 *w2t, double2 *X, int rows, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds = (160 * 1024) / OCC - 1024;
    constexpr unsigned W = TILES / T;
    CK(hipFuncSetAttribute((const void *)k_occ<OCC, T, NBAR, LATE_LO>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((k_occ<OCC, T, NBAR, LATE_LO>), dim3(W * rows), dim3(512), lds, 0, Z, w2t, X, 7u);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_occ<OCC, T, NBAR, LATE_LO>), dim3(W * rows), dim3(512), lds, 0, Z, w2t, X, 7u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    int per = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)k_occ<OCC, T, NBAR, LATE_LO>, 512, lds));
    printf("  OCC %d (API %d per CU) T %2d NBAR %d%s: %8.3f ms\n", OCC, per, T, NBAR, LATE_LO ? " late-lo" : "", ms / reps);
    return ms / reps;
}

template <int T>
float run_loader(const double2 *Z, const double2 *w2t, double2 *X, int rows, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds = 2 * 4096 * 16;
    constexpr unsigned W = TILES / T;
    CK(hipFuncSetAttribute((const void *)k_occ_loader<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_occ_loader<T>, dim3(W * rows), dim3(576), lds, 0, Z, w2t, X, 7u);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_occ_loader<T>, dim3(W * rows), dim3(576), lds, 0, Z, w2t, X, 7u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("  loader wave (1 WG/CU, 8 store waves + 1 global_load_lds wave) T %2d: %8.3f ms\n", T, ms / reps);
    return ms / reps;
}

int main(int argc, char **argv)
{
    const int rows = argc > 1 ? atoi(argv[1]) : 512, reps = 5;
    double2 *Z, *X, *w2t;
    const size_t zbytes = (size_t)rows * H * 16, xbytes = (size_t)rows * N * 16;
    CK(hipMalloc(&Z, zbytes));
    CK(hipMalloc(&X, xbytes));
    CK(hipMalloc(&w2t, (size_t)H * 16));
    CK(hipMemset(Z, 0, zbytes));
    CK(hipMemset(X, 0, xbytes));
    CK(hipMemset(w2t, 0, (size_t)H * 16));
    printf("rows %d: Z %.1f GB read, X %.1f GB written; ms per %d rows (walk replica, no FFT arithmetic)\n", rows,
           zbytes / 1e9, xbytes / 1e9, rows);
    for (int rep = 0; rep < 2; rep++) {
        printf("pass %d\n", rep);
        run<2, 32, 2>(Z, w2t, X, rows, reps);
        run<2, 32, 6>(Z, w2t, X, rows, reps);
        run<2, 32, 6, true>(Z, w2t, X, rows, reps);
        run<3, 32, 6>(Z, w2t, X, rows, reps);
        run<4, 32, 6>(Z, w2t, X, rows, reps);
        run<3, 16, 6>(Z, w2t, X, rows, reps);
        run<4, 16, 6>(Z, w2t, X, rows, reps);
        run<1, 32, 6>(Z, w2t, X, rows, reps);
        run_loader<32>(Z, w2t, X, rows, reps);
        run_loader<16>(Z, w2t, X, rows, reps);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
