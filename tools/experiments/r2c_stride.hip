// Memory-pattern probe for the r2c split walk (k_r2c_walk1, csrc/hsfft_pass_pf.h): the walk's
// tile loads (512 rows t x one 128-B segment, rows `pitch` entries apart) and its four output
// streams (512 rows u x 128 B, rows B = 4096 entries = 64 KiB apart), in the walk's order (walks
// of 32 tile pairs, 8 rotation classes, two 512-thread workgroups per CU), without arithmetic.
// Question: is the walk bound by the 64-KiB row stride of its accesses (DRAM channel / bank
// aliasing), and does a padded row pitch for the intermediate Z (library-owned, so its layout
// is free) cure the loads?  Timing only.
//   hipcc -O3 --offload-arch=gfx950 -o tools/experiments/r2c_stride tools/experiments/r2c_stride.hip
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

constexpr unsigned B = 4096, P = 512, H = B * P, N = 2 * H, T = 32, TILES = B / 16, W = TILES / T;

__device__ __forceinline__ unsigned xcd_remap(unsigned blk)
{
    const unsigned nwg = gridDim.x, q8 = nwg / 8, r8_ = nwg % 8, xcd = blk % 8;
    return (xcd < r8_ ? xcd * (q8 + 1) : r8_ * (q8 + 1) + (xcd - r8_) * q8) + blk / 8;
}

// MODE bit 0: tile loads (hi + lo), bit 1: four output streams, bit 2: output rows padded too
// (X row u at u * (B + xpad): NOT the reference layout, for the comparison only)
template <int MODE>
__global__ __launch_bounds__(512, 4) void k_walk(const double2 *Z, unsigned pitch, unsigned zdist, double2 *X,
                                                 unsigned xpad, unsigned sink)
{
    extern __shared__ double2 lds[];
    const unsigned blk = xcd_remap(blockIdx.x), b = blk / W, s = blk % W;
    const unsigned t = threadIdx.x, g = t & 7, jt = t >> 3;
    const double2 *row = Z + (size_t)b * zdist;
    double2 *Xr = X + (size_t)b * (N + (MODE & 4 ? 2 * 512 * xpad : 0));
    const unsigned j0 = s * T, o = ((b % 8) * T) / 8;
    const unsigned xb = (MODE & 4) ? B + xpad : B;
    double ar = 0, ai = 0;
#pragma unroll 1
    for (unsigned jr = 0; jr < T; jr++) {
        const unsigned j = j0 + (o + jr) % T, qlo = 8 * j + 1, qhi = B - 8 * j - 8;
        double hr[8], hi[8], lr[8], li[8];
        if (MODE & 1) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = row[(size_t)(jt + 64 * i) * pitch + qhi + g];
                hr[i] = v.x;
                hi[i] = v.y;
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = row[(size_t)(jt + 64 * i) * pitch + qlo + g];
                lr[i] = v.x;
                li[i] = v.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) hr[i] = hi[i] = lr[i] = li[i] = (double)(i + j);
        }
        /* one barrier per tile pair: the real walk's phases keep the workgroup together */
        lds[t] = make_double2(hr[0] + lr[7], hi[3] + li[4]);
        __syncthreads();
        const double2 z = lds[t ^ 1];
        __syncthreads();
        if (MODE & 2) {
#pragma unroll
            for (int jj = 0; jj < 8; jj++) {
                const unsigned u = jt + jj * 64, p = u * xb + 8 * j + g, m = (P - 1 - u) * xb + (B - 8 * j - 8) + g;
                Xr[p] = make_double2(hr[jj] + z.x, lr[jj]);
                Xr[(size_t)H + p] = make_double2(hi[jj], li[jj] + z.y);
                Xr[m] = make_double2(lr[jj], hr[jj]);
                Xr[(size_t)H + m] = make_double2(li[jj], hi[jj]);
            }
        } else {
#pragma unroll
            for (int jj = 0; jj < 8; jj++) {
                ar += hr[jj] + lr[jj];
                ai += hi[jj] - li[jj];
            }
            ar += z.x;
        }
    }
    if (ar == (double)sink && ai == 1.5) X[t] = make_double2(ar, ai); /* never true: keeps the loads */
}


// stores only, tiles CW columns wide (CW * 16 B contiguous per u-row and stream): the four
// streams of a tile pair written as 512 / (64 / CW) wave instructions of 64 / CW rows x CW entries
template <int CW>
__global__ __launch_bounds__(512, 4) void k_storesw(double2 *X, unsigned sink)
{
    extern __shared__ double2 lds[];
    constexpr unsigned TW = TILES * 8 / CW, WW = TW / T; /* tile pairs per row at this width, walks */
    const unsigned blk = xcd_remap(blockIdx.x), b = blk / WW, s = blk % WW;
    const unsigned t = threadIdx.x, g = t % CW, jt = t / CW; /* 512 / CW rows per pass */
    constexpr unsigned RPP = 512 / CW, NPASS = P / RPP;
    double2 *Xr = X + (size_t)b * N;
    const unsigned j0 = s * T, o = ((b % 8) * T) / 8;
    const double2 z = make_double2((double)t, (double)sink);
#pragma unroll 1
    for (unsigned jr = 0; jr < T; jr++) {
        const unsigned j = j0 + (o + jr) % T, q = CW * j, qm = B - CW * j - CW;
        lds[t] = z;
        __syncthreads();
        const double2 zz = lds[t ^ 1];
        __syncthreads();
#pragma unroll
        for (unsigned pp = 0; pp < NPASS; pp++) {
            const unsigned u = jt + pp * RPP, p = u * B + q + g, m = (P - 1 - u) * B + qm + g;
            Xr[p] = zz;
            Xr[(size_t)H + p] = zz;
            Xr[m] = zz;
            Xr[(size_t)H + m] = zz;
        }
    }
}

template <int CW>
float run_w(double2 *X, int rows, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds = 80 * 1024;
    constexpr unsigned TW = TILES * 8 / CW, WW = TW / T;
    CK(hipFuncSetAttribute((const void *)k_storesw<CW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_storesw<CW>, dim3(WW * rows), dim3(512), lds, 0, X, 7u);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_storesw<CW>, dim3(WW * rows), dim3(512), lds, 0, X, 7u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <int MODE>
float run(const double2 *Z, unsigned pitch, double2 *X, unsigned xpad, int rows, int reps)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds = 80 * 1024; /* walk1's LDS: two workgroups per CU */
    const unsigned zdist = pitch * P;
    CK(hipFuncSetAttribute((const void *)k_walk<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_walk<MODE>, dim3(W * rows), dim3(512), lds, 0, Z, pitch, zdist, X, xpad, 7u);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL(k_walk<MODE>, dim3(W * rows), dim3(512), lds, 0, Z, pitch, zdist, X, xpad, 7u);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv)
{
    const int rows = argc > 1 ? atoi(argv[1]) : 512, reps = 5;
    const unsigned maxpad = 256;
    double2 *Z, *X;
    const size_t zbytes = (size_t)rows * (B + maxpad) * P * 16, xbytes = (size_t)rows * (N + 2 * 512 * maxpad) * 16;
    CK(hipMalloc(&Z, zbytes));
    CK(hipMalloc(&X, xbytes));
    CK(hipMemset(Z, 0, zbytes));
    CK(hipMemset(X, 0, xbytes));
    const double gbz = rows * (double)H * 16 / 1e9;
    printf("rows %d: Z %.1f GB read, X %.1f GB written; ms per %d rows (walk only)\n", rows, gbz, 2 * gbz, rows);
    const unsigned pads[] = {0, 8, 16, 64, 256};
    for (int rep = 0; rep < 2; rep++) {
        {
            const float m8 = run_w<8>(X, rows, reps), m16 = run_w<16>(X, rows, reps), m32 = run_w<32>(X, rows, reps),
                        m64 = run_w<64>(X, rows, reps);
            printf("stores only, tile width  8 / 16 / 32 / 64 entries: %.3f / %.3f / %.3f / %.3f ms (%.2f / %.2f / %.2f / %.2f TB/s)\n",
                   m8, m16, m32, m64, 2 * gbz / m8, 2 * gbz / m16, 2 * gbz / m32, 2 * gbz / m64);
        }
        for (unsigned pad : pads) {
            const float ms = run<1>(Z, B + pad, X, 0, rows, reps);
            printf("loads only, Z pitch B + %3u        %8.3f ms  (%.2f TB/s)\n", pad, ms, gbz / ms);
        }
        {
            const float ms = run<2>(Z, B, X, 0, rows, reps);
            printf("stores only (reference X layout)  %8.3f ms  (%.2f TB/s)\n", ms, 2 * gbz / ms);
        }
        for (unsigned pad : {8u, 64u}) {
            const float ms = run<6>(Z, B, X, pad, rows, reps);
            printf("stores only, X rows padded + %3u   %8.3f ms  (%.2f TB/s)\n", pad, ms, 2 * gbz / ms);
        }
        for (unsigned pad : pads) {
            const float ms = run<3>(Z, B + pad, X, 0, rows, reps);
            printf("loads + stores, Z pitch B + %3u    %8.3f ms  (%.2f TB/s)\n", pad, ms, 3 * gbz / ms);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
