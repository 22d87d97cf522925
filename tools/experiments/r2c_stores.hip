// Memory-pattern probe for the r2c split pass (k_r2c_fused, csrc/hsfft_pass_pf.h): the same
// row loads ([t][q], t < 512, 8-column tiles lo / hi), twiddle streams and four output
// streams (X[k], X[N-k], X[h-k], X[h+k]), without the FFT arithmetic.  Timing only.
//   hipcc -O3 --offload-arch=gfx950 -o gpurun_out/r2c_stores tools/experiments/r2c_stores.hip
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

constexpr unsigned B = 4096, P = 512, H = B * P, N = 2 * H;

__device__ __forceinline__ unsigned xcd_remap(unsigned blk)
{
    const unsigned nwg = gridDim.x, q8 = nwg / 8, r8_ = nwg % 8, xcd = blk % 8;
    return (xcd < r8_ ? xcd * (q8 + 1) : r8_ * (q8 + 1) + (xcd - r8_) * q8) + blk / 8;
}

// MODE bits: 1 data loads, 2 twiddle loads (stage-2 run + twiddle2), 4 aligned streams
// (X[N-k], X[h-k]), 8 straddling streams (X[k], X[h+k]), 16 straddle removed (qlo = 8j)
template <int MODE>
__global__ __launch_bounds__(512, 2) void k_probe(const double2 *in, const double2 *tw, const double2 *w2t,
                                                  double2 *out)
{
    extern __shared__ double2 lds[];
    const unsigned tiles = B / 16 + 1;
    const unsigned blk = xcd_remap(blockIdx.x), b = blk / tiles, jr = blk % tiles;
    /* bit 6: tile order rotated per row (rows 64 MB apart alias in the DRAM channel map) */
    const unsigned j = (MODE & 64) ? (jr + b * 97u) % tiles : jr;
    if (j == tiles - 1) return;
    const unsigned t = threadIdx.x, g = t & 7, jt = t >> 3;
    const double2 *row = in + (size_t)b * H;
    double2 *X = out + (size_t)b * N;
    const unsigned qlo = (MODE & 16) ? 8 * j : 8 * j + 1, qhi = B - 8 * j - 8;
    double ar = 0, ai = 0;
    if (MODE & 1) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = row[(jt + i * 64) * B + qhi + g];
            const double2 w = row[(jt + i * 64) * B + qlo + g];
            ar += v.x + w.x;
            ai += v.y + w.y;
        }
    }
    if (MODE & 2) {
#pragma unroll
        for (int i = 0; i < 7; i++) { /* stage-2 runs of both tiles: 7 x 64 x 8 entries each */
            const double2 v = tw[B * 64 - 1 + 7 * (qhi + B * (jt & 63)) + i];
            const double2 w = tw[B * 64 - 1 + 7 * (qlo + B * (jt & 63)) + i];
            ar += v.x + w.x;
            ai += v.y - w.y;
        }
    }
    lds[t] = make_double2(ar, ai);
    __syncthreads();
    const double2 z = lds[t ^ 1];
#pragma unroll
    for (int jj = 0; jj < 8; jj++) {
        /* bit 5: every stream aligned (the primary streams at 8j, the mirrored at 8j + 1) */
        const unsigned u = jt + jj * 64, k = u * B + qlo + g, hk = H - k;
        const unsigned kp = (MODE & 32) ? u * B + 8 * j + g : k;
        double2 w = z;
        if (MODE & 2) {
            const double2 a = w2t[k], c = w2t[hk];
            w.x += a.x + c.x;
            w.y += a.y + c.y;
        }
        if (MODE & 8) X[kp] = w;
        if (MODE & 4) X[N - k] = make_double2(w.x, -w.y);
        if (MODE & 4) X[hk] = make_double2(w.y, w.x);
        if (MODE & 8) X[H + kp] = make_double2(-w.x, w.y);
    }
}


// one output stream: tile j's 8 columns (lanes g) of every u-row, k = U(u) * B + J(j) + G(g);
// f bit 0: j descending (q = B - 8 - 8j), bit 1: u descending (u -> 1023 - u), bit 2: lanes descending,
// bit 3: second copy of the stream H elements (32 MB) further on
__global__ __launch_bounds__(512, 2) void k_one(double2 *out, int f, int rows, int D)
{
    extern __shared__ double2 lds[];
    const unsigned tiles = B / 16 + 1;
    const unsigned blk = xcd_remap(blockIdx.x), b = blk / tiles, j = blk % tiles;
    if (j == tiles - 1) return;
    const unsigned t = threadIdx.x, g = (f & 4) ? 7 - (t & 7) : (t & 7), jt = t >> 3;
    double2 *X = out + (size_t)b * N;
    /* bit 12: straddling tiles (q0 = 8j + 1, one element in the next 128-B line) */
    const unsigned q = ((f & 1) ? B - 8 - 8 * j : 8 * j) + ((f & 4096) ? 1 : 0);
    lds[t] = make_double2(t, j);
    __syncthreads();
    const double2 z = lds[t ^ 1];
    /* bit 6: mirror stores use u of jj+4; bit 7: all primary stores first, then the mirrors;
     * bit 8: mirror stores use the u of the thread jt ^ 32 (another wave) */
    if (f & 8192) { /* aligned half lines: 16 u-rows x 64 B per instruction (bit 14: the two
                       * halves of a line from two different workgroups: tiles j and j ^ 1) */
        const unsigned l = t & 63, w = t >> 6;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = w * 16 + (l >> 2) + 128 * (jj >> 1);
            const unsigned qq = (f & 16384) ? 8 * (j & ~1u) + 4 * (j & 1) + (l & 3) + 8 * (jj & 1)
                                            : q + 4 * (jj & 1) + (l & 3);
            X[u * B + qq] = z;
        }
        return;
    }
#pragma unroll
    for (int jj = 0; jj < 8; jj++) {
        const unsigned u0 = jt + jj * 64, u = (f & 2) ? 1023 - u0 : u0, k = u * B + q + g;
        X[k] = z;
        if (f & 8) X[(k + H) % N] = z;
        if (!(f & 128)) {
            const unsigned um = ((f & 256) ? (jt ^ 32) : jt) + ((f & 64) ? ((jj + 4) & 7) : jj) * 64;
            /* D: the mirror stores belong to the tile D tiles back (a deferred write) */
            const unsigned qm = (f & 1) ? q : (q + B - 8 * D) % (B / 2), km = um * B + qm + g;
            /* bit 9: mirror stores non-temporal; bit 10: mirror stores into row b + 1 (the
             * row-walking schedule's deferred write of the previous row) */
            double2 *Y = (f & 1024) ? out + (size_t)((b + 1) % rows) * N : X;
            if (f & 512) {
                if (f & 16) __builtin_nontemporal_store(z.x, &Y[2 * H - km].x), __builtin_nontemporal_store(z.y, &Y[2 * H - km].y);
                if (f & 32) __builtin_nontemporal_store(z.x, &Y[H - km].x), __builtin_nontemporal_store(z.y, &Y[H - km].y);
            } else {
                if (f & 16) Y[2 * H - km] = z;
                if (f & 32) Y[H - km] = z;
            }
        }
    }
    if (f & 128) {
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * 64, k = u * B + q + g;
            if (f & 16) X[2 * H - k] = z;
            if (f & 32) X[H - k] = z;
        }
    }
}

// contiguous copy of the same bytes for reference (16 B per lane, 1 KiB per wave instruction)
__global__ __launch_bounds__(256) void k_copy(const double2 *in, double2 *out, size_t nin)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < nin) {
        const double2 v = in[i];
        out[2 * i - (i & 63)] = v;
        out[2 * i - (i & 63) + 64] = v;
    }
}

template <int MODE>
float run(const double2 *in, const double2 *tw, const double2 *w2t, double2 *out, int rows, int reps)
{
    const unsigned tiles = B / 16 + 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t lds = (512 * 8 + 504) * 16;
    CK(hipFuncSetAttribute((const void *)k_probe<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_probe<MODE>, dim3(tiles * rows), dim3(512), lds, 0, in, tw, w2t, out);
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_probe<MODE>, dim3(tiles * rows), dim3(512), lds, 0, in, tw, w2t, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv)
{
    const int rows = argc > 1 ? atoi(argv[1]) : 512, reps = 5;
    double2 *in, *tw, *w2t, *out;
    CK(hipMalloc(&in, (size_t)rows * H * 16));
    CK(hipMalloc(&out, ((size_t)rows * N + 64) * 16)); /* + pad: X[N - 0] of the no-straddle probe */
    CK(hipMalloc(&tw, (size_t)N * 16));
    CK(hipMalloc(&w2t, (size_t)N * 16));
    CK(hipMemset(in, 0, (size_t)rows * H * 16));
    CK(hipMemset(tw, 0, (size_t)N * 16));
    CK(hipMemset(w2t, 0, (size_t)N * 16));
    const double gb_in = rows * (double)H * 16 / 1e9, gb_out = 2 * gb_in;
    printf("rows %d: data in %.1f GB, out %.1f GB\n", rows, gb_in, gb_out);
#define R(M, label)                                                                                             \
    {                                                                                                           \
        const float ms = run<M>(in, tw, w2t, out, rows, reps);                                                  \
        printf("mode %2d %-44s %8.3f ms\n", M, label, ms);                                                      \
    }

    const int fl[] = {0};
    const int fl_unused[] = {0, 8, 16, 16 | (1 << 16), 16 | (8 << 16), 16 | (64 << 16), 16 | (128 << 16), 16 | 1024 | (64 << 16), 56, 56 | (64 << 16), 56 | (128 << 16), 56 | (32 << 16)};
    for (int f : fl) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const unsigned tiles = B / 16 + 1;
        const size_t lds = (512 * 8 + 504) * 16;
        CK(hipFuncSetAttribute((const void *)k_one, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(k_one, dim3(tiles * rows), dim3(512), lds, 0, out, f & 0xffff, rows, f >> 16);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_one, dim3(tiles * rows), dim3(512), lds, 0, out, f & 0xffff, rows, f >> 16);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("f=%4d D=%3d (j %s, u %s, lanes %s) k%s%s%s  %8.3f ms\n", f & 0xffff, f >> 16, f & 1 ? "desc" : "asc",
               f & 2 ? "desc" : "asc", f & 4 ? "desc" : "asc", f & 8 ? " +H+k" : "", f & 16 ? " +2H-k" : "", f & 32 ? " +H-k" : "", ms / reps);
    }
    R(31 - 16, "loads + twiddles + 4 streams (k_r2c_fused)");
    R(15 | 64, "same, tile order rotated per row");
    R(15 | 32, "same, all four streams aligned");
    R(15 | 32 | 64, "aligned + rotated");
    R(13 | 64, "loads + 4 streams, no twiddles, rotated");
    R(13 | 32, "loads + 4 aligned streams, no twiddles");
    R(12 | 32, "4 aligned streams only");
    R(13, "loads + 4 streams, no twiddles");
    R(29, "loads + 4 streams, no twiddles, no straddle");
    R(1 | 4, "loads + aligned streams");
    R(1 | 8, "loads + straddling streams");
    R(1 | 2, "loads + twiddles, no stores");
    R(1, "loads only");
    R(12, "4 streams only");
    R(4, "aligned streams only");
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const size_t nin = (size_t)rows * H;
        hipLaunchKernelGGL(k_copy, dim3((nin + 255) / 256), dim3(256), 0, 0, in, out, nin);
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_copy, dim3((nin + 255) / 256), dim3(256), 0, 0, in, out, nin);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("contiguous copy, same bytes (1 read, 2 writes)           %8.3f ms  (%.2f TB/s)\n", ms / reps,
               (gb_in + gb_out) / ms / reps);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
