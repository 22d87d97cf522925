/*
 * hsfft_device.hip -- HIP/CDNA4 (gfx950) device layer of libhsfft.so.
 *
 * Kernels
 *   k_pass_generic : one fused Stockham pass (any radix list, LDS ping-pong).  Replaces the
 *                    recursion + combine loops of mixed_radix_dit_rec (ref
 *                    src/highSpeedFFT.c:318-1629) for one range of stages.
 *   k_pass_r8      : hsfft_pass_r8.h -- register-resident radix-8 passes (hot path).
 *   k_fill_*       : splitmix64 synthetic inputs (bench / tests).
 *   k_r2c_post / k_c2r_pre : real-signal split / merge (ref src/real.c:108-132, :169-179).
 *   k_cmul / k_scale_real / k_copy_rows : convolution helpers (ref src/convolve.c:137-160).
 *
 * Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (no FMA contraction: the results
 * must be bit-identical to the reference's separately rounded multiplies and adds).
 */
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <vector>

#include "hsfft_butterfly.h"
#include "hsfft_internal.h"

namespace {

thread_local char g_err[512];

/* Lazily created per-device objects (streams, events): created once under g_init_mtx,
 * published through the atomic flags, so host threads may race on first use. */
std::mutex g_init_mtx;

hipStream_t lazy_stream(hipStream_t (&tab)[HS_MAX_DEV], std::atomic<bool> (&ready)[HS_MAX_DEV], int dev)
{
    if (!ready[dev].load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> g(g_init_mtx);
        if (!ready[dev].load(std::memory_order_relaxed)) {
            if (hipStreamCreateWithFlags(&tab[dev], hipStreamNonBlocking) != hipSuccess) tab[dev] = 0;
            ready[dev].store(true, std::memory_order_release);
        }
    }
    return tab[dev];
}

hipStream_t g_stream[HS_MAX_DEV];
std::atomic<bool> g_stream_init[HS_MAX_DEV];

int set_err(hipError_t e, const char *what)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -2;
}

#define HCHK(call)                                                      \
    do {                                                                \
        hipError_t e_ = (call);                                         \
        if (e_ != hipSuccess) return set_err(e_, #call);                \
    } while (0)

hipStream_t g_stream2[HS_MAX_DEV], g_stream3[HS_MAX_DEV];
std::atomic<bool> g_stream2_init[HS_MAX_DEV], g_stream3_init[HS_MAX_DEV];
thread_local int t_sidx = 0; /* 0: library stream, 1: pipeline / H2D stream, 2: D2H stream, 3: this thread's own */
thread_local hipStream_t t_own[HS_MAX_DEV]; /* per-thread streams (concurrent small fft_exec calls) */
std::atomic<long long> g_own_created{0};       /* per-thread streams created (diagnostics) */

int cur_dev()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= HS_MAX_DEV) dev = 0;
    return dev;
}

hipStream_t primary() { return lazy_stream(g_stream, g_stream_init, cur_dev()); }

/* the stream kernels are launched on: the library stream, or (inside a pipelined chain)
 * the second stream that runs pass B of chunk c while pass A of chunk c+1 runs */
hipStream_t stream()
{
    if (t_sidx == 0) return primary();
    const int dev = cur_dev();
    if (t_sidx == 3) {
        if (!t_own[dev]) { /* (a thread adopts an exited thread's stream first: hsd_thread_adopt) */
            if (hipStreamCreateWithFlags(&t_own[dev], hipStreamNonBlocking) != hipSuccess) t_own[dev] = 0;
            else g_own_created.fetch_add(1, std::memory_order_relaxed);
        }
        return t_own[dev];
    }
    if (t_sidx == 2) return lazy_stream(g_stream3, g_stream3_init, dev);
    return lazy_stream(g_stream2, g_stream2_init, dev);
}

/* event ring (cross-stream ordering) and timing events, per device; used under the
 * device's API lock (hsfft_exec.c), created lazily under g_init_mtx */
#define HS_NEV 64
hipEvent_t g_ev[HS_MAX_DEV][HS_NEV];
std::atomic<bool> g_ev_init[HS_MAX_DEV];

/* ------------------------------------------------------------------ generic pass kernel */
struct KArgs {
    const double2 *in;
    double2 *out;
    const double2 *tw;
    const double *gcs;
    const double2 *laux, *saux;
    long long idist, odist, A, B, nsig, tiles_q, tiles;
    int P, nst, leaf, Wm, Wq, G;
    int sgn, dir, conj, load_op, store_op;
    int radix[HS_MAX_PASS_STAGES];
    int gcs_off[HS_MAX_PASS_STAGES];
};

__device__ __forceinline__ double2 hook_load(const KArgs &a, const double2 *in, long long n)
{
    if (a.load_op == HS_LOAD_CHIRP) {
        if (n >= a.nsig) return make_double2(0.0, 0.0);
        double2 x = in[n], h = a.laux[n];
        if (a.dir == 1) return make_double2(x.x * h.x + x.y * h.y, -x.x * h.y + x.y * h.x);
        return make_double2(x.x * h.x - x.y * h.y, x.x * h.y + x.y * h.x);
    }
    return in[n];
}

__device__ __forceinline__ void hook_store(const KArgs &a, double2 *out, long long n, double2 y)
{
    if (a.store_op == HS_STORE_SPEC) {
        double2 k = a.saux[n];
        if (a.dir == 1) {
            double t = y.x * k.x - y.y * k.y;
            y.y = y.x * k.y + y.y * k.x;
            y.x = t;
        } else {
            double t = y.x * k.x + y.y * k.y;
            y.y = -y.x * k.y + y.y * k.x;
            y.x = t;
        }
        out[n] = y;
    } else if (a.store_op == HS_STORE_CHIRP) {
        if (n >= a.nsig) return;
        double2 h = a.saux[n];
        if (a.dir == 1) out[n] = make_double2(y.x * h.x + y.y * h.y, -y.x * h.y + y.y * h.x);
        else out[n] = make_double2(y.x * h.x - y.y * h.y, y.x * h.y + y.y * h.x);
    } else {
        out[n] = y;
    }
}

template <int R>
__device__ void stage_fixed(const KArgs &a, const double2 *src, double2 *dst, int Lloc, bool leaf,
                            long long m0, long long q0)
{
    const int P = a.P, G = a.G;
    const int S = P / (Lloc * R);
    const int nb = (P / R) * G;
    const long long L = a.B * Lloc;
    for (int bf = threadIdx.x; bf < nb; bf += blockDim.x) {
        const int gi = bf % G, j = bf / G;
        const int kloc = j % Lloc, ml = j / Lloc;
        double xr[R], xi[R];
#pragma unroll
        for (int i = 0; i < R; i++) {
            double2 v = src[((ml + i * S) * Lloc + kloc) * G + gi];
            xr[i] = v.x;
            xi[i] = v.y;
        }
        if (!leaf) {
            const long long q = q0 + gi % a.Wq, m = m0 + gi / a.Wq;
            const long long k = q + a.B * kloc;
            const bool skip = ((R == 4 || R == 5 || R == 7) && k == 0) || q >= a.B || m >= a.A;
            if (!skip) {
                const double2 *w = a.tw + (L - 1 + (long long)(R - 1) * k);
#pragma unroll
                for (int i = 1; i < R; i++) {
                    double2 t = w[i - 1];
                    hsb::twmul(xr[i], xi[i], t.x, a.conj ? -t.y : t.y);
                }
            }
        }
        hsb::bfly<R>(xr, xi, a.sgn, leaf);
#pragma unroll
        for (int jj = 0; jj < R; jj++) dst[(ml * Lloc * R + kloc + jj * Lloc) * G + gi] = make_double2(xr[jj], xi[jj]);
    }
}

__device__ void stage_odd(const KArgs &a, const double2 *src, double2 *dst, int R, int Lloc,
                          const double *cs, long long m0, long long q0)
{
    const int P = a.P, G = a.G;
    const int S = P / (Lloc * R);
    const int nb = (P / R) * G;
    const long long L = a.B * Lloc;
    for (int bf = threadIdx.x; bf < nb; bf += blockDim.x) {
        const int gi = bf % G, j = bf / G;
        const int kloc = j % Lloc, ml = j / Lloc;
        double xr[64], xi[64];
        for (int i = 0; i < R; i++) {
            double2 v = src[((ml + i * S) * Lloc + kloc) * G + gi];
            xr[i] = v.x;
            xi[i] = v.y;
        }
        const long long q = q0 + gi % a.Wq, m = m0 + gi / a.Wq;
        if (q < a.B && m < a.A) { /* odd radices multiply every column, k = 0 included (:1552-1560) */
            const long long k = q + a.B * kloc;
            const double2 *w = a.tw + (L - 1 + (long long)(R - 1) * k);
            for (int i = 1; i < R; i++) {
                double2 t = w[i - 1];
                hsb::twmul(xr[i], xi[i], t.x, a.conj ? -t.y : t.y);
            }
        }
        hsb::bfly_odd(xr, xi, R, a.sgn, cs, cs + (R - 1));
        for (int jj = 0; jj < R; jj++) dst[(ml * Lloc * R + kloc + jj * Lloc) * G + gi] = make_double2(xr[jj], xi[jj]);
    }
}

/* the same stage for a compile-time odd radix R (11..53): fully unrolled, so every value
 * lives in registers (stage_odd's runtime-sized arrays live in scratch memory).  The
 * butterfly is hsb::bfly_odd's arithmetic in the same order (ref :1475-1628): the symmetric
 * sums / differences overwrite the inputs in place, and each output pair is written to the
 * LDS image as soon as it is formed, so no output array is held. */
template <int R>
__device__ void stage_oddT(const KArgs &a, const double2 *src, double2 *dst, int Lloc, const double *cs,
                           long long m0, long long q0)
{
    constexpr int MID = (R - 1) / 2;
    const double *sn = cs + (R - 1);
    const int P = a.P, G = a.G;
    const int S = P / (Lloc * R);
    const int nb = (P / R) * G;
    const long long L = a.B * Lloc;
    const double sg = (double)a.sgn;
    for (int bf = threadIdx.x; bf < nb; bf += blockDim.x) {
        const int gi = bf % G, j = bf / G;
        const int kloc = j % Lloc, ml = j / Lloc;
        double xr[R], xi[R];
#pragma unroll
        for (int i = 0; i < R; i++) {
            double2 v = src[((ml + i * S) * Lloc + kloc) * G + gi];
            xr[i] = v.x;
            xi[i] = v.y;
        }
        const long long q = q0 + gi % a.Wq, m = m0 + gi / a.Wq;
        if (q < a.B && m < a.A) { /* odd radices multiply every column, k = 0 included (:1552-1560) */
            const long long k = q + a.B * kloc;
            const double2 *w = a.tw + (L - 1 + (long long)(R - 1) * k);
#pragma unroll
            for (int i = 1; i < R; i++) {
                double2 t = w[i - 1];
                hsb::twmul(xr[i], xi[i], t.x, a.conj ? -t.y : t.y);
            }
        }
        /* tr[i] -> xr[i+1], tr[i+MID] -> xr[R-1-i] (likewise ti) */
#pragma unroll
        for (int i = 0; i < MID; i++) {
            const double ar = xr[i + 1], br = xr[R - 1 - i], ai = xi[i + 1], bi = xi[R - 1 - i];
            xr[i + 1] = ar + br;
            xi[R - 1 - i] = ai - bi;
            xi[i + 1] = ai + bi;
            xr[R - 1 - i] = ar - br;
        }
        double2 *out = dst + (ml * Lloc * R + kloc) * G + gi;
        {
            double ar = xr[0], ai = xi[0];
#pragma unroll
            for (int i = 0; i < MID; i++) {
                ar += xr[i + 1];
                ai += xi[i + 1];
            }
            out[0] = make_double2(ar, ai);
        }
#pragma unroll
        for (int u = 0; u < MID; u++) {
            double ur = xr[0], ui = xi[0], vr = 0.0, vi = 0.0;
#pragma unroll
            for (int v = 0; v < MID; v++) {
                const int t = ((u + 1) * (v + 1)) % R - 1;
                const double c = cs[t], d = sn[t];
                ur += c * xr[v + 1];
                ui += c * xi[v + 1];
                vr -= d * xr[R - 1 - v];
                vi -= d * xi[R - 1 - v];
            }
            vr = sg * vr;
            vi = sg * vi;
            out[(u + 1) * Lloc * G] = make_double2(ur - vi, ui + vr);
            out[(R - u - 1) * Lloc * G] = make_double2(ur + vi, ui - vr);
        }
    }
}

/* OR: 0 = no odd radix in the pass, > 0 = the pass's only odd radix (compile-time stage,
 * registers sized for that radix), -1 = several odd radices (runtime stage_odd) */
template <int OR, int NT = 256>
__global__ __launch_bounds__(NT) void k_pass_generic(KArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    const long long blk = blockIdx.x;
    const long long b = blk / a.tiles, tile = blk % a.tiles;
    const long long m0 = (tile / a.tiles_q) * a.Wm, q0 = (tile % a.tiles_q) * a.Wq;
    const double2 *in = a.in + b * a.idist;
    double2 *out = a.out + b * a.odist;
    const int P = a.P, G = a.G;
    double2 *src = lds, *dst = lds + P * G;

    for (int e = threadIdx.x; e < P * G; e += blockDim.x) {
        const int gi = e % G, t = e / G;
        const long long m = m0 + gi / a.Wq, q = q0 + gi % a.Wq;
        double2 v = make_double2(0.0, 0.0);
        if (m < a.A && q < a.B) v = hook_load(a, in, ((long long)t * a.A + m) * a.B + q);
        src[t * G + gi] = v;
    }
    __syncthreads();

    int Lloc = 1;
    for (int s = 0; s < a.nst; s++) {
        const int r = a.radix[s];
        const bool leaf = a.leaf && s == 0;
        switch (r) {
        case 2: stage_fixed<2>(a, src, dst, Lloc, leaf, m0, q0); break;
        case 3: stage_fixed<3>(a, src, dst, Lloc, leaf, m0, q0); break;
        case 4: stage_fixed<4>(a, src, dst, Lloc, leaf, m0, q0); break;
        case 5: stage_fixed<5>(a, src, dst, Lloc, leaf, m0, q0); break;
        case 7: stage_fixed<7>(a, src, dst, Lloc, leaf, m0, q0); break;
        case 8: stage_fixed<8>(a, src, dst, Lloc, leaf, m0, q0); break;
        default:
            if constexpr (OR > 0) stage_oddT<OR>(a, src, dst, Lloc, a.gcs + a.gcs_off[s], m0, q0);
            else if constexpr (OR < 0) stage_odd(a, src, dst, r, Lloc, a.gcs + a.gcs_off[s], m0, q0);
            break;
        }
        __syncthreads();
        double2 *t = src;
        src = dst;
        dst = t;
        Lloc *= r;
    }

    for (int e = threadIdx.x; e < P * G; e += blockDim.x) {
        const int qi = e % a.Wq, rest = e / a.Wq;
        const int u = rest % P, mi = rest / P;
        const long long m = m0 + mi, q = q0 + qi;
        if (m < a.A && q < a.B) hook_store(a, out, (m * P + u) * a.B + q, src[u * G + mi * a.Wq + qi]);
    }
}

/* ------------------------------------------------------------------ helpers */
__device__ __forceinline__ double splitmix_u(unsigned long long seed, unsigned long long i)
{
    unsigned long long z = (seed ^ i) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 4503599627370496.0) - 1.0;
}

__global__ void k_fill_complex(double2 *x, long long count, unsigned long long seed, unsigned long long off)
{
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < count; j += (long long)gridDim.x * blockDim.x) {
        unsigned long long e = (unsigned long long)j + off;
        x[j] = make_double2(splitmix_u(seed, 2 * e), splitmix_u(seed, 2 * e + 1));
    }
}

__global__ void k_fill_real(double *x, long long count, unsigned long long seed, unsigned long long off)
{
    for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < count; j += (long long)gridDim.x * blockDim.x)
        x[j] = splitmix_u(seed, (unsigned long long)j + off);
}

/* ref real.c:108-132 */
__global__ void k_r2c_post(const double2 *Z, const double2 *w2, double2 *X, int h, long long zdist, long long xdist)
{
    const int b = blockIdx.y;
    const double2 *z = Z + b * zdist;
    double2 *x = X + b * xdist;
    const int N = 2 * h;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k <= h; k += gridDim.x * blockDim.x) {
        if (k == 0) {
            double2 z0 = z[0];
            x[0] = make_double2(z0.x + z0.y, 0.0);
            x[h] = make_double2(z0.x - z0.y, 0.0);
        } else if (k < h) {
            const double2 a = z[k], c = z[h - k], w = w2[k];
            const double t1 = a.y + c.y, t2 = c.x - a.x;
            const double re = (a.x + c.x + (t1 * w.x) + (t2 * w.y)) / 2.0;
            const double im = (a.y - c.y + (t2 * w.x) - (t1 * w.y)) / 2.0;
            x[k] = make_double2(re, im);
            x[N - k] = make_double2(re, -im);
        }
    }
}

/* same split, one thread per pair (k, h-k): Z is read once (k_r2c_post reads every element
 * twice) and the four mirrored outputs X[k], X[N-k], X[h-k], X[h+k] are written together.
 * Each output is computed by the reference's expression (real.c:112-122), so bit-identical. */
__device__ __forceinline__ double2 r2c_bin(double2 a, double2 c, double2 w)
{
    const double t1 = a.y + c.y, t2 = c.x - a.x;
    return make_double2((a.x + c.x + (t1 * w.x) + (t2 * w.y)) / 2.0, (a.y - c.y + (t2 * w.x) - (t1 * w.y)) / 2.0);
}

template <bool COMPACT>
__global__ void k_r2c_post2(const double2 *Z, const double2 *w2, double2 *X, int h, long long zdist, long long xdist)
{
    const int b = blockIdx.y;
    const double2 *z = Z + b * zdist;
    double2 *x = X + b * xdist;
    const int N = 2 * h, half = h / 2;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k <= half; k += gridDim.x * blockDim.x) {
        if (k == 0) {
            const double2 z0 = z[0];
            x[0] = make_double2(z0.x + z0.y, 0.0);
            x[h] = make_double2(z0.x - z0.y, 0.0);
            continue;
        }
        const double2 a = z[k], c = z[h - k];
        const double2 lo = r2c_bin(a, c, w2[k]);
        x[k] = lo;
        if (!COMPACT) x[N - k] = make_double2(lo.x, -lo.y);
        if (k != h - k) {
            const double2 hi = r2c_bin(c, a, w2[h - k]);
            x[h - k] = hi;
            if (!COMPACT) x[h + k] = make_double2(hi.x, -hi.y);
        }
    }
}

/* ref real.c:169-179 */
__global__ void k_c2r_pre(const double2 *X, const double2 *w2, double2 *Zi, int h, long long xdist, long long zdist)
{
    const int b = blockIdx.y;
    const double2 *x = X + b * xdist;
    double2 *z = Zi + b * zdist;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < h; k += gridDim.x * blockDim.x) {
        const double2 a = x[k], c = x[h - k], w = w2[k];
        const double t1 = -a.y - c.y, t2 = -c.x + a.x;
        z[k] = make_double2(a.x + c.x + (t1 * w.x) - (t2 * w.y), a.y - c.y + (t2 * w.x) + (t1 * w.y));
    }
}

/* convolve.c:147-151's spectral product feeding real.c:169-179's inverse pre-twiddle in one
 * pass: z[k] from (A.B)[k] and (A.B)[h-k]; each product is formed with k_cmul's expression
 * (a pair's partner product is recomputed, same bits), so the c2r input is bit-identical */
__device__ __forceinline__ double2 cmul1(double2 a, double2 c)
{
    return make_double2(a.x * c.x - a.y * c.y, a.x * c.y + a.y * c.x);
}

__global__ void k_c2r_pre_mul(const double2 *A, const double2 *Bv, const double2 *w2, double2 *Zi, int h,
                              long long xdist, long long zdist)
{
    const int b = blockIdx.y;
    const double2 *x = A + b * xdist, *y = Bv + b * xdist;
    double2 *z = Zi + b * zdist;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < h; k += gridDim.x * blockDim.x) {
        const double2 a = cmul1(x[k], y[k]), c = cmul1(x[h - k], y[h - k]), w = w2[k];
        const double t1 = -a.y - c.y, t2 = -c.x + a.x;
        z[k] = make_double2(a.x + c.x + (t1 * w.x) - (t2 * w.y), a.y - c.y + (t2 * w.x) + (t1 * w.y));
    }
}

/* convolve.c:157-160 then :163-201: dst[b][i] = src[b][soff + i] / divisor, i < n */
__global__ void k_copy_rows_div(const double *src, long long sdist, long long soff, double *dst, long long ddist,
                                long long n, double divisor)
{
    const long long b = blockIdx.y;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[b * ddist + i] = src[b * sdist + soff + i] / divisor;
}

/* ref convolve.c:147-151 */
__global__ void k_cmul(const double2 *A, const double2 *Bv, double2 *C, long long n, long long dist)
{
    const long long b = blockIdx.y;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const double2 a = A[b * dist + i], c = Bv[b * dist + i];
        C[b * dist + i] = make_double2(a.x * c.x - a.y * c.y, a.x * c.y + a.y * c.x);
    }
}

/* ref convolve.c:157-160 */
__global__ void k_scale_real(double *x, long long n, long long dist, double divisor)
{
    const long long b = blockIdx.y;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        x[b * dist + i] /= divisor;
}

/* row copy with zero fill: dst[b][i] = i < ncopy ? src[b][soff + i] : 0 for i < dlen
 * (zero padding of convolve.c:117-140 and the output slice of :163-201) */
__global__ void k_copy_rows(const double *src, long long sdist, long long soff, long long ncopy, double *dst,
                            long long ddist, long long dlen)
{
    const long long b = blockIdx.y;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < dlen; i += (long long)gridDim.x * blockDim.x)
        dst[b * ddist + i] = i < ncopy ? src[b * sdist + soff + i] : 0.0;
}

/* stream copy (practical HBM ceiling for the bench report) */
__global__ void k_copy16(const double2 *__restrict__ a, double2 *__restrict__ b, long long n)
{
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        b[i] = a[i];
}

/* copy variants for the HBM access-pattern study (tools/membench.py) */
typedef double v2d __attribute__((ext_vector_type(2)));
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copyU(const v2d *__restrict__ a, v2d *__restrict__ b, long long n)
{
    const long long stride = (long long)gridDim.x * blockDim.x * U;
    for (long long base = blockIdx.x * (long long)blockDim.x * U + threadIdx.x; base < n; base += stride) {
        v2d v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long i = base + (long long)u * blockDim.x;
            if (i < n) v[u] = NT ? __builtin_nontemporal_load(&a[i]) : a[i];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const long long i = base + (long long)u * blockDim.x;
            if (i < n) {
                if (NT) __builtin_nontemporal_store(v[u], &b[i]);
                else b[i] = v[u];
            }
        }
    }
}

/* differing 8-byte words (whole-buffer comparisons between schedules): one 64-bit
 * agent-scope atomic add per workgroup after a wave / workgroup reduction */
__global__ __launch_bounds__(256) void k_count_diff(const unsigned long long *__restrict__ a,
                                                    const unsigned long long *__restrict__ b, long long n,
                                                    unsigned long long *cnt)
{
    __shared__ unsigned long long part[4];
    unsigned long long c = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        c += a[i] != b[i];
    for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(cnt, t);
    }
}

hipEvent_t g_t0[HS_MAX_DEV], g_t1[HS_MAX_DEV];
hipEvent_t g_pev[HS_MAX_DEV][2 * HS_MAX_PASSES];
std::atomic<bool> g_timer_init[HS_MAX_DEV];

/* creates the per-device timing events once; false on failure */
bool timer_events(int dev)
{
    if (g_timer_init[dev].load(std::memory_order_acquire)) return true;
    std::lock_guard<std::mutex> g(g_init_mtx);
    if (g_timer_init[dev].load(std::memory_order_relaxed)) return true;
    if (hipEventCreate(&g_t0[dev]) != hipSuccess || hipEventCreate(&g_t1[dev]) != hipSuccess) return false;
    for (int k = 0; k < 2 * HS_MAX_PASSES; k++)
        if (hipEventCreate(&g_pev[dev][k]) != hipSuccess) return false;
    g_timer_init[dev].store(true, std::memory_order_release);
    return true;
}

int grid_for(long long n, int threads)
{
    long long g = (n + threads - 1) / threads;
    if (g > 65535) g = 65535;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

#include "hsfft_pass_r8.h"
#include "hsfft_pass_pf.h"
#include "hsfft_pass_mr.h"
#include "hsfft_blue_pf.h"
#include "hsfft_blue_xcd.h"

extern "C" {

int hsd_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int hsd_set_device(int dev)
{
    HCHK(hipSetDevice(dev));
    (void)stream();
    return 0;
}

int hsd_get_device(void)
{
    int d = -1;
    if (hipGetDevice(&d) != hipSuccess) return -1;
    return d;
}

void *hsd_malloc(size_t bytes)
{
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        set_err(e, "hipMalloc");
        return nullptr;
    }
    return p;
}

int hsd_free(void *p)
{
    if (p) HCHK(hipFree(p));
    return 0;
}

int hsd_h2d(void *d, const void *h, size_t bytes)
{
    HCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream()));
    HCHK(hipStreamSynchronize(stream()));
    return 0;
}

int hsd_d2h(void *h, const void *d, size_t bytes)
{
    HCHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream()));
    HCHK(hipStreamSynchronize(stream()));
    return 0;
}

int hsd_d2d_async(void *d, const void *s, size_t bytes)
{
    HCHK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, stream()));
    return 0;
}

int hsd_memset_async(void *d, int v, size_t bytes)
{
    HCHK(hipMemsetAsync(d, v, bytes, stream()));
    return 0;
}

/* persistent-launch state per device (bxc::k_bxcd): a counter block (2 counters per group, each
 * on its own 128-B line), zeroed on the launch's stream before every launch */
static unsigned *g_pl_ctr[HS_MAX_DEV];
static size_t g_pl_bytes[HS_MAX_DEV];

/* Error words of the persistent launches, per THREAD and device: a device block whose word 0
 * (the asynchronous sticky word) and word 32 (the synchronous call's word) a launch sets when one
 * of its in-launch waits timed out, and a page-locked host copy of both, refreshed on the
 * launch's stream behind every launch.  The asynchronous word is cumulative: it is read and
 * cleared only by hsd_sync_report() of the thread that launched (hsfft_synchronize, the timing
 * calls), so no other synchronisation -- a scratch pool growing, a device state being built, an
 * unrelated plan's call, another thread -- can consume or inherit it.  The synchronous word is
 * cleared before every synchronous launch and read right after it (hsd_blue_xcd returns 2).
 * The deferred word (16) is the host pipeline's (hsfft_exec_batched_host): cumulative over the
 * pipeline's launches, read and cleared once after its final stream wait (hsd_blue_deferred_take).
 * Words adopted from an exited thread (hsd_thread_adopt) are `inherited`: whatever that thread's
 * asynchronous or deferred launches left in words 0 / 16 is discarded, never reported to the new
 * owner -- on the library stream, behind those launches, before the new owner's first launch
 * (pl_words), or at its first report (pl_report, after the stream was waited for; a deferred
 * word is also discarded at the start of every host pipeline). */
struct PlErr {
    unsigned *dev;  /* 64 words on the device: [0] async sticky, [16] deferred, [32] sync */
    unsigned *host; /* 64 page-locked words: copies of the same */
    bool inherited;
};
static thread_local PlErr t_pl[HS_MAX_DEV];

static int pl_words(int dev, PlErr **out)
{
    PlErr *p = &t_pl[dev];
    if (p->dev && p->inherited) {
        /* the exited owner's asynchronous / deferred launches ran on the library stream: clear
         * words 0..31 (async 0, deferred 16) and their host copies behind them */
        HCHK(hipMemsetAsync(p->dev, 0, 32 * sizeof(unsigned), primary()));
        HCHK(hipMemcpyAsync(p->host, p->dev, 32 * sizeof(unsigned), hipMemcpyDeviceToHost, primary()));
        p->inherited = false;
    }
    if (!p->dev) {
        HCHK(hipMalloc((void **)&p->dev, 64 * sizeof(unsigned)));
        if (hipMemset(p->dev, 0, 64 * sizeof(unsigned)) != hipSuccess ||
            hipHostMalloc((void **)&p->host, 64 * sizeof(unsigned), hipHostMallocDefault) != hipSuccess) {
            const hipError_t e = hipGetLastError();
            (void)hipFree(p->dev);
            p->dev = nullptr;
            return set_err(e, "persistent-launch error words");
        }
        memset(p->host, 0, 64 * sizeof(unsigned));
    }
    *out = p;
    return 0;
}

static void pl_release_thread(int dev)
{
    PlErr *p = &t_pl[dev];
    if (p->dev) (void)hipFree(p->dev);
    if (p->host) (void)hipHostFree(p->host);
    p->dev = nullptr;
    p->host = nullptr;
    p->inherited = false;
}

/* Report (once) a timed-out wait of this thread's asynchronous persistent launches on the
 * current device.  Called after the library stream was synchronised, so the host copy is
 * final. */
static int pl_report(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= HS_MAX_DEV) return 0;
    PlErr *p = &t_pl[dev];
    if (!p->host || *(volatile unsigned *)p->host == 0) {
        p->inherited = false; /* (an inherited word 0 was clear: nothing to discard) */
        return 0;
    }
    const unsigned w = *(volatile unsigned *)p->host;
    *(volatile unsigned *)p->host = 0;
    (void)hipMemsetAsync(p->dev, 0, sizeof(unsigned), primary());
    (void)hipStreamSynchronize(primary());
    if (p->inherited) { /* the exited owner's error: discarded, not this thread's */
        p->inherited = false;
        return 0;
    }
    snprintf(g_err, sizeof g_err,
             "persistent Bluestein launch: an in-launch dependency wait timed out (error word %u); the outputs of this "
             "thread's Bluestein calls since its last hsfft_synchronize() on this device are invalid "
             "(HSFFT_BX_SYNC=1 re-runs such rows automatically)", w);
    return -2;
}

int hsd_blue_deferred_take(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= HS_MAX_DEV) return 0;
    PlErr *p = &t_pl[dev];
    if (!p->host || *(volatile unsigned *)(p->host + 16) == 0) return 0;
    *(volatile unsigned *)(p->host + 16) = 0;
    (void)hipMemsetAsync(p->dev + 16, 0, sizeof(unsigned), primary());
    (void)hipStreamSynchronize(primary());
    return 1;
}

/* wait for the library stream; a pending persistent-launch error stays pending */
int hsd_sync(void)
{
    HCHK(hipStreamSynchronize(primary()));
    return 0;
}

/* the same, and report this thread's pending persistent-launch error (hsfft_synchronize) */
int hsd_sync_report(void)
{
    HCHK(hipStreamSynchronize(primary()));
    return pl_report();
}

/* Bluestein M = 2^18 as one persistent launch (hsfft_blue_xcd.h).  img: ng x 4 x M points of
 * scratch.  Every workgroup must be resident at once: the occupancy API is asked on the host
 * and a grid that does not fit is refused (returned as 3: the caller runs the three-launch
 * path at once); inside the launch a per-group arrival census proves it (in a synchronous or
 * deferred call a group the API over-promised fails in ~2 ms, as a timed-out launch).  (Round
 * 4's cooperative-launch form crashed profiled processes at exit; removed
 * in round 6.)  HSFFT_BX_UNCHECKED=1 (tests only) skips the host check, so that the census has
 * to catch an oversized grid.
 * Asynchronous (sync == 0): the launch is queued on the library stream with a copy of this
 * thread's sticky error word behind it; a wait that still timed out (the last-resort bound,
 * ~1.3 s without progress; HSFFT_BX_TLIMIT ticks of the 100 MHz counter for tests) is reported
 * by this thread's next hsd_sync_report().  Synchronous (sync == 1): the call waits, and a
 * timed-out launch returns 2 so the caller re-runs its rows on the three-launch path.  Deferred
 * (sync == 2): queued like an asynchronous launch, its outcome in the deferred word, which the
 * caller reads with hsd_blue_deferred_take() after its own final stream wait.
 * Returns 0 on success (queued), 1 if not applicable, 2 (sync) if an in-launch wait timed out,
 * 3 if the grid cannot be co-resident, < 0 on a HIP error. */
int hsd_blue_xcd(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                 const void *hk, void *img, size_t img_bytes, long long nsig, int batch, int sgn, int ng, int sync)
{
    int dev = 0;
    HCHK(hipGetDevice(&dev));
    if (dev < 0 || dev >= HS_MAX_DEV) return -1;
    if (batch < 1 || (sgn != 1 && sgn != -1) || ng < 1 || ng > 64 || nsig < 1 || nsig > (long long)bxc::IMG ||
        img_bytes < (size_t)ng * bxc::NIMG * bxc::IMG * sizeof(double2))
        return 1;
    void (*fn)(bxc::XArgs) = sgn == 1 ? bxc::k_bxcd<1> : bxc::k_bxcd<-1>;
    HCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bxc::LDS_BYTES));
    const int grid = ng * (int)bxc::NTILE;
    const char *ue = getenv("HSFFT_BX_UNCHECKED");
    if (!(ue && atoi(ue))) { /* co-residency: workgroups per CU the occupancy API allows x CUs */
        int per_cu = 0, ncu = 0;
        HCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)fn, 512, bxc::LDS_BYTES));
        HCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        if ((long long)per_cu * ncu < grid) {
            snprintf(g_err, sizeof g_err, "hsd_blue_xcd: %d workgroups cannot be co-resident (%d per CU x %d CUs)", grid,
                     per_cu, ncu);
            return 3;
        }
    }
    PlErr *pe = nullptr;
    {
        const int rc = pl_words(dev, &pe);
        if (rc) return rc;
    }
    const size_t CS = bxc::CS;
    const size_t need = 3 * CS * (size_t)ng * sizeof(unsigned); /* hand-off counters + census per group */
    if (g_pl_bytes[dev] < need) {
        if (g_pl_ctr[dev]) {
            HCHK(hipStreamSynchronize(stream())); /* an earlier launch may still use the block */
            HCHK(hipFree(g_pl_ctr[dev]));
            g_pl_ctr[dev] = nullptr;
            g_pl_bytes[dev] = 0;
        }
        const size_t alloc = (need + 4095) & ~(size_t)4095;
        HCHK(hipMalloc((void **)&g_pl_ctr[dev], alloc));
        g_pl_bytes[dev] = alloc;
    }
    unsigned *ctr = g_pl_ctr[dev];
    /* the counters are zeroed before every launch (Guideline 16, re-initialise every call) */
    HCHK(hipMemsetAsync(ctr, 0, need, stream()));
    /* word: [0] asynchronous (sticky, hsd_sync_report), [16] deferred (cumulative until
     * hsd_blue_deferred_take), [32] synchronous (cleared per launch) */
    const int wi = sync == 1 ? 32 : sync == 2 ? 16 : 0;
    unsigned *err = pe->dev + wi;
    if (sync == 1) HCHK(hipMemsetAsync(err, 0, sizeof(unsigned), stream()));
    bxc::XArgs a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)in;
    a.out = (double2 *)out;
    a.tw = (const double2 *)tw;
    a.chirp = (const double2 *)chirp;
    a.hk = (const double2 *)hk;
    a.img = (double2 *)img;
    a.idist = idist;
    a.odist = odist;
    a.cnt = ctr;
    a.err = err;
    a.batch = (unsigned)batch;
    a.ng = (unsigned)ng;
    a.nsig = (unsigned)nsig;
    a.tlimit = bxc::T_LIMIT;
    a.climit = sync ? bxc::C_LIMIT : bxc::T_LIMIT; /* fail fast only where the caller re-runs the rows (1, 2) */
    {
        /* polls of the hand-off counters 4 x s_sleep 2 apart (was 1): in-process A/B on two boxes
         * 32.51 vs 32.61 and 32.13 vs 32.29 ms per 8192 rows (profiles/r05e_*, r05g_*) */
        const char *e = getenv("HSFFT_BX_SLEEP");
        a.sleep = e ? (unsigned)atoi(e) : 4u;
        e = getenv("HSFFT_BX_MAP");
        a.xmap = e ? (unsigned)atoi(e) & 1u : 1u;
        e = getenv("HSFFT_BX_JITTER"); /* uneven-load tests: per-phase delays, results unchanged */
        a.jitter = e ? (unsigned)atoi(e) : 0u;
        e = getenv("HSFFT_BX_TLIMIT"); /* tests: force the timeout path (ticks of 10 ns) */
        if (e && atoll(e) > 0) a.tlimit = (unsigned long long)atoll(e);
        e = getenv("HSFFT_BX_CLIMIT"); /* tests: the census bound (ticks of 10 ns) */
        if (e && atoll(e) > 0) a.climit = (unsigned long long)atoll(e);
    }
    static unsigned *s_dbg[HS_MAX_DEV];
    const char *dbgenv = getenv("HSFFT_BX_DEBUG");
    const bool dbg = dbgenv && atoi(dbgenv) && grid <= 4096;
    if (dbg) {
        if (!s_dbg[dev]) HCHK(hipMalloc((void **)&s_dbg[dev], 4096 * 8 * sizeof(unsigned)));
        HCHK(hipMemsetAsync(s_dbg[dev], 0, (size_t)grid * 8 * sizeof(unsigned), stream()));
        a.dbg = s_dbg[dev]; /* the call waits for the trace (its error word keeps its own contract) */
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(512), bxc::LDS_BYTES, stream(), a);
    HCHK(hipGetLastError());
    /* host copy of the word this launch could set (async / deferred: cumulative words) */
    unsigned *hw = pe->host + wi;
    HCHK(hipMemcpyAsync(hw, err, sizeof(unsigned), hipMemcpyDeviceToHost, stream()));
    if (sync != 1 && !dbg) return 0;
    HCHK(hipStreamSynchronize(stream()));
    const unsigned w = *(volatile unsigned *)hw;
    if (dbg) { /* mean us per row: P1, wait A, P2, wait B, P3 */
        static unsigned h[4096 * 8];
        HCHK(hipMemcpy(h, s_dbg[dev], (size_t)grid * 8 * sizeof(unsigned), hipMemcpyDeviceToHost));
        double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int wg = 0; wg < grid; wg++)
            for (int i = 0; i < 8; i++) t[i] += h[wg * 8 + i];
        const double rows = t[0] > 0 ? t[0] : 1;
        fprintf(stderr,
                "bxcd: wgs %d rows/wg %.1f  us per row: P1 %.2f (+drain %.2f) waitA %.2f P2 %.2f (+drain %.2f) waitB %.2f "
                "P3 %.2f\n",
                grid, t[0] / grid, t[1] / rows / 100.0, t[6] / rows / 100.0, t[2] / rows / 100.0, t[3] / rows / 100.0,
                t[7] / rows / 100.0, t[4] / rows / 100.0, t[5] / rows / 100.0);
    }
    if (sync == 1 && w) { /* the caller re-runs the rows */
        *(volatile unsigned *)hw = 0;
        snprintf(g_err, sizeof g_err, "hsd_blue_xcd: an in-launch wait timed out (error word %u)", w);
        return 2;
    }
    return 0;
}

/* differing 8-byte words; the counter is one per-device word kept for the process */
static unsigned long long *g_diff_word[HS_MAX_DEV];

int hsd_count_diff(const void *a, const void *b, long long nwords, unsigned long long *count)
{
    const int dev = cur_dev();
    if (!g_diff_word[dev]) HCHK(hipMalloc((void **)&g_diff_word[dev], sizeof(unsigned long long)));
    unsigned long long *d = g_diff_word[dev];
    HCHK(hipMemsetAsync(d, 0, sizeof *d, stream()));
    if (nwords > 0)
        hipLaunchKernelGGL(k_count_diff, dim3(8192), dim3(256), 0, stream(), (const unsigned long long *)a,
                           (const unsigned long long *)b, nwords, d);
    HCHK(hipGetLastError());
    HCHK(hipMemcpyAsync(count, d, sizeof *d, hipMemcpyDeviceToHost, stream()));
    HCHK(hipStreamSynchronize(stream()));
    return 0;
}

int hsd_cu_count(void)
{
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return n;
}

/* Pool of per-thread sets (hsfft_internal.h, hsd_tset): parked by exiting threads, adopted by
 * new ones, destroyed only by hsd_pool_drain.  Parking and adopting are host bookkeeping under a
 * mutex -- no HIP call (round 5's reaping synchronised and freed dead threads' objects on a new
 * thread's first call: +52 % per threaded small call). */
namespace {
struct TSet {
    hipStream_t own;
    PlErr pl;
    hsd_tset h;
};
std::mutex g_pool_mtx;
std::vector<TSet> g_pool[HS_MAX_DEV];
}  // namespace

long long hsd_thread_streams_created(void) { return g_own_created.load(std::memory_order_relaxed); }

void hsd_thread_park(int dev, const hsd_tset *h)
{
    if (dev < 0 || dev >= HS_MAX_DEV) return;
    TSet s;
    s.own = t_own[dev];
    s.pl = t_pl[dev];
    s.h = h ? *h : hsd_tset{{nullptr, nullptr}, 0, nullptr, 0};
    t_own[dev] = 0;
    t_pl[dev] = PlErr{nullptr, nullptr, false};
    if (!s.own && !s.pl.dev && !s.h.pin[0] && !s.h.pin[1] && !s.h.flag) return;
    std::lock_guard<std::mutex> g(g_pool_mtx);
    g_pool[dev].push_back(s);
}

int hsd_thread_adopt(int dev, hsd_tset *h)
{
    if (dev < 0 || dev >= HS_MAX_DEV || t_own[dev] || t_pl[dev].dev) return 0;
    TSet s;
    {
        std::lock_guard<std::mutex> g(g_pool_mtx);
        if (g_pool[dev].empty()) return 0;
        s = g_pool[dev].back();
        g_pool[dev].pop_back();
    }
    t_own[dev] = s.own; /* the stream's earlier work was waited for by its call */
    t_pl[dev] = s.pl;
    t_pl[dev].inherited = s.pl.dev != nullptr;
    if (h) *h = s.h;
    return 1;
}

int hsd_pool_drain(void)
{
    std::vector<TSet> sets[HS_MAX_DEV];
    {
        std::lock_guard<std::mutex> g(g_pool_mtx);
        for (int d = 0; d < HS_MAX_DEV; d++) sets[d].swap(g_pool[d]);
    }
    int cur = -1, n = 0;
    (void)hipGetDevice(&cur);
    for (int d = 0; d < HS_MAX_DEV; d++) {
        if (sets[d].empty()) continue;
        (void)hipSetDevice(d);
        for (const TSet &s : sets[d]) { /* the stream first: its work may use the rest */
            if (s.own) {
                (void)hipStreamSynchronize(s.own);
                (void)hipStreamDestroy(s.own);
            }
            if (s.pl.dev) (void)hipFree(s.pl.dev);
            if (s.pl.host) (void)hipHostFree(s.pl.host);
            for (void *p : {s.h.pin[0], s.h.pin[1], (void *)s.h.flag})
                if (p) (void)hipHostFree(p);
            n++;
        }
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    (void)hipGetLastError();
    return n;
}

/* Releases every device object this layer holds on the current device (after waiting for its
 * streams): the persistent-launch counters, the calling thread's error words (a pending error
 * is reported first, as hsd_sync_report would), the diff counter, the debug trace block, the
 * timing and ordering events, the library's streams and the calling thread's own stream.  All
 * of them are re-created on demand.  Returns the pending error or the first HIP error. */
int hsd_finalize_device(void)
{
    const int dev = cur_dev();
    int rc = 0;
    hipStream_t *tabs[3] = {g_stream, g_stream2, g_stream3};
    std::atomic<bool> *flags[3] = {g_stream_init, g_stream2_init, g_stream3_init};
    for (int s = 0; s < 3; s++)
        if (flags[s][dev].load(std::memory_order_acquire) && tabs[s][dev] &&
            hipStreamSynchronize(tabs[s][dev]) != hipSuccess && !rc)
            rc = set_err(hipGetLastError(), "hipStreamSynchronize");
    if (!rc) rc = pl_report();
    pl_release_thread(dev);
    if (t_own[dev]) {
        (void)hipStreamSynchronize(t_own[dev]);
        (void)hipStreamDestroy(t_own[dev]);
        t_own[dev] = 0;
    }
    std::lock_guard<std::mutex> g(g_init_mtx);
    if (g_pl_ctr[dev]) (void)hipFree(g_pl_ctr[dev]);
    g_pl_ctr[dev] = nullptr;
    g_pl_bytes[dev] = 0;
    if (g_diff_word[dev]) (void)hipFree(g_diff_word[dev]);
    g_diff_word[dev] = nullptr;
    if (g_ev_init[dev].load(std::memory_order_acquire)) {
        for (int k = 0; k < HS_NEV; k++) (void)hipEventDestroy(g_ev[dev][k]);
        g_ev_init[dev].store(false, std::memory_order_release);
    }
    if (g_timer_init[dev].load(std::memory_order_acquire)) {
        (void)hipEventDestroy(g_t0[dev]);
        (void)hipEventDestroy(g_t1[dev]);
        for (int k = 0; k < 2 * HS_MAX_PASSES; k++) (void)hipEventDestroy(g_pev[dev][k]);
        g_timer_init[dev].store(false, std::memory_order_release);
    }
    for (int s = 0; s < 3; s++)
        if (flags[s][dev].load(std::memory_order_acquire)) {
            if (tabs[s][dev]) (void)hipStreamDestroy(tabs[s][dev]);
            tabs[s][dev] = 0;
            flags[s][dev].store(false, std::memory_order_release);
        }
    (void)hipGetLastError();
    return rc;
}

int hsd_select_stream(int idx)
{
    t_sidx = idx < 0 || idx > 3 ? 0 : idx;
    return 0;
}

int hsd_stream_index(void) { return t_sidx; }

int hsd_h2d_async(void *d, const void *h, size_t bytes)
{
    HCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream()));
    return 0;
}

int hsd_d2h_async(void *h, const void *d, size_t bytes)
{
    HCHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream()));
    return 0;
}

int hsd_stream_sync(void)
{
    HCHK(hipStreamSynchronize(stream()));
    return 0;
}

/* Completion without the stream wait (small host-buffer calls, BASELINE config 1): the command
 * processor writes `v` into the page-locked word `flag` once every earlier operation of the
 * selected stream has completed (hipStreamWriteValue32: a queue packet, no kernel dispatch);
 * the host polls the word.  Measured floor for a 16 KB zero-copy kernel: 12.6 vs 15.5 us
 * with hipStreamSynchronize (tools/experiments/c1_latency.hip).  Falls back to the stream wait
 * after ~2 s without the value (a faulted queue never writes it; the wait then reports the
 * error). */
/* wait for a kernel of the selected stream to store v into the host word (hsd_launch.done),
 * stream wait as the fallback after ~2 s (a faulted kernel never stores it) */
static double wall_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int hsd_host_word_wait(unsigned *flag, unsigned v)
{
    const double t0 = wall_s();
    for (unsigned long n = 0;; n++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return 0;
        if ((n & 0xFFFF) == 0xFFFF && wall_s() - t0 > 2.0) break;
    }
    HCHK(hipStreamSynchronize(stream()));
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) return set_err(hipErrorUnknown, "kernel completion word");
    return 0;
}

int hsd_stream_signal_wait(unsigned *flag, unsigned v)
{
    HCHK(hipStreamWriteValue32(stream(), flag, v, 0));
    const double t0 = wall_s();
    for (unsigned long n = 0;; n++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return 0;
        if ((n & 0xFFFF) == 0xFFFF && wall_s() - t0 > 2.0) break;
    }
    HCHK(hipStreamSynchronize(stream()));
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) return set_err(hipErrorUnknown, "stream completion word");
    return 0;
}

/* page-lock caller memory for asynchronous copies; 1 if this call registered it */
int hsd_host_register(void *p, size_t bytes)
{
    if (hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess) return 1;
    (void)hipGetLastError(); /* already pinned (hipHostMalloc'd / registered) or not pinnable */
    return 0;
}

/* page-locked host memory that kernels can read and write directly over the host link
 * (the small-transform path of fft_exec) */
void *hsd_host_alloc(size_t bytes)
{
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault);
    if (e != hipSuccess) {
        set_err(e, "hipHostMalloc");
        return nullptr;
    }
    return p;
}

int hsd_host_free(void *p)
{
    if (p) HCHK(hipHostFree(p));
    return 0;
}

int hsd_host_unregister(void *p)
{
    HCHK(hipHostUnregister(p));
    return 0;
}

/* event ring for cross-stream ordering: record slot i on the current stream / make the
 * current stream wait for slot i's most recent record */
int hsd_event_record(int i)
{
    int dev = hsd_get_device();
    if (dev < 0 || dev >= HS_MAX_DEV) return -1;
    if (!g_ev_init[dev].load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> g(g_init_mtx);
        if (!g_ev_init[dev].load(std::memory_order_relaxed)) {
            for (int k = 0; k < HS_NEV; k++) HCHK(hipEventCreateWithFlags(&g_ev[dev][k], hipEventDisableTiming));
            g_ev_init[dev].store(true, std::memory_order_release);
        }
    }
    HCHK(hipEventRecord(g_ev[dev][i % HS_NEV], stream()));
    return 0;
}

int hsd_event_wait(int i)
{
    int dev = hsd_get_device();
    if (dev < 0 || dev >= HS_MAX_DEV || !g_ev_init[dev].load(std::memory_order_acquire)) return -1;
    HCHK(hipStreamWaitEvent(stream(), g_ev[dev][i % HS_NEV], 0));
    return 0;
}

void *hsd_stream(void) { return (void *)primary(); }

int hsd_is_device_ptr(const void *p)
{
    hipPointerAttribute_t at;
    memset(&at, 0, sizeof at);
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

const char *hsd_errstr(void) { return g_err; }

int hsd_run_pass(const hsd_pass *p, const hsd_launch *l)
{
    if (p->variant == HS_KV_R8X3) {
        const int rc = pf::launch(p, l, stream());
        if (rc <= 0) return rc;
        return r8::launch(p, l, stream());
    }
    if (p->variant == HS_KV_MR && l->load_op == HS_LOAD_PLAIN && l->store_op == HS_STORE_PLAIN)
        return mr::launch(p, l, stream());
    KArgs a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)l->in;
    a.out = (double2 *)l->out;
    a.tw = (const double2 *)l->tw;
    a.gcs = l->gcs;
    a.laux = (const double2 *)l->load_aux;
    a.saux = (const double2 *)l->store_aux;
    a.idist = l->idist;
    a.odist = l->odist;
    a.A = p->A;
    a.B = p->B;
    a.nsig = l->nsig;
    a.P = p->P;
    a.nst = p->nst;
    a.leaf = p->leaf;
    a.Wm = p->Wm;
    a.Wq = p->Wq;
    a.G = p->G;
    a.sgn = l->sgn;
    a.dir = l->dir;
    a.conj = l->conj;
    a.load_op = l->load_op;
    a.store_op = l->store_op;
    for (int s = 0; s < p->nst; s++) {
        a.radix[s] = p->radix[s];
        a.gcs_off[s] = p->gcs_off[s];
    }
    long long tm = (p->A + p->Wm - 1) / p->Wm, tq = (p->B + p->Wq - 1) / p->Wq;
    a.tiles_q = tq;
    a.tiles = tm * tq;
    long long grid = a.tiles * l->batch;
    size_t lds = 2 * (size_t)p->P * p->G * sizeof(double2);
    if (grid <= 0 || grid > 0x7fffffffLL || lds > 160 * 1024) {
        snprintf(g_err, sizeof g_err, "hsd_run_pass: bad launch geometry (grid %lld, lds %zu)", grid, lds);
        return -1;
    }
    int oddr = 0; /* the pass's odd radix (>= 11), -1 if it has two different ones */
    for (int s = 0; s < p->nst; s++) {
        const int r = p->radix[s];
        if (r == 2 || r == 3 || r == 4 || r == 5 || r == 7 || r == 8) continue;
        oddr = oddr == 0 || oddr == r ? r : -1;
    }
    if (getenv("HSFFT_ODD_RUNTIME") && oddr > 0) oddr = -1; /* dev: the runtime-radix stage */
    typedef void (*gfn)(KArgs);
    gfn fn;
    switch (oddr) { /* every odd radix the reference planner produces (factors(): 11..53) */
    case 0: fn = k_pass_generic<0>; break;
    case 11: fn = k_pass_generic<11>; break;
    case 13: fn = k_pass_generic<13>; break;
    case 17: fn = k_pass_generic<17>; break;
    case 19: fn = k_pass_generic<19>; break;
    case 23: fn = k_pass_generic<23>; break;
    case 29: fn = k_pass_generic<29>; break;
    case 31: fn = k_pass_generic<31>; break;
    case 37: fn = k_pass_generic<37>; break;
    case 41: fn = k_pass_generic<41>; break;
    case 43: fn = k_pass_generic<43>; break;
    case 47: fn = k_pass_generic<47>; break;
    case 53: fn = k_pass_generic<53>; break;
    default: fn = k_pass_generic<-1>; break;
    }
    /* whole rows of >= 1536 points (up to 5120): 1024 threads instead of 256 -- at 48-160 KiB
     * of LDS a CU holds 1-3 workgroups, so 256 threads left it with 4-12 waves (measured: 3000
     * 33.6 -> 56.0, 5000 36.5 -> 64.4, 17^3 31.2 -> 50.7 GSamples/s; the first pass of 100000
     * (P = 500, 4 columns) 32.6 -> 26.4, so passes of a multi-pass schedule keep 256;
     * HSFFT_GNT=256 everywhere) */
    int nt = 256;
    {
        const char *e = getenv("HSFFT_GNT");
        const int want = e ? atoi(e) : 1024;
        if (want >= 1024 && (long long)p->P * p->G >= 1536 && p->A == 1 && p->B == 1) {
            nt = 1024;
            switch (oddr) { /* the variants whose registers fit 1024 threads (<= 128 VGPRs) */
            case 0: fn = k_pass_generic<0, 1024>; break;
            case 11: fn = k_pass_generic<11, 1024>; break;
            case 13: fn = k_pass_generic<13, 1024>; break;
            case 17: fn = k_pass_generic<17, 1024>; break;
            default: nt = 256; break;
            }
        }
    }
    if (lds > 65536) HCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(nt), lds, stream(), a);
    HCHK(hipGetLastError());
    return 0;
}

int r8_has_variant(int r0, int n8, int G, int Wq, int first) { return r8::find(r0, n8, G, Wq, first != 0) != nullptr; }

int hsd_blue_mid(const void *in, void *out, long long dist, const void *tw, const void *hk, int batch, int sgn,
                 int conj, int dir, int sgn2, int conj2)
{
    if (conj == 0 && dir == sgn && sgn2 == -sgn && conj2 == 1) {
        const int rc = bpf::launch(0, in, dist, out, dist, tw, hk, 0, batch, sgn, stream());
        if (rc <= 0) return rc;
    }
    return r8::launch_blue_mid(in, out, dist, tw, hk, batch, sgn, conj, dir, sgn2, conj2, stream());
}

int hsd_blue_last(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                  long long nsig, int batch, int dir)
{
    return bpf::launch(1, in, idist, out, odist, tw, chirp, nsig, batch, dir, stream());
}

int hsd_blue_first(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                   long long nsig, int batch, int dir)
{
    return bpf::launch(2, in, idist, out, odist, tw, chirp, nsig, batch, dir, stream());
}

int hsd_r2c_last(const void *Z, long long zdist, void *X, long long xdist, const void *tw, const void *w2, long long h,
                 long long B, int batch, int sgn, int compact)
{
#ifdef HSFFT_DEV_PROBES
    /* development build: HSFFT_R2C_FUSE=2 the round-1 split kernel r8::k_r2c_last (77 vs 93
     * GSamples/s for the fused walk) */
    const char *e = getenv("HSFFT_R2C_FUSE");
    if (!compact && e && atoi(e) == 2) return r8::launch_r2c_last(Z, zdist, X, xdist, tw, w2, h, B, batch, sgn, stream());
#endif
    /* the split walks (pf::k_r2c_walk1 / k_r2c_fused); the host calls this only for the shapes
     * they take ([8,8,8] last pass, A == 1, B % 16 == 0) */
    const int rc = pf::launch_r2c_fused(Z, zdist, X, xdist, tw, w2, h, B, batch, sgn, stream(), compact != 0);
    if (rc == 1) {
        snprintf(g_err, sizeof g_err, "hsd_r2c_last: no split kernel for h=%lld B=%lld", h, B);
        return -1;
    }
    return rc;
}

int mr_has_variant(const hsd_pass *p)
{
    hsd_pass tmp = *p;
    return mr::select(&tmp) != nullptr;
}

int hsd_fill_complex(void *d, int64_t count, uint64_t seed, uint64_t offset)
{
    hipLaunchKernelGGL(k_fill_complex, dim3(4096), dim3(256), 0, stream(), (double2 *)d, (long long)count,
                       (unsigned long long)seed, (unsigned long long)offset);
    HCHK(hipGetLastError());
    return 0;
}

int hsd_fill_real(void *d, int64_t count, uint64_t seed, uint64_t offset)
{
    hipLaunchKernelGGL(k_fill_real, dim3(4096), dim3(256), 0, stream(), (double *)d, (long long)count,
                       (unsigned long long)seed, (unsigned long long)offset);
    HCHK(hipGetLastError());
    return 0;
}

/* the row helpers below index rows by blockIdx.y (at most 65535 per launch): larger
 * batches are launched in slices of Y_MAX rows */
#define Y_MAX 65535

int hsd_r2c_post(const void *Z, const void *tw2, void *X, int h, int batch, long long zdist, long long xdist)
{
    const char *e = getenv("HSFFT_R2C_POST");
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        const double2 *z = (const double2 *)Z + b0 * zdist;
        double2 *x = (double2 *)X + b0 * xdist;
        if (e && atoi(e) == 1)
            hipLaunchKernelGGL(k_r2c_post, dim3(grid_for(h + 1, 256), nb), dim3(256), 0, stream(), z,
                               (const double2 *)tw2, x, h, zdist, xdist);
        else
            hipLaunchKernelGGL(k_r2c_post2<false>, dim3(grid_for(h / 2 + 1, 256), nb), dim3(256), 0, stream(), z,
                               (const double2 *)tw2, x, h, zdist, xdist);
        HCHK(hipGetLastError());
    }
    return 0;
}

/* bins 0..h only (rows of h+1 complex): the non-redundant half of real.c's mirrored output */
int hsd_r2c_post_compact(const void *Z, const void *tw2, void *X, int h, int batch, long long zdist, long long xdist)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        hipLaunchKernelGGL(k_r2c_post2<true>, dim3(grid_for(h / 2 + 1, 256), nb), dim3(256), 0, stream(),
                           (const double2 *)Z + b0 * zdist, (const double2 *)tw2, (double2 *)X + b0 * xdist, h, zdist,
                           xdist);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_c2r_pre(const void *X, const void *tw2, void *Zin, int h, int batch, long long xdist, long long zdist)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        hipLaunchKernelGGL(k_c2r_pre, dim3(grid_for(h, 256), nb), dim3(256), 0, stream(), (const double2 *)X + b0 * xdist,
                           (const double2 *)tw2, (double2 *)Zin + b0 * zdist, h, xdist, zdist);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_cmul(const void *A, const void *Bv, void *C, long long n, int batch, long long dist)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        const long long o = b0 * dist;
        hipLaunchKernelGGL(k_cmul, dim3(grid_for(n, 256), nb), dim3(256), 0, stream(), (const double2 *)A + o,
                           (const double2 *)Bv + o, (double2 *)C + o, n, dist);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_scale_real(void *x, long long n, int batch, long long dist, double divisor)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        hipLaunchKernelGGL(k_scale_real, dim3(grid_for(n, 256), nb), dim3(256), 0, stream(), (double *)x + b0 * dist, n,
                           dist, divisor);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_c2r_pre_mul(const void *A, const void *Bv, const void *tw2, void *Zin, int h, int batch, long long xdist,
                    long long zdist)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        const long long o = b0 * xdist;
        hipLaunchKernelGGL(k_c2r_pre_mul, dim3(grid_for(h, 256), nb), dim3(256), 0, stream(), (const double2 *)A + o,
                           (const double2 *)Bv + o, (const double2 *)tw2, (double2 *)Zin + b0 * zdist, h, xdist, zdist);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_copy_rows_div(const void *src, long long sdist, long long soff, void *dst, long long ddist, long long n,
                      int batch, double divisor)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        hipLaunchKernelGGL(k_copy_rows_div, dim3(grid_for(n, 256), nb), dim3(256), 0, stream(),
                           (const double *)src + b0 * sdist, sdist, soff, (double *)dst + b0 * ddist, ddist, n, divisor);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_copy_rows(const void *src, long long sdist, long long soff, long long ncopy, void *dst, long long ddist,
                  long long dlen, int batch)
{
    for (int b0 = 0; b0 < batch; b0 += Y_MAX) {
        const int nb = batch - b0 < Y_MAX ? batch - b0 : Y_MAX;
        hipLaunchKernelGGL(k_copy_rows, dim3(grid_for(dlen, 256), nb), dim3(256), 0, stream(),
                           (const double *)src + b0 * sdist, sdist, soff, ncopy, (double *)dst + b0 * ddist, ddist, dlen);
        HCHK(hipGetLastError());
    }
    return 0;
}

int hsd_copy_bench(const void *src, void *dst, long long n16, int iters, float *ms)
{
    hipEvent_t e0, e1;
    HCHK(hipEventCreate(&e0));
    HCHK(hipEventCreate(&e1));
    /* the practical HBM ceiling: 4 x 16 B per lane in flight, 65536 x 256 threads (measured
     * the fastest copy variant on 0.5-64 GiB buffers, tools/membench_sizes.py: 5.8-6.0 TB/s) */
    hipLaunchKernelGGL((k_copyU<4, false>), dim3(65536), dim3(256), 0, stream(), (const v2d *)src, (v2d *)dst, n16);
    HCHK(hipEventRecord(e0, stream()));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL((k_copyU<4, false>), dim3(65536), dim3(256), 0, stream(), (const v2d *)src, (v2d *)dst, n16);
    HCHK(hipEventRecord(e1, stream()));
    HCHK(hipEventSynchronize(e1));
    HCHK(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

extern "C" int hsd_copy_bench_v(const void *src, void *dst, long long n16, int iters, int variant, int grid, float *ms)
{
    typedef void (*cfn)(const v2d *, v2d *, long long);
    static const cfn fns[] = {k_copyU<1, false>, k_copyU<4, false>, k_copyU<8, false>,
                              k_copyU<1, true>, k_copyU<4, true>, k_copyU<8, true>};
    if (variant < 0 || variant >= 6) return -1;
    hipEvent_t e0, e1;
    HCHK(hipEventCreate(&e0));
    HCHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(fns[variant], dim3(grid), dim3(256), 0, stream(), (const v2d *)src, (v2d *)dst, n16);
    HCHK(hipEventRecord(e0, stream()));
    for (int i = 0; i < iters; i++)
        hipLaunchKernelGGL(fns[variant], dim3(grid), dim3(256), 0, stream(), (const v2d *)src, (v2d *)dst, n16);
    HCHK(hipEventRecord(e1, stream()));
    HCHK(hipEventSynchronize(e1));
    HCHK(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return 0;
}

int hsd_timer_start(void)
{
    const int dev = cur_dev();
    if (!timer_events(dev)) return set_err(hipErrorOutOfMemory, "hipEventCreate");
    HCHK(hipEventRecord(g_t0[dev], stream()));
    return 0;
}

int hsd_timer_stop(float *ms)
{
    const int dev = cur_dev();
    HCHK(hipEventRecord(g_t1[dev], stream()));
    HCHK(hipEventSynchronize(g_t1[dev]));
    HCHK(hipEventElapsedTime(ms, g_t0[dev], g_t1[dev]));
    return pl_report(); /* a timed persistent launch whose waits timed out is an error, not a time */
}

int hsd_pass_timer_begin(int i)
{
    const int dev = cur_dev();
    if (!timer_events(dev)) return set_err(hipErrorOutOfMemory, "hipEventCreate");
    if (i < 0 || i >= HS_MAX_PASSES) return -1;
    HCHK(hipEventRecord(g_pev[dev][2 * i], stream()));
    return 0;
}

int hsd_pass_timer_end(int i)
{
    if (i < 0 || i >= HS_MAX_PASSES) return -1;
    HCHK(hipEventRecord(g_pev[cur_dev()][2 * i + 1], stream()));
    return 0;
}

int hsd_pass_timer_read(int n, float *ms)
{
    const int dev = cur_dev();
    for (int i = 0; i < n && i < HS_MAX_PASSES; i++) {
        HCHK(hipEventSynchronize(g_pev[dev][2 * i + 1]));
        HCHK(hipEventElapsedTime(&ms[i], g_pev[dev][2 * i], g_pev[dev][2 * i + 1]));
    }
    return pl_report();
}

}  // extern "C"
