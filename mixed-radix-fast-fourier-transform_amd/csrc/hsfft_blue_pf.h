/*
 * hsfft_blue_pf.h -- row-looped kernels for Bluestein's M = 2^18 = [8,8,8 | 8,8,8] (BASELINE
 * config 4, N = 99991), replacing r8::k_blue_mid and the chirp-store k_pass_b512 launch.
 *
 * Bluestein per row (ref src/highSpeedFFT.c:1735-1907): y = chirp * x (zero-padded to M), FFT,
 * times hk (the transformed chirp, :1797), inverse FFT, times chirp.  The two M-point FFTs run
 * as [8,8,8] passes; the forward FFT's second pass, the hk product and the inverse FFT's first
 * pass share their columns (q of the former = m of the latter), so they are one kernel
 * (k_bmid); the inverse's second pass stores through the chirp (k_blast).
 *
 * What differs from the r8 versions: a workgroup keeps its 8-column tile for T rows, so the
 * stage twiddles of the tile (the forward second pass's run is 57 KiB per tile, as many bytes
 * as the tile's data) are loaded once per T rows (LDS runs + stage-2 registers, as
 * pf::k_b512), and the sign / conjugation / direction are template constants.  Arithmetic is
 * the reference's (pf::stage, the chirp and hk products written as r8::chirp_in /
 * store_hook), so results are bit-identical to the r8 path and the CPU reference.
 */
#pragma once

namespace bpf {

using r8::Args;

/* block -> (row group, 8-column tile).  Default: XCD-aware remap, row-group major (every XCD
 * sweeps all 64 tiles).  a.tile_major: XCD x (blockIdx % 8 under round-robin dispatch; speed
 * only, never correctness) owns tiles [8x, 8x+8) of every row group, so the per-tile tables
 * (hk: 64 KiB per tile, the chirp) an XCD reads are 1/8 of them -- 512 KiB, L2-resident. */
__device__ __forceinline__ void split_block(const Args &a, unsigned &bg, unsigned &tile)
{
    const unsigned tiles = (unsigned)a.tiles;
    if (a.tile_major) {
        const unsigned x = blockIdx.x % 8, r = blockIdx.x / 8, tpx = tiles / 8;
        tile = x * tpx + r % tpx;
        bg = r / tpx;
    } else {
        const unsigned blk = pf::xcd_remap(blockIdx.x);
        bg = blk / tiles;
        tile = blk % tiles;
    }
}

/* hk product of the spectrum (ref :1803-1827 -- r8::store_hook HS_STORE_SPEC) */
template <int DIR>
__device__ __forceinline__ void spec(double &yr, double &yi, double2 k)
{
    const double r = yr, i = yi;
    if (DIR == 1) {
        yr = r * k.x - i * k.y;
        yi = r * k.y + i * k.x;
    } else {
        yr = r * k.x + i * k.y;
        yi = -r * k.y + i * k.x;
    }
}

/* chirp product of the output (ref :1871-1886 -- r8::store_hook HS_STORE_CHIRP) */
template <int DIR>
__device__ __forceinline__ double2 chirp_out(double yr, double yi, double2 h)
{
    if (DIR == 1) return make_double2(yr * h.x + yi * h.y, -yr * h.y + yi * h.x);
    return make_double2(yr * h.x - yi * h.y, yr * h.y + yi * h.x);
}

/* forward twiddle runs of q-tile q0 at L = B (stage 0) and L = 8B (stage 1), LDS layout of
 * pf::k_b512: [0, 56) stage 0, [56 (1 + kloc), +56) stage 1 */
template <bool CONJ>
__device__ __forceinline__ void runs_to_lds(double2 *ltw, const double2 *tw, unsigned B, unsigned q0, unsigned tid)
{
    if (tid < 504) {
        const unsigned r = tid / 56, e = tid % 56;
        const long long src = r == 0 ? (long long)B - 1 + 7LL * q0 + e : 8LL * B - 1 + 7LL * (q0 + (long long)B * (r - 1)) + e;
        double2 v = tw[src];
        if (CONJ) v.y = -v.y;
        ltw[tid] = v;
    }
}

/* Forward first pass [8,8,8] (leaf, L = 1, 8, 64) on the chirped, zero-padded input
 * (ref :1803-1827 -- r8::chirp_in), columns m0..m0+7 of T rows.  M = 2^18 >= 2N-1, so only
 * t < 256 (i < 4 of a thread's 8 points t = jt + 64 i) can hold input: the other four are
 * the reference's zero padding (exact +0.0, fed through the same butterfly).  The chirp
 * values of the thread's points are row-invariant and stay in registers for all T rows. */
/* SPLIT: exchanges through a 32 KiB image (real parts, then imaginary parts), so that three
 * workgroups fit per CU (LDS 40 KiB, launch bound 6 waves per SIMD: <= 80 VGPRs) */
template <int T, int S, bool SPLIT = false>
__global__ __launch_bounds__(512, SPLIT ? 6 : 4) void k_bfirst(Args a)
{
    constexpr int P = 512, TPG = 64, G = 8;
    constexpr unsigned A = 512;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + (SPLIT ? P * G / 2 : P * G); /* tw[0, 511): stages L = 8 (kloc < 8) and 64 */
    unsigned bg, tile;
    split_block(a, bg, tile);
    const unsigned tid0 = threadIdx.x;
    const unsigned b0 = bg * T, nb = (unsigned)a.batch, nsig = (unsigned)a.nsig;
    const unsigned m0 = tile * G;
    double2 h[4];
    {
        const unsigned g = tid0 % G, jt = tid0 / G, m = m0 + g;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const unsigned n = (jt + i * TPG) * A + m;
            h[i] = a.laux[n < nsig ? n : 0];
        }
    }
    if (tid0 < 511) ltw[tid0] = a.tw[tid0];
    __syncthreads();
    const int nit = (int)min((unsigned)T, nb - b0);
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned g = tid % G, jt = tid / G, m = m0 + g;
        const double2 *row = a.in + (long long)(b0 + it) * a.idist;
        double xr[8], xi[8];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const unsigned n = (jt + i * TPG) * A + m;
            const bool inside = n < nsig;
            const double2 x = row[inside ? n : 0];
            double2 v = make_double2(0.0, 0.0);
            if (inside) {
                if (S == 1) v = make_double2(x.x * h[i].x + x.y * h[i].y, -x.x * h[i].y + x.y * h[i].x);
                else v = make_double2(x.x * h[i].x - x.y * h[i].y, x.x * h[i].y + x.y * h[i].x);
            }
            xr[i] = v.x;
            xi[i] = v.y;
            xr[i + 4] = 0.0;
            xi[i + 4] = 0.0;
        }
        double2 w[7];
        pf::stage<8, S>(xr, xi, w, true);
        r8::exchange<8, 1, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = ltw[7 + 7 * (jt & 7) + i];
        pf::stage<8, S>(xr, xi, w, false);
        r8::exchange<8, 8, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = ltw[63 + 7 * (jt & 63) + i];
        pf::stage<8, S>(xr, xi, w, false);
        double2 *orow = a.out + (long long)(b0 + it) * a.odist;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) pf::stg(orow + jj * TPG, (m * P + jt) * 16u, make_double2(xr[jj], xi[jj]));
    }
}

/* Forward second pass [8,8,8] at L = B = 512 of q-tile q0, hk product, inverse first pass
 * [8,8,8] (leaf, column m = q, sign -S, conjugated twiddles), for T rows.
 * in: forward first-pass output rows, out: inverse first-pass output rows, saux: hk. */
template <int T, int S>
__global__ __launch_bounds__(512, 4) void k_bmid(Args a)
{
    constexpr int P = 512, TPG = 64, G = 8;
    constexpr unsigned B = 512;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + P * G; /* forward runs, 504 entries */
    unsigned bg, tile;
    split_block(a, bg, tile);
    const unsigned tid0 = threadIdx.x, q0 = tile * G;
    const unsigned b0 = bg * T, nb = (unsigned)a.batch;
    const double2 *hk = a.saux;

    double2 *itw = ltw + 504; /* tw[0, 511): the inverse first pass's stages L = 8, 64 */
    double2 w2[7];
    r8::load_tw_co<64>(w2, a, tid0 / G, q0);
    runs_to_lds<false>(ltw, a.tw, B, q0, tid0);
    if (tid0 < 511) itw[tid0] = a.tw[tid0];
    r8::redistribute_tw(w2, lds);
    __syncthreads();

    const int nit = (int)min((unsigned)T, nb - b0);
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned g = tid % G, jt = tid / G, q = q0 + g;
        const unsigned lane = (jt * B + q) * 16u;
        const double2 *row = a.in + (long long)(b0 + it) * a.idist;
        double xr[8], xi[8];
        double2 k[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = pf::ldg(row + (size_t)i * TPG * B, lane);
            xr[i] = v.x;
            xi[i] = v.y;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) k[i] = pf::ldg(hk + (size_t)i * TPG * B, lane);
        /* forward FFT, second pass (twiddles as pf::b512_body) */
        double2 w[7];
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = ltw[7 * g + i];
        pf::stage<8, S>(xr, xi, w, false);
        r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = ltw[56 * (1 + (jt & 7)) + 7 * g + i];
        pf::stage<8, S>(xr, xi, w, false);
        r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
        pf::stage<8, S>(xr, xi, w2, false);
        /* spectrum product: thread holds u = jt + 64 jj of column q, element u*B + q */
#pragma unroll
        for (int jj = 0; jj < 8; jj++) spec<S>(xr[jj], xi[jj], k[jj]);
        /* inverse FFT, first pass on column m = q: leaf, then L = 8, 64 (k = k_local; the
         * small tables are cache-resident and nothing else is in flight here) */
        pf::stage<8, -S>(xr, xi, w, true);
        r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
        pf::tw8_lds<true>(w, itw, 8, jt & 7);
        pf::stage<8, -S>(xr, xi, w, false);
        r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
        pf::tw8_lds<true>(w, itw, 64, jt & 63);
        pf::stage<8, -S>(xr, xi, w, false);
        double2 *orow = a.out + (long long)(b0 + it) * a.odist;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) pf::stg(orow + jj * TPG, (q * P + jt) * 16u, make_double2(xr[jj], xi[jj]));
    }
}

/* Inverse FFT's second pass [8,8,8] at L = B = 512 (sign -S, conjugated twiddles) of q-tile
 * q0 for T rows, stored through the chirp for n < nsig (direction S).  Row prefetch (PREF)
 * is a template option the launcher does not use (as for pf::k_b512: with it the kernel spills 20 B). */
template <int T, int S, bool PREF = true, bool SPLIT = false>
__global__ __launch_bounds__(512, SPLIT ? 6 : 4) void k_blast(Args a)
{
    constexpr int P = 512, TPG = 64, G = 8;
    constexpr unsigned B = 512;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + (SPLIT ? P * G / 2 : P * G);
    unsigned bg, tile;
    split_block(a, bg, tile);
    const unsigned tid0 = threadIdx.x, q0 = tile * G;
    const unsigned b0 = bg * T, nb = (unsigned)a.batch;
    const unsigned nsig = (unsigned)a.nsig;

    double pr[8], pi[8];
    if constexpr (PREF) {
        const double2 *row = a.in + (long long)b0 * a.idist;
        const unsigned lane = ((tid0 / G) * B + q0 + tid0 % G) * 16u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = pf::ldg(row + (size_t)i * TPG * B, lane);
            pr[i] = v.x;
            pi[i] = v.y;
        }
    }
    double2 w2[7];
    if constexpr (SPLIT) { /* per-lane run (the redistribution image would not fit) */
        const long long base = 64LL * B - 1 + 7LL * (q0 + tid0 % G + (long long)B * (tid0 / G));
#pragma unroll
        for (int i = 0; i < 7; i++) w2[i] = a.tw[base + i];
        runs_to_lds<true>(ltw, a.tw, B, q0, tid0);
    } else {
        r8::load_tw_co<64>(w2, a, tid0 / G, q0);
        runs_to_lds<true>(ltw, a.tw, B, q0, tid0);
        r8::redistribute_tw(w2, lds);
    }
#pragma unroll
    for (int i = 0; i < 7; i++) w2[i].y = -w2[i].y;
    __syncthreads();

    const int nit = (int)min((unsigned)T, nb - b0);
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned g = tid % G, jt = tid / G, q = q0 + g;
        const unsigned lane = (jt * B + q) * 16u;
        double xr[8], xi[8];
        if constexpr (PREF) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                xr[i] = pr[i];
                xi[i] = pi[i];
            }
        } else {
            const double2 *rowc = a.in + (long long)(b0 + it) * a.idist;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = pf::ldg(rowc + (size_t)i * TPG * B, lane);
                xr[i] = v.x;
                xi[i] = v.y;
            }
        }
        /* next row's loads (the last iteration re-reads its own row: no branch around the
         * loads, so nothing in the loop drains vmcnt early) */
        if constexpr (PREF) {
            const unsigned bn = it + 1 < nit ? b0 + it + 1 : b0 + it;
            const double2 *rown = a.in + (long long)bn * a.idist;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = pf::ldg(rown + (size_t)i * TPG * B, lane);
                pr[i] = v.x;
                pi[i] = v.y;
            }
        }
        double2 w[7];
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = ltw[7 * g + i];
        pf::stage<8, -S>(xr, xi, w, false);
        r8::exchange<8, 1, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = ltw[56 * (1 + (jt & 7)) + 7 * g + i];
        pf::stage<8, -S>(xr, xi, w, false);
        r8::exchange<8, 8, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
        pf::stage<8, -S>(xr, xi, w2, false);
        /* output n = u*B + q, u = jt + 64 jj; only n < nsig is stored (ref :1871-1886) */
        double2 *orow = a.out + (long long)(b0 + it) * a.odist;
        const double2 *ch = a.saux;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned n = (jt + jj * TPG) * B + q;
            if (n < nsig) orow[n] = chirp_out<S>(xr[jj], xi[jj], ch[n]);
        }
    }
}

typedef void (*kfn)(Args);

inline int env(const char *name, int dflt)
{
    const char *s = getenv(name);
    return s ? atoi(s) : dflt;
}

/* launch the row-looped middle (which = 0), last (1) or first (2) kernel; 1 if not enabled */
inline int launch(int which, const void *in, long long idist, void *out, long long odist, const void *tw,
                  const void *aux, long long nsig, int batch, int sgn, hipStream_t st)
{
    const int mask = env("HSFFT_BLUE_PF", 7);
    if (!((mask >> which) & 1) || (sgn != 1 && sgn != -1)) return 1;
    /* 8 rows per workgroup (measured c4: T 2 17.8, 4 18.7, 8 19.1 GS/s); the last kernel without
     * a row prefetch (20.98 vs 20.26 GS/s with it: it spills); the split-exchange variants
     * (three workgroups per CU) measured +0.6 % / -5 % and were removed in round 3 */
    constexpr int T = 8;
    kfn fn;
    if (which == 2) fn = sgn == 1 ? k_bfirst<8, 1> : k_bfirst<8, -1>;
    else if (which == 0) fn = sgn == 1 ? k_bmid<8, 1> : k_bmid<8, -1>;
    else fn = sgn == 1 ? k_blast<8, 1, false> : k_blast<8, -1, false>;
    Args a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)in;
    a.out = (double2 *)out;
    a.tw = (const double2 *)tw;
    a.saux = (const double2 *)aux;
    a.laux = (const double2 *)aux;
    a.idist = idist;
    a.odist = odist;
    a.A = 1;
    a.B = 512;
    a.nsig = nsig;
    a.batch = batch;
    a.tiles = a.tiles_q = 512 / 8;
    /* HSFFT_BLUE_XT bit 0 first, bit 1 middle, bit 2 last kernel: XCD-owned tiles (c4 under rocprof:
     * mask 0 21.05, 7 21.37, 3 22.11 GS/s -- the last kernel reads in natural order; earlier 20.9 -> 21.4
     * with all three; tiles % 8 == 0, so grid % 8 == 0) */
    a.tile_major = (env("HSFFT_BLUE_XT", 3) >> (which == 2 ? 0 : which == 0 ? 1 : 2)) & 1;
    const long long grid = a.tiles * ((batch + T - 1) / T);
    if (grid <= 0 || grid > 0x7fffffffLL) return -1;
    /* image + twiddle runs (k_bfirst: 511; k_bmid: 504 forward runs + 511 inverse entries) */
    const size_t lds = (size_t)(512 * 8 + (which == 0 ? 1016 : 512)) * sizeof(double2);
    HCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(512), lds, st, a);
    HCHK(hipGetLastError());
    return 0;
}

}  // namespace bpf
