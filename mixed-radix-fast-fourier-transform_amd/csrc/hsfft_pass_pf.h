/*
 * hsfft_pass_pf.h -- software-pipelined register passes for the power-of-two hot path
 * (BASELINE config 2: 2^20 = [4,8,8,8 | 8,8,8]; same shapes serve 2^18 / 2^21 / 2^22).
 *
 * Why a second family next to hsfft_pass_r8.h: a k_pass workgroup loads its tile, waits,
 * computes and stores, so a CU only keeps HBM busy through the other resident workgroups
 * (measured: ~4.8 TB/s per pass against a 6.0 TB/s copy of the same buffers).  Here every
 * workgroup walks several tiles (first pass: TL column tiles of one row; later pass: T rows
 * of one column tile) and issues the loads of tile i+1 before computing tile i, so 64 KiB
 * per workgroup are always in flight.  That only works if nothing inside the loop waits on
 * the vector-memory counter: the twiddles of every stage are the same for all tiles a
 * workgroup walks (first pass: k = k_local; later pass: k = q + B*k_local with q fixed), so
 * they are loaded once, before the loop, and kept in registers; the butterfly sign and the
 * twiddle conjugation are template constants (conjugation applied once at load).
 *
 * Arithmetic is unchanged (hsfft_butterfly.h: the reference's operand order, no FMA), so
 * results are bit-identical to k_pass and to the CPU reference.
 */
#pragma once

namespace pf {

#ifdef HSFFT_DEV_PROBES
/* development build only (results WRONG when changed): mask on the k_local of the global
 * L = 512 twiddles of a 4096-point first pass (HSFFT_PFA_PROBE=1: 7, i.e. one 7-entry run) */
__device__ unsigned pf_probe_twmask = 0xffffffffu;
#define PF_TWMASK pf_probe_twmask
#else
#define PF_TWMASK 0xffffffffu
#endif

using r8::Args;
using r8::Shape;

__device__ __forceinline__ unsigned xcd_remap(unsigned blk)
{
    const unsigned nwg = gridDim.x, q8 = nwg / 8, r8_ = nwg % 8, xcd = blk % 8;
    return (xcd < r8_ ? xcd * (q8 + 1) : r8_ * (q8 + 1) + (xcd - r8_) * q8) + blk / 8;
}

/* twiddles of one radix-8 stage for a thread whose butterfly has k = k0 + B*kloc
 * (ref :1310-1474: tw[L-1 + 7k + i-1], L = B*LLOC); CONJ negates the imaginary parts */
template <bool CONJ>
__device__ __forceinline__ void tw8(double2 (&w)[7], const double2 *tw, long long L, long long k)
{
    const double2 *p = tw + (L - 1 + 7 * k);
#pragma unroll
    for (int i = 0; i < 7; i++) {
        double2 v = p[i];
        if (CONJ) v.y = -v.y;
        w[i] = v;
    }
}

/* one stage on this thread's 8 points: twiddles (radix-8 combine only) + 8/R butterflies */
template <int R, int SGN>
__device__ __forceinline__ void stage(double (&xr)[8], double (&xi)[8], const double2 (&w)[7], bool leaf)
{
    constexpr int NB = 8 / R;
#pragma unroll
    for (int c = 0; c < NB; c++) {
        if (!leaf) {
#pragma unroll
            for (int i = 1; i < R; i++) hsb::twmul(xr[c * R + i], xi[c * R + i], w[i - 1].x, w[i - 1].y);
        }
        hsb::bfly<R>(&xr[c * R], &xi[c * R], SGN, leaf);
    }
}

/* global access as uniform base + 32-bit per-lane byte offset (saddr form: one VGPR of
 * address per access instead of a 64-bit pair; rows are < 4 GiB) */
__device__ __forceinline__ double2 ldg(const void *base, unsigned boff)
{
    return *(const double2 *)((const char *)base + boff);
}
__device__ __forceinline__ void stg(void *base, unsigned boff, double2 v) { *(double2 *)((char *)base + boff) = v; }
/* non-temporal forms (streamed once: keep them from displacing cache-resident data) */
typedef double pf_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ldg_nt(const void *base, unsigned boff)
{
    const pf_d2v v = __builtin_nontemporal_load((const pf_d2v *)((const char *)base + boff));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void stg_nt(void *base, unsigned boff, double2 v)
{
    pf_d2v u;
    u.x = v.x;
    u.y = v.y;
    __builtin_nontemporal_store(u, (pf_d2v *)((char *)base + boff));
}

/* ------------------------------------------------------------------ first pass
 * [R0, 8^N8] leaf pass (B == 1): input [t][m] (t < P, m < A), output [m][u].  A workgroup
 * owns G adjacent columns per tile and walks TL tiles of one row with stride `groups`, so the
 * workgroups next to it (same XCD after xcd_remap) work on the neighbouring columns at the
 * same time and each 128-B line is fetched into L2 once for 8/G of them. */
template <int R0, int N8, int G>
__device__ __forceinline__ void first_load(double (&xr)[8], double (&xi)[8], const double2 *row, unsigned A,
                                           unsigned m, unsigned jt)
{
    constexpr int P = Shape<R0, N8>::P, TPG = Shape<R0, N8>::TPG, NB = 8 / R0, S0 = P / R0;
    const unsigned lane = (jt * A + m) * 16u;
#pragma unroll
    for (int c = 0; c < NB; c++)
#pragma unroll
        for (int i = 0; i < R0; i++) {
            const double2 v = ldg(row + (size_t)(c * TPG + i * S0) * A, lane);
            xr[c * R0 + i] = v.x;
            xi[c * R0 + i] = v.y;
        }
}

/* twiddles of stage s of a first pass from the LDS copy of tw[0, P) */
template <bool CONJ>
__device__ __forceinline__ void tw8_lds(double2 (&w)[7], const double2 *ltw, unsigned L, unsigned kloc)
{
#pragma unroll
    for (int i = 0; i < 7; i++) {
        double2 v = ltw[L - 1 + 7 * kloc + i];
        if (CONJ) v.y = -v.y;
        w[i] = v;
    }
}

/* stages + exchanges + store of one first-pass tile held in xr/xi; ocol = output column */
template <int R0, int N8, int G, int SGN, bool CONJ, bool TWG = false, bool NTS = false>
__device__ __forceinline__ void first_body(double (&xr)[8], double (&xi)[8], double2 *lds, const double2 *ltw,
                                           double2 *orow, unsigned m, unsigned jt, unsigned g,
                                           const double2 *gtw = nullptr)
{
    /* TWG: the third combine stage's twiddles come from the plan's table in global memory
     * (L2-resident) instead of the LDS copy, so P = 4096 keeps an 8 KiB LDS table */
    using S = Shape<R0, N8>;
    constexpr int P = S::P, TPG = S::TPG;
    double2 w[7];
    stage<R0, SGN>(xr, xi, w, true);
    if constexpr (N8 >= 1) {
        r8::exchange<R0, 1, 8, TPG, P, G, true>(xr, xi, lds, jt, g);
        tw8_lds<CONJ>(w, ltw, S::Lloc(1), jt & (S::Lloc(1) - 1));
        stage<8, SGN>(xr, xi, w, false);
    }
    if constexpr (N8 >= 2) {
        r8::exchange<8, S::Lloc(1), 8, TPG, P, G, true>(xr, xi, lds, jt, g);
        tw8_lds<CONJ>(w, ltw, S::Lloc(2), jt & (S::Lloc(2) - 1));
        stage<8, SGN>(xr, xi, w, false);
    }
    if constexpr (N8 >= 3) {
        if constexpr (TWG) tw8<CONJ>(w, gtw, S::Lloc(3), jt & (S::Lloc(3) - 1) & PF_TWMASK);
        r8::exchange<8, S::Lloc(2), 8, TPG, P, G, true>(xr, xi, lds, jt, g);
        if constexpr (!TWG) tw8_lds<CONJ>(w, ltw, S::Lloc(3), jt & (S::Lloc(3) - 1));
        stage<8, SGN>(xr, xi, w, false);
    }
    /* last stage: output u = jt + jj*LL of the column, written to [m][u] */
    constexpr int LL = S::Lloc(S::NST - 1);
#pragma unroll
    for (int jj = 0; jj < 8; jj++) {
        if constexpr (NTS) stg_nt(orow + jj * LL, (m * P + jt) * 16u, make_double2(xr[jj], xi[jj]));
        else stg(orow + jj * LL, (m * P + jt) * 16u, make_double2(xr[jj], xi[jj]));
    }
}

/* ------------------------------------------------------------------ first pass, paired loads
 * Same [R0, 8^N8] first pass and the same G-column compute as k_first, but every column read
 * is a 2G-column row segment (G = 2: 64 B, G = 1: 32 B): a workgroup owns 2G adjacent
 * columns m0.. (two G-column tiles), and the 2G lanes of threads jt, jt+1 (even / odd, each
 * with h < G) load one row segment per instruction: load A gives the even thread its own
 * tile-0 values (row jt) and the odd thread the even one's tile-1 values; load B the other
 * way round (row jt+1).  A DPP swap (lanes G apart inside a quad) returns the borrowed values.
 * k_first's G-column segments cost one L2 request per 16 G bytes, and that request rate, not
 * HBM, is what holds it below the copy rate (TA stalled by TC). */
template <int G>
__device__ __forceinline__ double pair_swap(double v)
{
    constexpr int CTRL = G == 2 ? 0x4E : 0xB1; /* quad_perm [2,3,0,1] / [1,0,3,2] */
    int2 u;
    __builtin_memcpy(&u, &v, 8);
    u.x = __builtin_amdgcn_mov_dpp(u.x, CTRL, 0xF, 0xF, false);
    u.y = __builtin_amdgcn_mov_dpp(u.y, CTRL, 0xF, 0xF, false);
    double r;
    __builtin_memcpy(&r, &u, 8);
    return r;
}

template <int R0, int N8, int G, int SGN, bool CONJ, bool NTS = false>
__global__ __launch_bounds__((Shape<R0, N8>::TPG * G), 4) void k_firstq(Args a)
{
    using S = Shape<R0, N8>;
    constexpr int P = S::P, TPG = S::TPG, NT = TPG * G, NB = 8 / R0, S0 = P / R0;
    /* P = 4096: the L = 512 stage's twiddles from global memory (LDS: 32 + 8 KiB) */
    constexpr bool TWG = N8 >= 3 && P > 2048;
    constexpr int NTAB = TWG ? S::Lloc(3) - 1 : P - 1;
    static_assert((G == 1 || G == 2) && N8 >= 1 && TPG % 2 == 0, "paired loads");
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + P * G / 2; /* after the split image (P * G doubles) */
    const unsigned blk = a.xcd_groups > 0 ? xcd_remap(blockIdx.x) : blockIdx.x;
    const unsigned groups = (unsigned)a.tiles_q; /* 2G-column groups per row */
    const unsigned b = blk / groups, sg = blk % groups;
    const unsigned A = (unsigned)a.A, nsup = A / (2 * G);
    const double2 *row = a.in + (long long)b * a.idist;
    double2 *orow = a.out + (long long)b * a.odist;
#pragma unroll 1
    for (int i = threadIdx.x; i < NTAB; i += NT) ltw[i] = a.tw[i];
    __syncthreads();
    const int nit = (int)((nsup - 1 - sg) / groups + 1);
    /* the paired row-segment loads of column group `it` */
    auto load_group = [&](double2 (&va)[8], double2 (&vb)[8], int it, unsigned tid) {
        const unsigned h = tid % G, jt = tid / G, odd = jt & 1;
        const unsigned m0 = (sg + it * groups) * (2 * G);
        const unsigned offA = ((jt - odd) * A + m0 + h + G * odd) * 16u;
        const unsigned offB = ((jt + 1 - odd) * A + m0 + h + G - G * odd) * 16u;
#pragma unroll
        for (int c = 0; c < NB; c++)
#pragma unroll
            for (int i = 0; i < R0; i++) {
                const double2 *rb = row + (size_t)(c * TPG + i * S0) * A;
                va[c * R0 + i] = ldg(rb, offA);
                vb[c * R0 + i] = ldg(rb, offB);
            }
    };
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const unsigned h = tid % G, jt = tid / G, odd = jt & 1;
        const unsigned m0 = (sg + it * groups) * (2 * G);
        double2 va[8], vb[8];
        load_group(va, vb, it, tid);
        double xr[8], xi[8], yr[8], yi[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const double2 own = odd ? vb[k] : va[k], oth = odd ? va[k] : vb[k];
            xr[k] = own.x;
            xi[k] = own.y;
            yr[k] = pair_swap<G>(oth.x);
            yi[k] = pair_swap<G>(oth.y);
        }
        first_body<R0, N8, G, SGN, CONJ, TWG, NTS>(xr, xi, lds, ltw, orow, m0 + h, jt, h, a.tw);
        first_body<R0, N8, G, SGN, CONJ, TWG, NTS>(yr, yi, lds, ltw, orow, m0 + G + h, jt, h, a.tw);
    }
}

/* ------------------------------------------------------------------ later pass [8,8,8]
 * P = 512 at L = B (A == 1): input [t][q] (t < 512, q < B), output [u][q].  A workgroup
 * owns 8 adjacent q-columns (128-B rows) and walks T rows of the batch; all three stages'
 * twiddles (k = q + B*kloc) are row-independent: stages 0/1 as LDS runs, stage 2 in
 * registers. */
/* stages + exchanges + store of one [8,8,8] tile-row; ocol = output row + q */
template <int SGN, bool NTS = false>
__device__ __forceinline__ void b512_body(double (&xr)[8], double (&xi)[8], const double2 (&w2)[7], double2 *lds,
                                          const double2 *ltw, double2 *orow, unsigned B, unsigned lane, unsigned jt,
                                          unsigned g)
{
    constexpr int P = 512, TPG = 64, G = 8;
    double2 w[7];
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ltw[7 * g + i];
    stage<8, SGN>(xr, xi, w, false);
    r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ltw[56 * (1 + (jt & 7)) + 7 * g + i];
    stage<8, SGN>(xr, xi, w, false);
    r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
    stage<8, SGN>(xr, xi, w2, false);
#pragma unroll
    for (int jj = 0; jj < 8; jj++) {
        if constexpr (NTS) stg_nt(orow + (size_t)jj * TPG * B, lane, make_double2(xr[jj], xi[jj]));
        else stg(orow + (size_t)jj * TPG * B, lane, make_double2(xr[jj], xi[jj]));
    }
}

template <int T, int SGN, bool CONJ>
__global__ __launch_bounds__(512, 4) void k_b512(Args a)
{
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    /* [0, 4096): exchange image; then the stage-0 run (8 q x 7) and the 8 stage-1 runs
     * (k_local = 0..7, 8 q x 7 each) of this tile's twiddles */
    double2 *ltw = lds + P * G;
    const unsigned blk = a.xcd_groups > 0 ? xcd_remap(blockIdx.x) : blockIdx.x;
    const unsigned tiles = (unsigned)a.tiles;
    const unsigned bg = blk / tiles, tile = blk % tiles;
    const unsigned tid0 = threadIdx.x;
    const unsigned B = (unsigned)a.B;
    const unsigned q0 = tile * G;
    const unsigned b0 = bg * T, nb = (unsigned)a.batch;

    /* stage-2 twiddles (k = q + B*k_local, k_local < 64): coalesced runs redistributed
     * through this wave's slice of the image, kept in registers for all T rows */
    double2 w2[7];
    r8::load_tw_co<64>(w2, a, tid0 / G, q0);
    if (tid0 < 504) {
        const int r = tid0 / 56, e = tid0 % 56;
        const long long src = r == 0 ? (long long)B - 1 + 7LL * q0 + e
                                     : 8LL * B - 1 + 7LL * (q0 + (long long)B * (r - 1)) + e;
        double2 v = a.tw[src];
        if (CONJ) v.y = -v.y;
        ltw[tid0] = v;
    }
    r8::redistribute_tw(w2, lds);
    if (CONJ) {
#pragma unroll
        for (int i = 0; i < 7; i++) w2[i].y = -w2[i].y;
    }
    __syncthreads();

    /* no row prefetch: measured 22.8 ms with it off (106 VGPRs) vs 23.4 ms with it on (128
     * VGPRs + 40 B of spill) per 4096 x 2^20 */
    const int nit = (int)min((unsigned)T, nb - b0);
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned g = tid % G, jt = tid / G;
        const unsigned b = b0 + it, lane = (jt * B + q0 + g) * 16u;
        const double2 *row = a.in + (long long)b * a.idist;
        double xr[8], xi[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = ldg(row + (size_t)i * TPG * B, lane);
            xr[i] = v.x;
            xi[i] = v.y;
        }
        b512_body<SGN>(xr, xi, w2, lds, ltw, a.out + (long long)b * a.odist, B, lane, jt, g);
    }
}

/* ------------------------------------------------------------------ r2c split in pass B
 * real.c's split (ref :108-132) fused into the last [8,8,8] pass of the inner c2c of h = P*B
 * points (2^21 for r2c 2^22): output k = u*B + q pairs with h - k = (P-1-u)*B + (B-q), so the
 * q-columns [8j+1, 8j+9) ("lo") and [B-8j-8, B-8j) ("hi") are closed under the pairing.  A
 * workgroup transforms both tiles (k_b512's stages: stage-0/1 twiddle runs in LDS, stage-2
 * twiddles coalesced and redistributed), swaps the hi tile through LDS and writes X[k],
 * X[N-k], X[h-k], X[h+k] of its lo tile (COMPACT: rows of h+1 bins, X[k] and X[h-k] only).
 * Tile j == B/16 is column 0 (u <-> P-u, X[0], X[h]).
 * Saves the c2c output's write and re-read (16 of 56 bytes per real sample). */
/* one tile's row loads, its stage-0/1 twiddle runs (-> ltw) and stage-2 twiddles (coalesced,
 * redistributed through the image: every earlier reader of the image must be done) */
__device__ __forceinline__ void r2c_load(double (&xr)[8], double (&xi)[8], double2 (&w2)[7], const double2 *row,
                                         unsigned B, unsigned q0, const double2 *tw, double2 *lds, double2 *ltw,
                                         unsigned tid0)
{
    constexpr int TPG = 64;
    const unsigned lane0 = ((tid0 >> 3) * B + q0 + (tid0 & 7)) * 16u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const double2 v = ldg(row + (size_t)i * TPG * B, lane0);
        xr[i] = v.x;
        xi[i] = v.y;
    }
    r8::Args ta;
    ta.tw = tw;
    ta.B = B;
    r8::load_tw_co<64>(w2, ta, (int)(tid0 >> 3), q0);
    __syncthreads(); /* earlier readers of the image and of ltw are done */
    if (tid0 < 504) {
        const unsigned r = tid0 / 56, e = tid0 % 56;
        const long long src = r == 0 ? (long long)B - 1 + 7LL * q0 + e : 8LL * B - 1 + 7LL * (q0 + (long long)B * (r - 1)) + e;
        ltw[tid0] = tw[src];
    }
    r8::redistribute_tw(w2, lds);
    __syncthreads(); /* ltw written; every wave has read its redistributed twiddles back */
}

/* the tile's three stages; SPLIT: exchanges through doubles [0, 4096) only */
template <int SGN, bool SPLIT>
__device__ __forceinline__ void r2c_stages(double (&xr)[8], double (&xi)[8], const double2 (&w2)[7], double2 *lds,
                                           const double2 *ltw, unsigned tid0)
{
    constexpr int TPG = 64, P = 512, G = 8;
    unsigned tid = tid0;
    asm volatile("" : "+v"(tid));
    const unsigned g = tid & 7, jt = tid >> 3;
    double2 w[7];
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ltw[7 * g + i];
    stage<8, SGN>(xr, xi, w, false);
    r8::exchange<8, 1, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ltw[56 * (1 + (jt & 7)) + 7 * g + i];
    stage<8, SGN>(xr, xi, w, false);
    r8::exchange<8, 8, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
    stage<8, SGN>(xr, xi, w2, false);
}

template <int SGN, bool COMPACT>
__global__ __launch_bounds__(512, 4) void k_r2c_fused(Args a, unsigned h)
{
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + P * G;
    double *ld = reinterpret_cast<double *>(lds); /* [0, 4096): split image / hi imag, [4096, 8192): hi real */
    const unsigned blk = xcd_remap(blockIdx.x);
    const unsigned tiles = (unsigned)a.tiles, b = blk / tiles, j = blk % tiles;
    const unsigned tid0 = threadIdx.x, B = (unsigned)a.B, N = 2 * h;
    const double2 *row = a.in + (long long)b * a.idist;
    double2 *X = a.out + (long long)b * a.odist;
    const double2 *w2t = a.saux;
    double xr[8], xi[8];
    double2 w2[7];
    const unsigned g = tid0 & 7, jt = tid0 >> 3;
    if (j < tiles - 1) {
        const unsigned qlo = 8 * j + 1, qhi = B - 8 * j - 8;
        double hr[8], hi[8];
        r2c_load(hr, hi, w2, row, B, qhi, a.tw, lds, ltw, tid0);
        r2c_stages<SGN, false>(hr, hi, w2, lds, ltw, tid0);
        r2c_load(xr, xi, w2, row, B, qlo, a.tw, lds, ltw, tid0);
        /* the hi tile's real parts wait in the image's upper half (the lo tile's split
         * exchanges use the lower half), so only its imaginary parts stay in registers */
#pragma unroll
        for (int jj = 0; jj < 8; jj++) ld[4096 + (jt + jj * TPG) * G + g] = hr[jj];
        r2c_stages<SGN, true>(xr, xi, w2, lds, ltw, tid0);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) ld[(jt + jj * TPG) * G + g] = hi[jj];
        __syncthreads();
        const unsigned q = qlo + g;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, k = u * B + q, hk = h - k;
            const unsigned s = (P - 1 - u) * G + (7 - g);
            const double2 zk = make_double2(xr[jj], xi[jj]), zh = make_double2(ld[4096 + s], ld[s]);
            double re, im;
            r8::r2c_pair(zk, zh, w2t[k], re, im);
            X[k] = make_double2(re, im);
            if (!COMPACT) X[N - k] = make_double2(re, -im);
            r8::r2c_pair(zh, zk, w2t[hk], re, im);
            X[hk] = make_double2(re, im);
            if (!COMPACT) X[N - hk] = make_double2(re, -im);
        }
    } else { /* column 0: k = u*B pairs with (P-u)*B */
        r2c_load(xr, xi, w2, row, B, 0, a.tw, lds, ltw, tid0);
        r2c_stages<SGN, false>(xr, xi, w2, lds, ltw, tid0);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) lds[(jt + jj * TPG) * G + g] = make_double2(xr[jj], xi[jj]);
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, k = u * B;
            const double2 zk = make_double2(xr[jj], xi[jj]);
            if (u == 0) {
                X[0] = make_double2(zk.x + zk.y, 0.0);
                X[h] = make_double2(zk.x - zk.y, 0.0);
            } else {
                const double2 zh = lds[(P - u) * G];
                double re, im;
                r8::r2c_pair(zk, zh, w2t[k], re, im);
                X[k] = make_double2(re, im);
                if (!COMPACT) X[N - k] = make_double2(re, -im);
            }
        }
    }
}

/* lane (g-1) of this 8-lane group (DIR = -1) or lane (g+1) (DIR = +1), wrapping in the group */
template <int DIR>
__device__ __forceinline__ double2 grp_shift(double2 v)
{
    const int lane = __lane_id(), src = (lane & ~7) | ((lane + DIR) & 7);
    return make_double2(__shfl(v.x, src, 64), __shfl(v.y, src, 64));
}

/* ------------------------------------------------------------------ r2c split, 512-thread walk
 * k_r2c_walk's whole-line stores with k_r2c_fused's sequential hi / lo tiles, in ONE 8-wave
 * workgroup per CU with 256 VGPRs, software pipelined instead of relying on a second resident
 * workgroup: the lo tile's points and twiddle runs load while the hi tile is transformed, the
 * next hi tile's while the lo tile is transformed (two register buffers A / B, transformed in
 * place).  The lo thread writes all four streams of its pair; X[k] and X[h+k] go out on whole
 * lines through the one-lane shift and the carried entry (LDS, same thread), as in k_r2c_walk. */
struct R2cBuf {
    double r[8], i[8];
    double2 w[7]; /* stage-2 twiddle run, coalesced order (redistributed when used) */
    double2 l;    /* this thread's entry of the stage-0/1 twiddle runs (threads < 504) */
};

/* TWP (timing probe, -DHSFFT_DEV_PROBES builds only): every tile reads column 0's twiddle
 * runs (cache-resident; results wrong) */
template <bool TWP = false>
__device__ __forceinline__ void r2cw2_issue(R2cBuf &d, const double2 *row, unsigned B, unsigned q0, const double2 *tw,
                                            unsigned tid)
{
    constexpr int TPG = 64;
    const unsigned lane0 = ((tid >> 3) * B + q0 + (tid & 7)) * 16u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const double2 v = ldg(row + (size_t)i * TPG * B, lane0);
        d.r[i] = v.x;
        d.i[i] = v.y;
    }
    const unsigned qt = TWP ? 0u : q0;
    r8::Args ta;
    ta.tw = tw;
    ta.B = B;
    r8::load_tw_co<64>(d.w, ta, (int)(tid >> 3), qt);
    const unsigned t = tid < 504 ? tid : 0, r = t / 56, e = t % 56;
    const long long src = r == 0 ? (long long)B - 1 + 7LL * qt + e : 8LL * B - 1 + 7LL * (qt + (long long)B * (r - 1)) + e;
    d.l = tw[src];
}

/* twiddles of the buffered tile -> ltw (runs) and w2 (redistributed through the image) */
__device__ __forceinline__ void r2cw2_tw(const R2cBuf &d, double2 (&w2)[7], double2 *lds, double2 *ltw, unsigned tid)
{
#pragma unroll
    for (int i = 0; i < 7; i++) w2[i] = d.w[i];
    __syncthreads(); /* earlier readers of the image and of ltw are done */
    if (tid < 504) ltw[tid] = d.l;
    r8::redistribute_tw(w2, lds);
    __syncthreads();
}

constexpr int R2CW2_LDS = (512 * 8 + 504 + 1024) * 16;

/* V (measurement variants; 0 is the default): bit 0 phase trace into a.dbg; -DHSFFT_DEV_PROBES
 * builds only (results WRONG): bit 1 twiddle2 read from one cache-resident line per lane group,
 * bit 2 every tile's stage-2 twiddles from column 0.  Measured and dropped (round 3):
 * non-temporal data loads and / or output stores (c5 88.3 / 91.3 / 85.2 vs 95.1-96.2 on one
 * box); the lo tile's twiddle2 prefetched by LDS-DMA and the hi tile's into registers during
 * the lo stages (bit-exact, 228 VGPRs: 104.6-105.0 vs 105.3-105.7 -- the wait moves from the
 * pairs phase to the lo phase); one output stream (X[N-k]) parked in LDS and stored during the
 * next tile's hi phase (bit-exact, 209 VGPRs, 152 KiB LDS: 103.0-103.2 vs 102.4-103.6 -- the
 * pairs phase sheds 0.7 us, the hi phase gains 2.1).  Probes: with no twiddle traffic at all c5
 * gains 2.5 % (108.3 / 107.7 vs 105.7 / 105.3): the twiddle re-reads are not what bounds the walk. */
template <int SGN, int V = 0>
__global__ __launch_bounds__(512, 2) void k_r2c_walk2(Args a, unsigned h, unsigned T, unsigned W)
{
    constexpr bool TRC = (V & 1) != 0, P_TW2 = (V & 2) != 0, P_TWS = (V & 4) != 0;
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + P * G, *cry = ltw + 504;
    double *ld = reinterpret_cast<double *>(lds); /* [0, 4096): split image / hi imag, [4096, 8192): hi real */
    /* a.tile_major (1, 2): consecutive blocks (one XCD) take the same walk segment of
     * consecutive rows, so the segment's twiddle runs and twiddle2 slice are read from that
     * XCD's L2 */
    const unsigned blk = xcd_remap(blockIdx.x), nb = (unsigned)a.batch;
    const unsigned b = a.tile_major ? blk % nb : blk / (W + 1), s = a.tile_major ? blk / nb : blk % (W + 1);
    const unsigned tid0 = threadIdx.x, B = (unsigned)a.B, N = 2 * h;
    const double2 *row = a.in + (long long)b * a.idist;
    double2 *X = a.out + (long long)b * a.odist;
    const double2 *w2t = a.saux;
    if (s == W) { /* column 0 (k = u*B pairs with (P-u)*B), as k_r2c_fused */
        const unsigned g = tid0 & 7, jt = tid0 >> 3;
        double xr[8], xi[8];
        double2 w2[7];
        r2c_load(xr, xi, w2, row, B, 0, a.tw, lds, ltw, tid0);
        r2c_stages<SGN, false>(xr, xi, w2, lds, ltw, tid0);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) lds[(jt + jj * TPG) * G + g] = make_double2(xr[jj], xi[jj]);
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, k = u * B;
            const double2 zk = make_double2(xr[jj], xi[jj]);
            if (u == 0) {
                X[0] = make_double2(zk.x + zk.y, 0.0);
                X[h] = make_double2(zk.x - zk.y, 0.0);
            } else {
                const double2 zh = lds[(P - u) * G];
                double re, im;
                r8::r2c_pair(zk, zh, w2t[k], re, im);
                X[k] = make_double2(re, im);
                X[N - k] = make_double2(re, -im);
            }
        }
        return;
    }
    const unsigned j0 = s * T, j1 = min(j0 + T, B / 16), len = j1 - j0;
    /* a.tile_major == 2: the walk starts at tile o of its segment and wraps (two chains:
     * [j0+o, j1) then [j0, j0+o)), o from the row, so the workgroups of one XCD that share a
     * segment (and its twiddles, from L2) read and write at different offsets of their rows --
     * rows lie 32 MiB apart, so equal offsets would land in the same DRAM channels */
    /* tile_major >= 3: only tile_major - 1 rotation classes, evenly spaced, so groups of
     * workgroups share a tile (and its twiddles) at the same time */
    const unsigned nrot = a.tile_major >= 3 ? (unsigned)a.tile_major - 1 : 0u;
    const unsigned o = len == 0 ? 0u
                     : a.tile_major == 2 ? (b * 7u) % len
                     : nrot ? ((b % nrot) * len) / nrot : 0u;
    R2cBuf A, Bf;
    /* phase trace (a.dbg): thread 0 sums 100 MHz ticks per phase -- [0] tile pairs, [1] hi
     * twiddles + stages, [2] lo twiddles + stages, [3] pairs + stores */
    unsigned tr1 = 0, tr2 = 0, tr3 = 0, tk = TRC ? (unsigned)__builtin_amdgcn_s_memrealtime() : 0u;
#define R2C_MARK(acc)                                                         \
    if constexpr (TRC) {                                                      \
        const unsigned tn = (unsigned)__builtin_amdgcn_s_memrealtime();       \
        acc += tn - tk;                                                       \
        tk = tn;                                                              \
    }
    r2cw2_issue<P_TWS>(A, row, B, B - 8 * (j0 + o) - 8, a.tw, tid0); /* hi of the first tile */
#pragma unroll 1
    for (unsigned jr = 0; jr < len; jr++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned g = tid & 7, jt = tid >> 3;
        const unsigned j = j0 + (o + jr) % len;
        const unsigned qlo = 8 * j + 1;
        r2cw2_issue<P_TWS>(Bf, row, B, qlo, a.tw, tid); /* lo(j) loads while hi(j) is transformed */
        double2 w2[7];
        /* ---- hi(j), in place in A */
        r2cw2_tw(A, w2, lds, ltw, tid);
        r2c_stages<SGN, false>(A.r, A.i, w2, lds, ltw, tid);
        R2C_MARK(tr1)
        double him[8];
#pragma unroll
        for (int jj = 0; jj < 8; jj++) him[jj] = A.i[jj];
        /* ---- lo(j), in place in Bf */
        r2cw2_tw(Bf, w2, lds, ltw, tid);

#pragma unroll
        for (int jj = 0; jj < 8; jj++) ld[4096 + (jt + jj * TPG) * G + g] = A.r[jj]; /* hi real parts wait here */
        {   /* the next tile's hi loads while lo(j) is transformed; unconditional (the last tile
             * reloads itself) */
            const unsigned jn = jr + 1 < len ? j0 + (o + jr + 1) % len : j;
            r2cw2_issue<P_TWS>(A, row, B, B - 8 * jn - 8, a.tw, tid);
        }
        r2c_stages<SGN, true>(Bf.r, Bf.i, w2, lds, ltw, tid);
        R2C_MARK(tr2)
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) ld[(jt + jj * TPG) * G + g] = him[jj];
        __syncthreads();
        /* ---- pairs: X[N-k], X[h-k] aligned; X[k], X[h+k] shifted one lane onto line [8j, 8j+8) */
        const bool cstart = jr == 0 || j == j0; /* a chain starts: no carry for this line */
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, k = u * B + qlo + g, hk = h - k;
            const unsigned sl = (P - 1 - u) * G + (7 - g);
            const double2 zk = make_double2(Bf.r[jj], Bf.i[jj]), zh = make_double2(ld[4096 + sl], ld[sl]);
            double re, im, re2, im2;
            const double2 wk = P_TW2 ? w2t[tid0 & 63] : w2t[k];
            const double2 whk = P_TW2 ? w2t[(tid0 & 63) + 64] : w2t[hk];
            r8::r2c_pair(zk, zh, wk, re, im);
            r8::r2c_pair(zh, zk, whk, re2, im2);
            X[N - k] = make_double2(re, -im);
            X[hk] = make_double2(re2, im2);
            const double2 va = grp_shift<-1>(make_double2(re, im)), vb = grp_shift<-1>(make_double2(re2, -im2));
            const unsigned p = u * B + 8 * j + g;
            if (g != 0) {
                X[p] = va;
                X[h + p] = vb;
            } else {
                if (!cstart) {
                    X[p] = cry[u];
                    X[h + p] = cry[512 + u];
                } else if (jr != 0 && j1 < B / 16) { /* the first chain's carry: bin 8*j1 */
                    X[u * B + 8 * j1] = cry[u];
                    X[h + u * B + 8 * j1] = cry[512 + u];
                }
                cry[u] = va;
                cry[512 + u] = vb;
            }
        }
        R2C_MARK(tr3)
    }
#undef R2C_MARK
    if (TRC && tid0 == 0) {
        unsigned *d = a.dbg + blockIdx.x * 4;
        d[0] = len;
        d[1] = tr1;
        d[2] = tr2;
        d[3] = tr3;
    }
    /* the last chain's carry: bin 8*(j0+o), or 8*j1 without rotation (at the row's last tile,
     * column B/2, already written by the aligned streams) */
    const unsigned jend = o > 0 ? j0 + o : j1;
    if (len > 0 && jend < B / 16 && (tid0 & 7) == 0) {
        const unsigned jt = tid0 >> 3;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, p = u * B + 8 * jend;
            X[p] = cry[u];
            X[h + p] = cry[512 + u];
        }
    }
}

/* ------------------------------------------------------------------ r2c split, two walks per CU
 * k_r2c_walk2's split walk (whole-line stores through the one-lane shift and the carried entry)
 * without its software pipeline, sized so that TWO workgroups share a CU (round 4): at most 128
 * VGPRs and 80 KiB of LDS -- the split image (32 KiB), the hi tile's real parts (32 KiB) and the
 * carry (16 KiB).  One tile buffer per thread; the stage-0 / stage-1 twiddle runs are read from
 * the plan's table in global memory (L2 / Infinity-Cache hits) instead of an LDS copy, the
 * stage-1 run issued behind stage 0.  A CU then overlaps one walk's loads and store drains with
 * the other walk's stages, where the one-per-CU walk serialises them in its own phase order
 * (every load issued after a store burst waits for that burst: vmcnt is in order). */
constexpr int R2CW1_LDS = (512 * 8 + 1024) * 16;

/* a run of 7 twiddles at table index idx (stage 0: B - 1 + 7q; stage 1: 8B - 1 + 7(q + B kl)) */
__device__ __forceinline__ void tw_run(double2 (&w)[7], const double2 *tw, unsigned idx)
{
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ldg(tw, (idx + i) * 16u);
}

/* r8::redistribute_tw at an explicit 7-KiB wave region */
__device__ __forceinline__ void redistribute_at(double2 (&w)[7], double2 *region)
{
    const unsigned lane = threadIdx.x & 63;
    double2 *reg = region + (lane >> 3) * 56;
#pragma unroll
    for (int j = 0; j < 7; j++) reg[(lane & 7) + 8 * j] = w[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = reg[(lane & 7) * 7 + i];
}

/* PROBE (timing probes of k_r2c_walk1, -DHSFFT_DEV_PROBES builds only; results wrong): bit 0 no
 * twiddle2 loads, bit 1 no stage twiddle loads, bit 2 no stage arithmetic (the twiddles are
 * folded in with one add each so that their loads stay), bit 3 no exchanges / redistribution,
 * bit 4 no output stores (kept behind a condition that is false at run time) */
template <int PROBE>
__device__ __forceinline__ void p_tw_run(double2 (&w)[7], const double2 *tw, unsigned idx)
{
    if constexpr (PROBE & 2) {
#pragma unroll
        for (int i = 0; i < 7; i++) w[i] = make_double2(0.5 + i, 0.25 - i);
    } else {
        tw_run(w, tw, idx);
    }
}
template <int PROBE, int SGN>
__device__ __forceinline__ void p_stage(double (&xr)[8], double (&xi)[8], const double2 (&w)[7])
{
    if constexpr (PROBE & 4) {
#pragma unroll
        for (int i = 0; i < 7; i++) {
            xr[i + 1] += w[i].x;
            xi[i + 1] += w[i].y;
        }
    } else {
        stage<8, SGN>(xr, xi, w, false);
    }
}

/* one tile's row loads */
__device__ __forceinline__ void w1_rows(double (&xr)[8], double (&xi)[8], const double2 *row, unsigned B, unsigned q0,
                                        unsigned tid)
{
    constexpr int TPG = 64;
    const unsigned g = tid & 7, jt = tid >> 3;
    const unsigned lane0 = (jt * B + q0 + g) * 16u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const double2 v = ldg(row + (size_t)i * TPG * B, lane0);
        xr[i] = v.x;
        xi[i] = v.y;
    }
}

/* one tile's row loads and its stage-0 run (registers) */
template <int PROBE = 0>
__device__ __forceinline__ void w1_load(double (&xr)[8], double (&xi)[8], double2 (&w)[7], const double2 *row,
                                        unsigned B, unsigned q0, const double2 *tw, unsigned tid)
{
    w1_rows(xr, xi, row, B, q0, tid);
    p_tw_run<PROBE>(w, tw, B - 1 + 7 * (q0 + (tid & 7)));
}

/* the tile's three stages with one twiddle run live at a time (<= 128 VGPRs with the hi tile's
 * imaginary parts alongside): stage 0 with w, the stage-1 run loaded after the first exchange,
 * the coalesced stage-2 run after the second and redistributed through the
 * image's first half (waves 0-3, then 4-7: the second half may hold the hi tile's real parts);
 * split exchanges through doubles [0, 4096) */
template <int SGN, int PROBE = 0>
__device__ __forceinline__ void w1_stages(double (&xr)[8], double (&xi)[8], double2 (&w)[7], double2 *lds,
                                          const double2 *tw, unsigned B, unsigned q0, unsigned tid0)
{
    constexpr int TPG = 64, P = 512, G = 8;
    unsigned tid = tid0;
    asm volatile("" : "+v"(tid));
    const unsigned g = tid & 7, jt = tid >> 3;
    p_stage<PROBE, SGN>(xr, xi, w);
    if constexpr (!(PROBE & 8)) r8::exchange<8, 1, 8, TPG, P, G, true>(xr, xi, lds, jt, g);
    p_tw_run<PROBE>(w, tw, 8 * B - 1 + 7 * (q0 + g + B * (jt & 7))); /* after the exchange: issued
                                                                        * earlier, its 28 VGPRs spill */
    p_stage<PROBE, SGN>(xr, xi, w);
    if constexpr (!(PROBE & 8)) r8::exchange<8, 8, 8, TPG, P, G, true>(xr, xi, lds, jt, g); /* ends with a barrier */
    if constexpr (!(PROBE & 2)) {
        r8::Args ta;
        ta.tw = tw;
        ta.B = B;
        r8::load_tw_co<64>(w, ta, (int)jt, q0);
    } else {
        p_tw_run<PROBE>(w, tw, 0);
    }
    if constexpr (!(PROBE & 8)) {
        const unsigned wave = tid0 >> 6;
        if (wave < 4) redistribute_at(w, lds + wave * 448);
        __syncthreads();
        if (wave >= 4) redistribute_at(w, lds + (wave - 4) * 448);
    }
    p_stage<PROBE, SGN>(xr, xi, w);
}

#ifdef HSFFT_DEV_PROBES
/* this workgroup's CU: XCD, shader engine, shader array and CU fields of HW_ID (< 2048) */
__device__ __forceinline__ unsigned cu_slot()
{
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   /* HW_REG_HW_ID */
    const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11)); /* HW_REG_XCC_ID */
    return ((xcc & 7) << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15);
}
#endif

/* PFH: the next tile's hi rows are loaded at the start of this tile's pairs phase, i.e. before
 * its store burst, so waiting for them does not wait for the stores (vmcnt is in order); PFL:
 * the lo rows are loaded at the start of the hi phase, while the hi tile is transformed.
 * STOK (development build, round 5 -- the test of the store-burst alignment hypothesis): the
 * two walks a CU holds never have store bursts in flight together.  A per-CU token word
 * (a.dbg[cu_slot()], zero when free) is taken by thread 0 before the pairs phase and returned
 * once the phase's stores have drained (1) or once they are issued (2); the wait is bounded
 * (50 us, about one tile pair), after which the walk stores without the token */
template <int SGN, bool PFH = false, bool PFL = false, int PROBE = 0, int STOK = 0>
__global__ __launch_bounds__(512, 4) void k_r2c_walk1(Args a, unsigned h, unsigned T, unsigned W)
{
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *cry = lds + P * G;
    double *ld = reinterpret_cast<double *>(lds); /* [0, 4096): split image / hi imag, [4096, 8192): hi real */
    const unsigned blk = xcd_remap(blockIdx.x), nb = (unsigned)a.batch;
    const unsigned b = a.tile_major ? blk % nb : blk / (W + 1), s = a.tile_major ? blk / nb : blk % (W + 1);
    const unsigned tid0 = threadIdx.x, B = (unsigned)a.B, N = 2 * h;
    const double2 *row = a.in + (long long)b * a.idist;
    double2 *X = a.out + (long long)b * a.odist;
    const double2 *w2t = a.saux;
    if (s == W) { /* column 0 (k = u*B pairs with (P-u)*B), as k_r2c_fused (LDS: image + 8 KiB runs) */
        double2 *ltw = lds + P * G;
        const unsigned g = tid0 & 7, jt = tid0 >> 3;
        double xr[8], xi[8];
        double2 w2[7];
        r2c_load(xr, xi, w2, row, B, 0, a.tw, lds, ltw, tid0);
        r2c_stages<SGN, false>(xr, xi, w2, lds, ltw, tid0);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) lds[(jt + jj * TPG) * G + g] = make_double2(xr[jj], xi[jj]);
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, k = u * B;
            const double2 zk = make_double2(xr[jj], xi[jj]);
            if (u == 0) {
                X[0] = make_double2(zk.x + zk.y, 0.0);
                X[h] = make_double2(zk.x - zk.y, 0.0);
            } else {
                const double2 zh = lds[(P - u) * G];
                double re, im;
                r8::r2c_pair(zk, zh, w2t[k], re, im);
                X[k] = make_double2(re, im);
                X[N - k] = make_double2(re, -im);
            }
        }
        return;
    }
    /* walk segment, rotation and carry chains exactly as k_r2c_walk2 */
    const unsigned j0 = s * T, j1 = min(j0 + T, B / 16), len = j1 - j0;
    const unsigned nrot = a.tile_major >= 3 ? (unsigned)a.tile_major - 1 : 0u;
    const unsigned o = len == 0 ? 0u
                     : a.tile_major == 2 ? (b * 7u) % len
                     : nrot ? ((b % nrot) * len) / nrot : 0u;
    double pr[8], pi[8]; /* PFH: the next hi tile's rows */
    if constexpr (PFH)
        if (len > 0) w1_rows(pr, pi, row, B, B - 8 * (j0 + o) - 8, tid0);
#pragma unroll 1
    for (unsigned jr = 0; jr < len; jr++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned g = tid & 7, jt = tid >> 3;
        const unsigned j = j0 + (o + jr) % len;
        const unsigned qlo = 8 * j + 1, qhi = B - 8 * j - 8;
        double xr[8], xi[8], him[8];
        double2 w[7];
        /* ---- hi(j) */
        if constexpr (PFH) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                xr[i] = pr[i];
                xi[i] = pi[i];
            }
            p_tw_run<PROBE>(w, a.tw, B - 1 + 7 * (qhi + g));
        } else {
            w1_load<PROBE>(xr, xi, w, row, B, qhi, a.tw, tid);
        }
        double lr[8], li[8]; /* PFL: the lo tile's rows */
        if constexpr (PFL) w1_rows(lr, li, row, B, qlo, tid);
        __syncthreads(); /* the previous pairs phase has read the image */
        w1_stages<SGN, PROBE>(xr, xi, w, lds, a.tw, B, qhi, tid);
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            ld[4096 + (jt + jj * TPG) * G + g] = xr[jj]; /* hi real parts wait in the image's second half */
            him[jj] = xi[jj];
        }
        /* ---- lo(j) */
        if constexpr (PFL) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                xr[i] = lr[i];
                xi[i] = li[i];
            }
            p_tw_run<PROBE>(w, a.tw, B - 1 + 7 * (qlo + g));
        } else {
            w1_load<PROBE>(xr, xi, w, row, B, qlo, a.tw, tid);
        }
        __syncthreads(); /* every wave's hi stage-2 twiddles are read back from the image */
        w1_stages<SGN, PROBE>(xr, xi, w, lds, a.tw, B, qlo, tid);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) ld[(jt + jj * TPG) * G + g] = him[jj];
        __syncthreads();
        /* ---- pairs: X[N-k], X[h-k] aligned; X[k], X[h+k] shifted one lane onto line [8j, 8j+8) */
#ifdef HSFFT_DEV_PROBES
        bool own = false;
        unsigned *tok = nullptr;
        if constexpr (STOK != 0) {
            tok = a.dbg + cu_slot();
            if (tid0 == 0) {
                const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
                unsigned tries = 0;
                for (;; tries++) {
                    if (atomicCAS(tok, 0u, blockIdx.x + 1u) == 0u) {
                        own = true;
                        break;
                    }
                    if ((unsigned)__builtin_amdgcn_s_memrealtime() - t0 > 5000u) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                /* statistics after the 2048 token words: pairs phases, phases that waited, timeouts,
                 * 10-ns ticks waited */
                if (a.tiles_q) {
                    atomicAdd(a.dbg + 2048, 1u);
                    if (tries) {
                        atomicAdd(a.dbg + 2049, 1u);
                        atomicAdd(a.dbg + 2051, (unsigned)__builtin_amdgcn_s_memrealtime() - t0);
                    }
                    if (!own) atomicAdd(a.dbg + 2050, 1u);
                }
            }
            __syncthreads();
        }
#endif
        if constexpr (PFH) { /* unconditional: the last tile reloads itself */
            const unsigned jn = jr + 1 < len ? j0 + (o + jr + 1) % len : j;
            w1_rows(pr, pi, row, B, B - 8 * jn - 8, tid);
        }
        const bool cstart = jr == 0 || j == j0;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, k = u * B + qlo + g, hk = h - k;
            const unsigned sl = (P - 1 - u) * G + (7 - g);
            const double2 zk = make_double2(xr[jj], xi[jj]), zh = make_double2(ld[4096 + sl], ld[sl]);
            double re, im, re2, im2;
            const double2 wk = (PROBE & 1) ? make_double2(0.5, 0.25) : w2t[k];
            const double2 whk = (PROBE & 1) ? make_double2(0.25, 0.5) : w2t[hk];
            r8::r2c_pair(zk, zh, wk, re, im);
            r8::r2c_pair(zh, zk, whk, re2, im2);
            const bool st = !(PROBE & 16) || h == 0; /* h > 0 always: the probe stores nothing */
            if (st) {
                X[N - k] = make_double2(re, -im);
                X[hk] = make_double2(re2, im2);
            }
            const double2 va = grp_shift<-1>(make_double2(re, im)), vb = grp_shift<-1>(make_double2(re2, -im2));
            const unsigned p = u * B + 8 * j + g;
            if (g != 0) {
                if (st) {
                    X[p] = va;
                    X[h + p] = vb;
                }
            } else {
                if (!cstart && st) {
                    X[p] = cry[u];
                    X[h + p] = cry[512 + u];
                } else if (jr != 0 && j1 < B / 16) { /* the first chain's carry: bin 8*j1 */
                    X[u * B + 8 * j1] = cry[u];
                    X[h + u * B + 8 * j1] = cry[512 + u];
                }
                cry[u] = va;
                cry[512 + u] = vb;
            }
        }
#ifdef HSFFT_DEV_PROBES
        if constexpr (STOK != 0) {
            if constexpr (STOK == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid0 == 0 && own) atomicCAS(tok, blockIdx.x + 1u, 0u);
        }
#endif
    }
    const unsigned jend = o > 0 ? j0 + o : j1;
    if (len > 0 && jend < B / 16 && (tid0 & 7) == 0) {
        const unsigned jt = tid0 >> 3;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const unsigned u = jt + jj * TPG, p = u * B + 8 * jend;
            X[p] = cry[u];
            X[h + p] = cry[512 + u];
        }
    }
}

inline int env(const char *name, int dflt);

/* returns 1 if not applicable, 0 on launch, < 0 on error */
inline int launch_r2c_fused(const void *Z, long long zdist, void *X, long long xdist, const void *tw, const void *w2,
                            long long h, long long B, int batch, int sgn, hipStream_t st, bool compact = false)
{
    if (B % 16 || B * 512 != h || h > 0x40000000LL || (sgn != 1 && sgn != -1)) return 1;
    Args a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)Z;
    a.out = (double2 *)X;
    a.tw = (const double2 *)tw;
    a.saux = (const double2 *)w2;
    a.idist = zdist;
    a.odist = xdist;
    a.A = 1;
    a.B = B;
    a.batch = batch;
    a.tiles = a.tiles_q = B / 16 + 1;
    /* default: k_r2c_walk2, walks of 8 tile pairs, segment-major, the walk start of row b at
     * tile b % 8 (HSFFT_R2C_ORDER=9: 8 rotation classes).  Interleaved on one box (two passes
     * each, GSamples/s): 105.8 / 105.8 vs 103.5-104.3 for the (b*7) % 16 rotation with walks of
     * 16 (ORDER=2), 99.7-99.8 row-major with walks of 32 (0), 98.4-98.8 with 4 classes and 94.3-94.7
     * with 2 (ORDER=5, 3: FETCH 32.3 / 29.3 GB per 512 rows, the twiddles mostly from L2, yet
     * slower: workgroups that read the same lines at the same time contend); plain
     * segment-major (1) 88.7-90.8 elsewhere; HSFFT_R2C_WALK=0 (and the compact layout):
     * k_r2c_fused */
    /* default (round 4): k_r2c_walk1 -- two walks per CU, walks of 32 tile pairs, 8 rotation
     * classes; in-process A/B per 512 rows against k_r2c_walk2 (walks of 8): 20.40 vs 20.31 ms on a
     * fast-write allocation, 20.97 vs 22.20 on a medium one, 22.25-23.60 vs 24.23-25.77 on three
     * slow ones (profiles/r04d-f_*).  HSFFT_R2C_WALK=2: walk2; 0: k_r2c_fused */
    /* product: k_r2c_walk1 (default) or, HSFFT_R2C_WALK=0, k_r2c_fused -- the independent
     * schedule the every-word test compares against, and the compact layout's kernel.  The
     * measured-slower walks (k_r2c_walk2, walk1's other prefetch forms, the other walk orders,
     * the phase trace) are compiled only into the development build (-DHSFFT_DEV_PROBES) */
    const int walk = env("HSFFT_R2C_WALK", 3) != 0 ? 3 : 0;
    if (!compact && walk != 0) {
#ifdef HSFFT_DEV_PROBES
        const bool w2 = env("HSFFT_R2C_WALK", 3) == 2 || env("HSFFT_R2C_DEBUG", 0) != 0;
        const int wt_dflt = w2 ? 8 : 32;
#else
        const int wt_dflt = 32;
#endif
        const long long T = env("HSFFT_R2C_WT", wt_dflt) > 0 ? env("HSFFT_R2C_WT", wt_dflt) : wt_dflt,
                        W = (B / 16 + T - 1) / T;
        const long long grid = (W + 1) * (long long)batch;
        if (grid <= 0 || grid > 0x7fffffffLL) return -1;
        typedef void (*wfn)(Args, unsigned, unsigned, unsigned);
        /* k_r2c_walk1<SGN, PFH = true>: the next hi tile's rows loaded before the pairs phase's
         * stores, 20.00 vs 20.15 ms per 512 rows in-process (profiles/r04i_i_c5.txt) */
        wfn fw = sgn == 1 ? k_r2c_walk1<1, true> : k_r2c_walk1<-1, true>;
        int lds_bytes = R2CW1_LDS;
        a.tile_major = 9; /* 8 rotation classes */
        bool dbg = false, stok_stats = false;
#ifdef HSFFT_DEV_PROBES
        {
            /* development build: HSFFT_R2C_WALK=2 k_r2c_walk2 (round 3's one-per-CU walk, walks of
             * 8 by default); HSFFT_R2C_DEBUG=1 its phase trace; HSFFT_R2C_PROBE (timing only, results
             * wrong): 1 no twiddle2 traffic, 2 no stage-2 twiddle traffic, 3 neither */
            dbg = env("HSFFT_R2C_DEBUG", 0) != 0;
            if (w2) {
                static const wfn fws[2][8] = {
                    {k_r2c_walk2<1, 0>, k_r2c_walk2<1, 1>, k_r2c_walk2<1, 2>, k_r2c_walk2<1, 3>, k_r2c_walk2<1, 4>,
                     k_r2c_walk2<1, 5>, k_r2c_walk2<1, 6>, k_r2c_walk2<1, 7>},
                    {k_r2c_walk2<-1, 0>, k_r2c_walk2<-1, 1>, k_r2c_walk2<-1, 2>, k_r2c_walk2<-1, 3>, k_r2c_walk2<-1, 4>,
                     k_r2c_walk2<-1, 5>, k_r2c_walk2<-1, 6>, k_r2c_walk2<-1, 7>}};
                fw = fws[sgn == 1 ? 0 : 1][(dbg ? 1 : 0) | (env("HSFFT_R2C_PROBE", 0) & 3) << 1];
                lds_bytes = R2CW2_LDS;
            } else {
                /* walk1's other prefetch forms: HSFFT_R2C_PFH 0 none, 2 the lo rows with the hi phase,
                 * 3 both (20.11 vs 20.00 ms, profiles/r04i_i_c5.txt) */
                switch (env("HSFFT_R2C_PFH", 1)) {
                case 0: fw = sgn == 1 ? k_r2c_walk1<1> : k_r2c_walk1<-1>; break;
                case 2: fw = sgn == 1 ? k_r2c_walk1<1, false, true> : k_r2c_walk1<-1, false, true>; break;
                case 3: fw = sgn == 1 ? k_r2c_walk1<1, true, true> : k_r2c_walk1<-1, true, true>; break;
                default: break;
                }
                /* HSFFT_R2C_W1PROBE (timing only, results wrong; the default PFH walk, sgn 1): see PROBE */
                switch (sgn == 1 ? env("HSFFT_R2C_W1PROBE", 0) : 0) {
                case 3: fw = k_r2c_walk1<1, true, false, 3>; break;
                case 4: fw = k_r2c_walk1<1, true, false, 4>; break;
                case 8: fw = k_r2c_walk1<1, true, false, 8>; break;
                case 12: fw = k_r2c_walk1<1, true, false, 12>; break;
                case 15: fw = k_r2c_walk1<1, true, false, 15>; break;
                case 16: fw = k_r2c_walk1<1, true, false, 16>; break;
                case 31: fw = k_r2c_walk1<1, true, false, 31>; break;
                default: break;
                }
                /* HSFFT_R2C_STOK 1 / 2: the per-CU store token (see k_r2c_walk1), bit-exact */
                const int stok = env("HSFFT_R2C_STOK", 0);
                if (stok == 1 || stok == 2) {
                    static unsigned *s_tok = nullptr;
                    if (!s_tok) {
                        HCHK(hipMalloc((void **)&s_tok, 2052 * sizeof(unsigned)));
                        HCHK(hipMemset(s_tok, 0, 2052 * sizeof(unsigned)));
                    }
                    a.dbg = s_tok;
                    stok_stats = env("HSFFT_R2C_STOK_STATS", 0) != 0;
                    a.tiles_q = stok_stats ? 1 : 0; /* walk1 does not read tiles_q otherwise */
                    fw = stok == 1 ? (sgn == 1 ? k_r2c_walk1<1, true, false, 0, 1> : k_r2c_walk1<-1, true, false, 0, 1>)
                                   : (sgn == 1 ? k_r2c_walk1<1, true, false, 0, 2> : k_r2c_walk1<-1, true, false, 0, 2>);
                }
            }
            /* walk orders: 0 row-major, 1 segment-major, 2 rotated, >= 3 rotation classes */
            a.tile_major = env("HSFFT_R2C_ORDER", 9);
        }
#endif
        static unsigned *s_dbg = nullptr;
        static long long s_dbg_n = 0;
        if (dbg) {
            if (s_dbg_n < grid) {
                if (s_dbg) HCHK(hipFree(s_dbg));
                HCHK(hipMalloc((void **)&s_dbg, (size_t)grid * 4 * sizeof(unsigned)));
                s_dbg_n = grid;
            }
            HCHK(hipMemsetAsync(s_dbg, 0, (size_t)grid * 4 * sizeof(unsigned), st));
            a.dbg = s_dbg;
        }
        HCHK(hipFuncSetAttribute((const void *)fw, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
        hipLaunchKernelGGL(fw, dim3((unsigned)grid), dim3(512), lds_bytes, st, a, (unsigned)h, (unsigned)T, (unsigned)W);
        HCHK(hipGetLastError());
        if (stok_stats) { /* development build: the store token's statistics of this launch */
            unsigned hs[4];
            HCHK(hipMemcpyAsync(hs, a.dbg + 2048, sizeof hs, hipMemcpyDeviceToHost, st));
            HCHK(hipStreamSynchronize(st));
            HCHK(hipMemsetAsync(a.dbg + 2048, 0, sizeof hs, st));
            fprintf(stderr, "r2c store token: %u pairs phases, %u waited (mean %.2f us), %u timed out\n", hs[0], hs[1],
                    hs[1] ? hs[3] / 100.0 / hs[1] : 0.0, hs[2]);
        }
        if (dbg) { /* mean us per tile pair of the walking workgroups */
            unsigned *hb = (unsigned *)malloc((size_t)grid * 4 * sizeof(unsigned));
            if (!hb) return -1;
            HCHK(hipMemcpyAsync(hb, s_dbg, (size_t)grid * 4 * sizeof(unsigned), hipMemcpyDeviceToHost, st));
            HCHK(hipStreamSynchronize(st));
            double t[4] = {0, 0, 0, 0};
            for (long long w = 0; w < grid; w++)
                for (int i = 0; i < 4; i++) t[i] += hb[w * 4 + i];
            free(hb);
            const double n = t[0] > 0 ? t[0] : 1;
            fprintf(stderr, "r2c_walk2: tile pairs %.0f  us per tile pair: hi %.2f lo %.2f pairs+stores %.2f\n", t[0],
                    t[1] / n / 100.0, t[2] / n / 100.0, t[3] / n / 100.0);
        }
        return 0;
    }
    const long long grid = a.tiles * (long long)batch;
    if (grid <= 0 || grid > 0x7fffffffLL) return -1;
    const size_t lds = (size_t)(512 * 8 + 504) * sizeof(double2);
    void (*fn)(Args, unsigned) = compact ? (sgn == 1 ? k_r2c_fused<1, true> : k_r2c_fused<-1, true>)
                                         : (sgn == 1 ? k_r2c_fused<1, false> : k_r2c_fused<-1, false>);
    HCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(512), lds, st, a, (unsigned)h);
    HCHK(hipGetLastError());
    return 0;
}

/* ------------------------------------------------------------------ host side */
typedef void (*kfn)(Args);

inline int env(const char *name, int dflt)
{
    const char *s = hs_getenv(name); /* getenv, or the small path's per-call snapshot */
    return s ? atoi(s) : dflt;
}

template <int T>
inline kfn b512_fn(int sgn, int conj)
{
    if (sgn == 1) return conj ? k_b512<T, 1, true> : k_b512<T, 1, false>;
    return conj ? k_b512<T, -1, true> : k_b512<T, -1, false>;
}

/* the pipelined kernel for this pass, or nullptr (then hsfft_pass_r8.h's k_pass runs) */
inline kfn pick(const hsd_pass *p, const hsd_launch *l, int *G, int *TL, int *threads, size_t *lds)
{
    /* bit0: first pass (26.9 vs 28.0 ms per 4096 x 2^20), bit1: later [8,8,8] pass (23.2-23.9
     * vs 23.5-24.2 ms for k_pass_b512 over five paired runs) */
    const int mask = env("HSFFT_PF", 3);
    if (l->load_op != HS_LOAD_PLAIN || l->store_op != HS_STORE_PLAIN) return nullptr;
    if (l->sgn != 1 && l->sgn != -1) return nullptr;
    for (int s = 1; s < p->nst; s++)
        if (p->radix[s] != 8) return nullptr;
    if ((mask & 1) && p->B == 1 && p->leaf && p->nst == 4 && p->radix[0] == 4) { /* 2^20's pass A: [4,8,8,8] */
        /* k_firstq: 24.0-24.3 ms per 4096 x 2^20 against 27.0-27.2 for its 32-B-segment
         * predecessor k_first (round 1; removed in round 3).  One column group per workgroup
         * (HSFFT_PFQ, default 1 since round 4): in-process 46.19 / 45.86 vs 46.49 / 46.06 ms per
         * step for walks of 4 groups on two boxes, walks of 2 47.17 (profiles/r04aa_*, r04ab_*) */
        if (p->A % 4 == 0) { /* 64-B loads: *G = 4 columns per tile for the grid */
            *G = 4;
            *TL = env("HSFFT_PFQ", 1) > 0 ? env("HSFFT_PFQ", 1) : 1;
            *threads = 512;
            *lds = (size_t)2048 * 2 * sizeof(double) + 2048 * sizeof(double2);
            /* non-temporal output stores (HSFFT_PFA_NT bit 1, default on since round 4): 48.42 vs
             * 49.48 ms per 4096 x 2^20 in-process (profiles/r04i_i_c2_nt.txt) */
            if ((env("HSFFT_PFA_NT", 3) & 2) && !l->conj)
                return l->sgn == 1 ? k_firstq<4, 3, 2, 1, false, true> : k_firstq<4, 3, 2, -1, false, true>;
            if (l->sgn == 1) return l->conj ? k_firstq<4, 3, 2, 1, true> : k_firstq<4, 3, 2, 1, false>;
            return l->conj ? k_firstq<4, 3, 2, -1, true> : k_firstq<4, 3, 2, -1, false>;
        }
        return nullptr;
    }
    if ((mask & 1) && p->B == 1 && p->leaf && p->nst == 4 && p->radix[0] == 8 && p->A % 2 == 0) {
        /* [8,8,8,8] first pass (2^21 = r2c 2^22's inner pass A): 32-B paired loads, one column
         * per thread group, L = 512 twiddles from global memory; one column group per workgroup
         * (HSFFT_PFP, default 1 since round 4): c5 21.89 / 20.84 vs 22.01 / 21.04 ms per 512 rows
         * for walks of 4 on two boxes, walks of 2 22.69 (profiles/r04aa_*, r04ab_*) */
        const int q = env("HSFFT_PFP", 1);
        if (q > 0) {
            *G = 2; /* columns per tile group, for the grid */
            *TL = q;
            *threads = 512;
            *lds = (size_t)4096 * sizeof(double) + 511 * sizeof(double2);
            /* non-temporal output stores (HSFFT_PFA_NT bit 0, default on): the 8 MiB of output an
             * XCD's 64 workgroups write per column group no longer evict the input lines their
             * neighbours still have to read -- FETCH -17 %, pass A 7.29 -> 7.01 ms per 512 rows,
             * c5 21.44 -> 21.12 ms (profiles/r04g_*) */
            if ((env("HSFFT_PFA_NT", 3) & 1) && !l->conj)
                return l->sgn == 1 ? k_firstq<8, 3, 1, 1, false, true> : k_firstq<8, 3, 1, -1, false, true>;
            if (l->sgn == 1) return l->conj ? k_firstq<8, 3, 1, 1, true> : k_firstq<8, 3, 1, 1, false>;
            return l->conj ? k_firstq<8, 3, 1, -1, true> : k_firstq<8, 3, 1, -1, false>;
        }
    }
    if ((mask & 2) && p->B > 1 && p->nst == 3 && p->radix[0] == 8 && p->A == 1 && p->B % 8 == 0) {
        /* rows per workgroup: the tile's twiddles (64 KiB) are read once per TL rows (512 KiB
         * of data at TL = 8: 12.5 % over-read; 16: 6 %, 32: 3 %) */
        const int t = env("HSFFT_PFB", 8);
        *TL = t >= 32 ? 32 : t >= 16 ? 16 : t >= 8 ? 8 : t >= 4 ? 4 : 2;
        *G = 8;
        *threads = 512;
        *lds = (size_t)(512 * 8 + 504) * sizeof(double2);
        switch (*TL) {
        case 32: return b512_fn<32>(l->sgn, l->conj);
        case 16: return b512_fn<16>(l->sgn, l->conj);
        case 8: return b512_fn<8>(l->sgn, l->conj);
        case 4: return b512_fn<4>(l->sgn, l->conj);
        default: return b512_fn<2>(l->sgn, l->conj);
        }
    }
    return nullptr;
}

/* returns 1 if no pipelined kernel applies, 0 on launch, < 0 on error */
inline int launch(const hsd_pass *p, const hsd_launch *l, hipStream_t st)
{
    int G = 0, TL = 0, threads = 0;
    size_t lds = 0;
    kfn fn = pick(p, l, &G, &TL, &threads, &lds);
    if (!fn) return 1;
#ifdef HSFFT_DEV_PROBES
    {
        const unsigned m = env("HSFFT_PFA_PROBE", 0) ? 7u : 0xffffffffu;
        HCHK(hipMemcpyToSymbol(HIP_SYMBOL(pf_probe_twmask), &m, sizeof m));
    }
#endif
    Args a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)l->in;
    a.out = (double2 *)l->out;
    a.tw = (const double2 *)l->tw;
    a.idist = l->idist;
    a.odist = l->odist;
    a.A = p->A;
    a.B = p->B;
    a.sgn = l->sgn;
    a.dir = l->dir;
    a.conj = l->conj;
    a.xcd_groups = env("HSFFT_XCD", 1);
    a.batch = l->batch;
    long long grid;
    if (p->B == 1) {
        const long long ntiles = p->A / G, groups = (ntiles + TL - 1) / TL;
        a.tiles_q = groups;
        a.tiles = groups;
        grid = groups * l->batch;
    } else {
        a.tiles = p->B / 8;
        a.tiles_q = a.tiles;
        grid = a.tiles * ((l->batch + TL - 1) / TL);
    }
    if (grid <= 0 || grid > 0x7fffffffLL) {
        snprintf(g_err, sizeof g_err, "pf: bad grid %lld", grid);
        return -1;
    }
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return set_err(e, "hipFuncSetAttribute");
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(threads), lds, st, a);
    HCHK(hipGetLastError());
    return 0;
}

}  // namespace pf
