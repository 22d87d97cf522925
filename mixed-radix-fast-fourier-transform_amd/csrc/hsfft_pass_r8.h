/*
 * hsfft_pass_r8.h -- register-resident Stockham passes for power-of-two radix lists
 * (radix 2/4 first, then radix 8): the hot path of BASELINE configs 2 (2^20 = [4,8^6]),
 * 4 (Bluestein M = 2^18 = [8^6]) and 5 (r2c inner 2^21 = [8^7]).
 *
 * One workgroup transforms G groups (G = WM x WQ tile of (m, q) pairs, hsfft_internal.h) of
 * P = R0 * 8^N8 points.  Every thread owns 8 points of one group in registers for every
 * stage (8/R butterflies of radix R); stages hand data over through one LDS image
 * (index p*G + g), so the only global traffic is the pass's input read and output write
 * plus the plan's twiddles.  Index arithmetic is compile-time (shifts / masks).
 *
 * Arithmetic is the reference's (butterflies in hsfft_butterfly.h, twiddles from the plan's
 * own table, -ffp-contract=off), so the results are bit-identical to the generic kernel.
 */
#pragma once

namespace r8 {

struct Args {
    const double2 *in;
    double2 *out;
    const double2 *tw;
    const double2 *laux, *saux;
    long long idist, odist, A, B, nsig, tiles_q, tiles;
    int sgn, dir, conj, load_op, store_op;
    int xcd_groups;   /* >0: remap block ids so that consecutive tiles share an XCD */
    int tile_major;   /* 1: block order tile-major (all rows of a tile adjacent) */
    long long batch;
    unsigned *dbg;    /* optional per-workgroup phase trace (k_r2c_walk2, HSFFT_R2C_DEBUG) */
    unsigned *done;   /* k_pass launched as one workgroup: host completion word (hsd_launch) */
    unsigned done_val;
};

template <int N>
struct ilog2 {
    static constexpr int v = 1 + ilog2<N / 2>::v;
};
template <>
struct ilog2<1> {
    static constexpr int v = 0;
};

template <int R0, int N8>
struct Shape {
    static constexpr int NST = 1 + N8;
    static constexpr int P = R0 * (N8 >= 1 ? 8 : 1) * (N8 >= 2 ? 8 : 1) * (N8 >= 3 ? 8 : 1) * (N8 >= 4 ? 8 : 1);
    static constexpr int TPG = P / 8;
    /* radix and local L of stage s */
    static constexpr int R(int s) { return s == 0 ? R0 : 8; }
    static constexpr int Lloc(int s) { return s == 0 ? 1 : R0 * (s >= 2 ? 8 : 1) * (s >= 3 ? 8 : 1) * (s >= 4 ? 8 : 1); }
};

/* Twiddles of one stage for this thread's 8/R butterflies: tw[L-1 + (R-1)*k + i-1] with
 * k = q + B*kloc (ref :731-741 and the per-radix combine loops).  Loaded one stage ahead of
 * their use so the (L2/Infinity-Cache) latency overlaps the previous stage's work. */
template <int R, int LLOC, int TPG>
__device__ __forceinline__ void load_tw(double2 (&w)[7], const Args &a, int jt, long long q, bool valid)
{
    constexpr int NB = 8 / R;
    const long long L = a.B * LLOC;
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int kloc = (c * TPG + jt) & (LLOC - 1);
        /* invalid lanes read column 0 (always in range): no branch around the loads, which
         * would make hipcc wait vmcnt(0) after each one */
        const long long k = valid ? q + a.B * kloc : 0;
        const double2 *p = a.tw + (L - 1 + (long long)(R - 1) * k);
#pragma unroll
        for (int i = 1; i < R; i++) w[c * (R - 1) + i - 1] = p[i - 1];
    }
}

/* Coalesced twiddle staging for radix-8 stages with LLOC >= 8 in tiles of 8 q-columns
 * (G == WQ == 8): the 8 lanes of kloc-row r of a wave need the contiguous run
 * tw[L-1 + 7*(q0 + B*kloc) + 0..55]; lane l loads entries (l&7) + 8j (8 cache lines per
 * instruction instead of ~56 for the per-lane gather), then the run is redistributed
 * through the wave's own 7 KiB of the (idle) LDS image so that lane (g, r) gets entries
 * 7g..7g+6. */
template <int LLOC>
__device__ __forceinline__ void load_tw_co(double2 (&w)[7], const Args &a, int jt, long long q0)
{
    const int lane = threadIdx.x & 63;
    const int kloc = jt & (LLOC - 1); /* lane (g, jt): jt is the run's row, g picks entries */
    const long long base = a.B * LLOC - 1 + 7 * (q0 + a.B * kloc);
#pragma unroll
    for (int j = 0; j < 7; j++) w[j] = a.tw[base + (lane & 7) + 8 * j];
}

__device__ __forceinline__ void redistribute_tw(double2 (&w)[7], double2 *lds)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *reg = lds + wave * 448 + (lane >> 3) * 56;
#pragma unroll
    for (int j = 0; j < 7; j++) reg[(lane & 7) + 8 * j] = w[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = reg[(lane & 7) * 7 + i];
}

/* apply the stage's twiddles (unless this is the leaf) and the 8/R butterflies */
template <int R, int LLOC, int TPG>
__device__ __forceinline__ void do_stage(double (&xr)[8], double (&xi)[8], const double2 (&w)[7], const Args &a,
                                         int jt, long long q, bool leaf)
{
    constexpr int NB = 8 / R;
#pragma unroll
    for (int c = 0; c < NB; c++) {
        if (!leaf) {
            const int kloc = (c * TPG + jt) & (LLOC - 1);
            /* radix-4 combine skips the k == 0 column (ref :826-855); 2 and 8 never skip */
            const bool skip = R == 4 && q == 0 && kloc == 0;
            if (!skip) {
#pragma unroll
                for (int i = 1; i < R; i++) {
                    const double2 t = w[c * (R - 1) + i - 1];
                    hsb::twmul(xr[c * R + i], xi[c * R + i], t.x, a.conj ? -t.y : t.y);
                }
            }
        }
        hsb::bfly<R>(&xr[c * R], &xi[c * R], a.sgn, leaf);
    }
}

/* stage s outputs -> LDS -> stage s+1 inputs.  SPLIT exchanges the real parts, then the
 * imaginary parts, through a P*G-double image (half the LDS, so twice the workgroups per CU). */
/* LDS slot of point p: an XOR swizzle of p's low bits with higher bits (a bijection on
 * [0, P), applied by the writes and the reads of the same exchange), chosen per exchange shape
 * so that the wave's stores hit distinct banks.
 *  - 16-B exchanges (double2 per point): after a leaf stage (LLOC == 1) consecutive butterflies
 *    write R points apart; with fewer than 8 groups per 128-B bank window that is an R-way
 *    conflict, so p ^= (p / R) & (R - 1).
 *  - split exchanges (8-B doubles, real then imaginary parts), after a leaf stage only:
 *    p ^= (p >> s) & (R - 1) with s per (R, G), found with a bank model of ds_write_b64 (4
 *    groups of 16 lanes, 32 banks) and ds_read_b64 (2 groups of 32 lanes, 64 banks): the first
 *    exchange of the [4,8,8,8] first pass (G = 2, c2's pass A) goes from 8 to 4 cycles per store
 *    instruction (conflict-free), that of [8,8,8,8] (G = 1, c5's pass A) from 8 to 4; the reads
 *    stay conflict-free (round 2's swizzle: s = log2 R). */
struct Swz {
    int t, k, s;
};

constexpr int swz_log2(int x) { return x <= 1 ? 0 : 1 + swz_log2(x / 2); }

constexpr Swz split_swz(int R, int LLOC, int G)
{
    /* write groups of 16 lanes cover 16 / G butterflies; their R outputs jj sit LLOC apart */
    const int lg = G == 1 ? 0 : G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : -1;
    if (lg < 0 || R < 2) return {0, 0, 0};
    if (LLOC == 1) { /* XOR the jj bits with the butterfly index bits above the bank window */
        const int k = swz_log2(R);
        return {0, k, (4 - lg) > k ? 4 - lg : k};
    }
    /* later exchanges (LLOC > 1) keep the identity: a swizzle there has to XOR the jj bits of
     * the write address with the butterfly's ml bits, which turns the eight constant store
     * offsets into per-jj address arithmetic -- the bank model says the [4,8,8,8] / [8,8,8,8]
     * second exchanges would go from 8 to 4 cycles per store, but hipcc then spills 4-7 dwords
     * in pf::k_firstq (measured in the code object), so it is not used */
    return {0, 0, 0};
}

template <int R, int LLOC, int G, bool SPLIT = false>
__device__ __forceinline__ unsigned lds_slot(unsigned p)
{
#ifndef HSFFT_SPLIT_SWZ_R2 /* (experiment builds: -DHSFFT_SPLIT_SWZ_R2 keeps round 2's swizzle) */
    if constexpr (SPLIT) {
        constexpr Swz z = split_swz(R, LLOC, G);
        if constexpr (z.k > 0) return p ^ (((p >> z.s) & ((1u << z.k) - 1u)) << z.t);
        return p;
    } else
#endif
    {
        if constexpr (LLOC == 1 && G < 8 && R > 1) return p ^ ((p / R) & (R - 1));
        return p;
    }
}

/* Materialise LDS-loaded values before the barrier that follows their loads.  Without it
 * hipcc (ROCm 7.2) may sink a ds_read whose only uses lie after the barrier to those uses,
 * i.e. past the barrier: the next exchange's writes from faster waves then race with it
 * (observed: k_pass<4,3,1,1> / <8,3,1,1> lost whole columns).  The empty asm "uses" each
 * value where it stands and emits no instruction. */
__device__ __forceinline__ void pin(double (&x)[8])
{
#pragma unroll
    for (int i = 0; i < 8; i++) asm volatile("" : "+v"(x[i]));
}

template <int R, int LLOC, int R2, int TPG, int P, int G, bool SPLIT>
__device__ __forceinline__ void exchange(double (&xr)[8], double (&xi)[8], double2 *lds, unsigned jt, unsigned g)
{
    /* unsigned index math throughout: signed / and % by powers of two cost sign fix-ups */
    constexpr int NB = 8 / R, NB2 = 8 / R2, L2 = LLOC * R, S2 = P / (L2 * R2);
    if constexpr (!SPLIT) {
#pragma unroll
        for (int c = 0; c < NB; c++) {
            const unsigned b = c * TPG + jt;
            const unsigned kloc = b & (LLOC - 1), ml = b / LLOC;
#pragma unroll
            for (int jj = 0; jj < R; jj++) {
                const unsigned p = lds_slot<R, LLOC, G>(ml * LLOC * R + kloc + jj * LLOC);
                lds[p * G + g] = make_double2(xr[c * R + jj], xi[c * R + jj]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NB2; c++) {
            const unsigned b = c * TPG + jt;
            const unsigned kloc = b & (L2 - 1), ml = b / L2;
#pragma unroll
            for (int i = 0; i < R2; i++) {
                const unsigned p = lds_slot<R, LLOC, G>((ml + i * S2) * L2 + kloc);
                const double2 v = lds[p * G + g];
                xr[c * R2 + i] = v.x;
                xi[c * R2 + i] = v.y;
            }
        }
        pin(xr);
        pin(xi);
        __syncthreads();
    } else {
        double *ld = reinterpret_cast<double *>(lds);
#pragma unroll
        for (int part = 0; part < 2; part++) {
            double(&x)[8] = part ? xi : xr;
#pragma unroll
            for (int c = 0; c < NB; c++) {
                const unsigned b = c * TPG + jt;
                const unsigned kloc = b & (LLOC - 1), ml = b / LLOC;
#pragma unroll
                for (int jj = 0; jj < R; jj++) ld[lds_slot<R, LLOC, G, true>(ml * LLOC * R + kloc + jj * LLOC) * G + g] = x[c * R + jj];
            }
            __syncthreads();
#pragma unroll
            for (int c = 0; c < NB2; c++) {
                const unsigned b = c * TPG + jt;
                const unsigned kloc = b & (L2 - 1), ml = b / L2;
#pragma unroll
                for (int i = 0; i < R2; i++) x[c * R2 + i] = ld[lds_slot<R, LLOC, G, true>((ml + i * S2) * L2 + kloc) * G + g];
            }
            pin(x);
            __syncthreads();
        }
    }
}

/* Bluestein hooks (ref :1803-1827, :1838-1855, :1871-1886), applied to values that were
 * loaded unconditionally (no per-element branch around a load) */
__device__ __forceinline__ double2 chirp_in(const Args &a, double2 x, double2 h, bool inside)
{
    if (!inside) return make_double2(0.0, 0.0);
    if (a.dir == 1) return make_double2(x.x * h.x + x.y * h.y, -x.x * h.y + x.y * h.x);
    return make_double2(x.x * h.x - x.y * h.y, x.x * h.y + x.y * h.x);
}

__device__ __forceinline__ void store_hook(const Args &a, double2 *out, long long n, double yr, double yi)
{
    if (a.store_op == HS_STORE_PLAIN) {
        out[n] = make_double2(yr, yi);
    } else if (a.store_op == HS_STORE_SPEC) {
        const double2 k = a.saux[n];
        if (a.dir == 1) out[n] = make_double2(yr * k.x - yi * k.y, yr * k.y + yi * k.x);
        else out[n] = make_double2(yr * k.x + yi * k.y, -yr * k.y + yi * k.x);
    } else if (n < a.nsig) {
        const double2 h = a.saux[n];
        if (a.dir == 1) out[n] = make_double2(yr * h.x + yi * h.y, -yr * h.y + yi * h.x);
        else out[n] = make_double2(yr * h.x - yi * h.y, yr * h.y + yi * h.x);
    }
}

/* waves per SIMD the kernel's LDS footprint allows, capped at 6: asks the register
 * allocator for at most 512/6 VGPRs when LDS would let a third workgroup in (split
 * exchange of a 512-thread first pass: 32 KiB per workgroup) */
template <int R0, int N8, int G, bool FIRST, bool SPLIT>
constexpr int occ_hint()
{
    constexpr int thr = Shape<R0, N8>::TPG * G, lds = Shape<R0, N8>::P * G * (SPLIT ? 8 : 16);
    constexpr int wg = 163840 / lds, w = wg * (thr / 64) / 4;
    return FIRST && thr == 512 && w >= 6 ? 6 : 1;
}

/* TWA (round 5): every stage's twiddles loaded right behind the inputs instead of one stage at a
 * time -- for the one-workgroup launches of the small host-buffer path (c1), whose input loads
 * cross the host link, so the stages' dependent table loads no longer follow one another */
template <int R0, int N8, int G, int WQ, bool FIRST, bool SPLIT, bool HOOK, bool TWA = false>
__global__ __launch_bounds__((Shape<R0, N8>::TPG * G), (TWA ? 1 : occ_hint<R0, N8, G, FIRST, SPLIT>())) void k_pass(Args a)
{
    using S = Shape<R0, N8>;
    constexpr int P = S::P, TPG = S::TPG, WM = G / WQ;
    static_assert(N8 <= 4 && TPG * G <= 1024, "pass shape");
    extern __shared__ __attribute__((aligned(16))) double2 lds[];

    /* block -> (row b, tile): 32-bit arithmetic (64-bit division expands to long loops) */
    unsigned blk = blockIdx.x;
    if (a.xcd_groups > 0) { /* bijective XCD remap (cdna_hip_programming.md §5 'XCD swizzle') */
        const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blk % 8;
        blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blk / 8;
    }
    const unsigned tiles = (unsigned)a.tiles, nb = (unsigned)a.batch, tq = (unsigned)a.tiles_q;
    const unsigned b = a.tile_major ? blk % nb : blk / tiles;
    const unsigned tile = a.tile_major ? blk / nb : blk % tiles;
    const int tid = threadIdx.x, g = tid % G, jt = tid / G;
    const long long m = (long long)(tile / tq) * WM + g / WQ;
    const long long q = FIRST ? 0 : (long long)(tile % tq) * WQ + g % WQ;
    const bool valid = m < a.A && q < a.B;
    const double2 *in = a.in + (long long)b * a.idist;
    double2 *out = a.out + (long long)b * a.odist;

    double xr[8], xi[8];
    { /* stage-0 inputs straight from global memory: t = c*TPG + jt + i*(P/R0); all loads are
       * issued unconditionally (clamped index) so they stay in flight together */
        constexpr int R = R0, NB = 8 / R0, S0 = P / R0;
        const bool chirp = HOOK && a.load_op == HS_LOAD_CHIRP;
#pragma unroll
        for (int c = 0; c < NB; c++)
#pragma unroll
            for (int i = 0; i < R; i++) {
                const long long t = c * TPG + jt + i * S0;
                const long long n = valid ? (t * a.A + m) * a.B + q : 0;
                const bool inside = !chirp || n < a.nsig;
                const long long nl = inside ? n : 0;
                double2 v = in[nl];
                if constexpr (HOOK) {
                    if (chirp) v = chirp_in(a, v, a.laux[nl], inside);
                }
                xr[c * R + i] = v.x;
                xi[c * R + i] = v.y;
            }
    }

    /* twiddles are loaded one stage ahead; CTW stages load coalesced runs and redistribute
     * them through the LDS image right after the exchange that precedes their use */
    constexpr bool CTW = !FIRST && G == 8 && WQ == 8 && !SPLIT && P * G >= 8 * (TPG * G / 64) * 56;
    const long long q0 = q - g % WQ;
    double2 wa[7], wb[7];
    if constexpr (FIRST && TWA) {
        static_assert(N8 <= 3 && G == 1 && TPG <= 256, "TWA: one-workgroup first passes up to 2048 points");
        double2 w1[7], w2[7], w3[7];
        if constexpr (N8 >= 1) load_tw<8, S::Lloc(1), TPG>(w1, a, jt, q, valid);
        if constexpr (N8 >= 2) load_tw<8, S::Lloc(2), TPG>(w2, a, jt, q, valid);
        if constexpr (N8 >= 3) load_tw<8, S::Lloc(3), TPG>(w3, a, jt, q, valid);
        do_stage<R0, 1, TPG>(xr, xi, wa, a, jt, q, true);
        if constexpr (N8 >= 1) {
            exchange<R0, 1, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            do_stage<8, S::Lloc(1), TPG>(xr, xi, w1, a, jt, q, false);
        }
        if constexpr (N8 >= 2) {
            exchange<8, S::Lloc(1), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            do_stage<8, S::Lloc(2), TPG>(xr, xi, w2, a, jt, q, false);
        }
        if constexpr (N8 >= 3) {
            exchange<8, S::Lloc(2), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            do_stage<8, S::Lloc(3), TPG>(xr, xi, w3, a, jt, q, false);
        }
    } else if constexpr (FIRST) { /* tiny, cache-resident tables: load at use, keep VGPRs low */
        do_stage<R0, 1, TPG>(xr, xi, wa, a, jt, q, true);
        if constexpr (N8 >= 1) {
            exchange<R0, 1, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            load_tw<8, S::Lloc(1), TPG>(wa, a, jt, q, valid);
            do_stage<8, S::Lloc(1), TPG>(xr, xi, wa, a, jt, q, false);
        }
        if constexpr (N8 >= 2) {
            exchange<8, S::Lloc(1), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            load_tw<8, S::Lloc(2), TPG>(wa, a, jt, q, valid);
            do_stage<8, S::Lloc(2), TPG>(xr, xi, wa, a, jt, q, false);
        }
        if constexpr (N8 >= 3) {
            exchange<8, S::Lloc(2), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            load_tw<8, S::Lloc(3), TPG>(wa, a, jt, q, valid);
            do_stage<8, S::Lloc(3), TPG>(xr, xi, wa, a, jt, q, false);
        }
        if constexpr (N8 >= 4) { /* whole-row 8192 = [2,8,8,8,8] */
            exchange<8, S::Lloc(3), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
            load_tw<8, S::Lloc(4), TPG>(wa, a, jt, q, valid);
            do_stage<8, S::Lloc(4), TPG>(xr, xi, wa, a, jt, q, false);
        }
    } else {
    static_assert(N8 <= 3, "later passes have at most three radix-8 stages");
    if constexpr (!FIRST) load_tw<R0, 1, TPG>(wa, a, jt, q, valid);
    if constexpr (N8 >= 1) {
        if constexpr (CTW) load_tw_co<S::Lloc(1)>(wb, a, jt, q0);
        else load_tw<8, S::Lloc(1), TPG>(wb, a, jt, q, valid);
    }
    do_stage<R0, 1, TPG>(xr, xi, wa, a, jt, q, FIRST);
    if constexpr (N8 >= 1) {
        if constexpr (N8 >= 2) {
            if constexpr (CTW) load_tw_co<S::Lloc(2)>(wa, a, jt, q0);
            else load_tw<8, S::Lloc(2), TPG>(wa, a, jt, q, valid);
        }
        exchange<R0, 1, 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
        if constexpr (CTW) redistribute_tw(wb, lds);
        do_stage<8, S::Lloc(1), TPG>(xr, xi, wb, a, jt, q, false);
    }
    if constexpr (N8 >= 2) {
        if constexpr (N8 >= 3) {
            if constexpr (CTW) load_tw_co<S::Lloc(3)>(wb, a, jt, q0);
            else load_tw<8, S::Lloc(3), TPG>(wb, a, jt, q, valid);
        }
        if constexpr (CTW) __syncthreads(); /* every wave has read its twiddles back */
        exchange<8, S::Lloc(1), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
        if constexpr (CTW) redistribute_tw(wa, lds);
        do_stage<8, S::Lloc(2), TPG>(xr, xi, wa, a, jt, q, false);
    }
    if constexpr (N8 >= 3) {
        if constexpr (CTW) __syncthreads();
        exchange<8, S::Lloc(2), 8, TPG, P, G, SPLIT>(xr, xi, lds, jt, g);
        if constexpr (CTW) redistribute_tw(wb, lds);
        do_stage<8, S::Lloc(3), TPG>(xr, xi, wb, a, jt, q, false);
    }
    }

    /* last stage: ml == 0, output u = kloc + jj*LL, written to [m][u][q] */
    constexpr int RL = S::R(S::NST - 1), LL = S::Lloc(S::NST - 1), NBL = 8 / RL;
    if (valid) {
#pragma unroll
        for (int c = 0; c < NBL; c++) {
            const int kloc = c * TPG + jt;
#pragma unroll
            for (int jj = 0; jj < RL; jj++) {
                const long long n = (m * P + kloc + jj * LL) * a.B + q;
                if constexpr (HOOK) store_hook(a, out, n, xr[c * RL + jj], xi[c * RL + jj]);
                else out[n] = make_double2(xr[c * RL + jj], xi[c * RL + jj]);
            }
        }
    }
    if (a.done) { /* the launch is this one workgroup (host-checked): tell the host it is done --
                   * every thread publishes its own stores at system scope, then one lane stores
                   * the word (a release store at system scope) */
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(a.done, a.done_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* Later-pass variant for [8,8,8] (P = 512) tiles of 8 q-columns that transforms T
 * consecutive rows with the same tile: the twiddles of all three stages are loaded (and
 * for stages 1-2 redistributed through LDS) once and reused T times, dividing the pass's
 * twiddle traffic -- for 2^20's pass B about as many bytes as the data itself -- by T. */
template <int T>
__global__ __launch_bounds__(512, 4) void k_pass_b512(Args a)
{
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    unsigned blk = blockIdx.x;
    if (a.xcd_groups > 0) {
        const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blk % 8;
        blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blk / 8;
    }
    const unsigned tiles = (unsigned)a.tiles;
    const unsigned bg = blk / tiles, tile = blk % tiles;
    const int tid = threadIdx.x, g = tid % G, jt = tid / G;
    const long long q0 = (long long)tile * G, q = q0 + g;
    /* stage-2 twiddles (the 14 MiB table) loaded coalesced once and kept in registers for
     * all T rows; stage 0/1 (0.2 / 1.8 MiB tables, cache-resident) are reloaded per row */
    double2 w2[7];
    load_tw_co<64>(w2, a, jt, q0);
    redistribute_tw(w2, lds);
    __syncthreads();
    const unsigned b0 = bg * T;
#pragma unroll 1
    for (int it = 0; it < T; it++) {
        const unsigned b = b0 + it;
        if (b >= (unsigned)a.batch) break;
        const double2 *in = a.in + (long long)b * a.idist;
        double2 *out = a.out + (long long)b * a.odist;
        double xr[8], xi[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = in[(long long)(jt + i * TPG) * a.B + q];
            xr[i] = v.x;
            xi[i] = v.y;
        }
        double2 w[7];
        load_tw<8, 1, TPG>(w, a, jt, q, true);
        do_stage<8, 1, TPG>(xr, xi, w, a, jt, q, false);
        load_tw<8, 8, TPG>(w, a, jt, q, true);
        exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
        do_stage<8, 8, TPG>(xr, xi, w, a, jt, q, false);
        exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
        do_stage<8, 64, TPG>(xr, xi, w2, a, jt, q, false);
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const long long n = (long long)(jt + jj * 64) * a.B + q;
            if (a.store_op == HS_STORE_PLAIN) out[n] = make_double2(xr[jj], xi[jj]);
            else store_hook(a, out, n, xr[jj], xi[jj]);
        }
    }
}

/* A later [8,8,8] pass (P = 512, A == 1) for the 8 q-columns q0..q0+7 of one row, as in
 * k_pass's coalesced-twiddle path; on return thread (g, jt) holds outputs u = jt + 64*jj of
 * column q0 + g.  Starts with a barrier, so it may follow any earlier LDS use. */
__device__ __forceinline__ void tile888(double (&xr)[8], double (&xi)[8], const Args &a, const double2 *in,
                                        long long q0, int jt, int g, double2 *lds)
{
    constexpr int P = 512, TPG = 64, G = 8;
    const long long q = q0 + g;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const double2 v = in[(long long)(jt + i * TPG) * a.B + q];
        xr[i] = v.x;
        xi[i] = v.y;
    }
    double2 wa[7], wb[7];
    load_tw<8, 1, TPG>(wa, a, jt, q, true);
    load_tw_co<8>(wb, a, jt, q0);
    do_stage<8, 1, TPG>(xr, xi, wa, a, jt, q, false);
    load_tw_co<64>(wa, a, jt, q0);
    __syncthreads(); /* earlier LDS readers (redistributed twiddles, exchanges) are done */
    exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
    redistribute_tw(wb, lds);
    do_stage<8, 8, TPG>(xr, xi, wb, a, jt, q, false);
    __syncthreads();
    exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
    redistribute_tw(wa, lds);
    do_stage<8, 64, TPG>(xr, xi, wa, a, jt, q, false);
}

/* Bluestein middle for M = 512*512 (ref :1797-1855): the last pass of the forward FFT of
 * the chirped row ([8,8,8] at L = B = 512, tiles of 8 q-columns), the spectrum product with
 * hk (:1803-1827) and the first pass of the inverse FFT ([8,8,8] leaf, conjugated twiddles,
 * sign -sgn; :1838-1855) on the same registers: column q of the former is column m = q of
 * the latter and thread jt holds points u = jt + 64*i of both, so the intermediate never
 * goes back to HBM.  a.sgn/a.conj: forward FFT; sgn2/conj2: inverse FFT; a.saux = hk. */
__global__ __launch_bounds__(512) void k_blue_mid(Args a, int sgn2, int conj2)
{
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    unsigned blk = blockIdx.x;
    {
        const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blk % 8;
        blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blk / 8;
    }
    const unsigned tiles = (unsigned)a.tiles, b = blk / tiles, tile = blk % tiles;
    const int tid = threadIdx.x, g = tid % G, jt = tid / G;
    const long long q0 = (long long)tile * G, q = q0 + g;
    const double2 *in = a.in + (long long)b * a.idist;
    double2 *out = a.out + (long long)b * a.odist;
    double xr[8], xi[8];
    tile888(xr, xi, a, in, q0, jt, g, lds); /* forward FFT, last pass */
    /* spectrum product: element u*B + q, u = jt + 64*jj (store_hook's HS_STORE_SPEC) */
#pragma unroll
    for (int jj = 0; jj < 8; jj++) {
        const double2 k = a.saux[(long long)(jt + jj * TPG) * a.B + q];
        const double yr = xr[jj], yi = xi[jj];
        if (a.dir == 1) {
            xr[jj] = yr * k.x - yi * k.y;
            xi[jj] = yr * k.y + yi * k.x;
        } else {
            xr[jj] = yr * k.x + yi * k.y;
            xi[jj] = -yr * k.y + yi * k.x;
        }
    }
    /* inverse FFT, first pass: column m = q, L = 1 */
    Args a2 = a;
    a2.B = 1;
    a2.sgn = sgn2;
    a2.conj = conj2;
    double2 wa[7];
    do_stage<8, 1, TPG>(xr, xi, wa, a2, jt, 0, true);
    __syncthreads(); /* every wave has read its redistributed twiddles */
    exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
    load_tw<8, 8, TPG>(wa, a2, jt, 0, true);
    do_stage<8, 8, TPG>(xr, xi, wa, a2, jt, 0, false);
    exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
    load_tw<8, 64, TPG>(wa, a2, jt, 0, true);
    do_stage<8, 64, TPG>(xr, xi, wa, a2, jt, 0, false);
#pragma unroll
    for (int jj = 0; jj < 8; jj++) out[q * P + jt + jj * TPG] = make_double2(xr[jj], xi[jj]);
}

inline int launch_blue_mid(const void *in, void *out, long long dist, const void *tw, const void *hk, int batch,
                           int sgn, int conj, int dir, int sgn2, int conj2, hipStream_t st)
{
    Args a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)in;
    a.out = (double2 *)out;
    a.tw = (const double2 *)tw;
    a.saux = (const double2 *)hk;
    a.idist = a.odist = dist;
    a.A = 1;
    a.B = 512;
    a.sgn = sgn;
    a.conj = conj;
    a.dir = dir;
    a.batch = batch;
    a.tiles = a.tiles_q = 512 / 8;
    const long long grid = a.tiles * (long long)batch;
    if (grid <= 0 || grid > 0x7fffffffLL) return -1;
    hipLaunchKernelGGL(k_blue_mid, dim3((unsigned)grid), dim3(512), 512 * 8 * sizeof(double2), st, a, sgn2, conj2);
    HCHK(hipGetLastError());
    return 0;
}

/* r2c split fused into the last c2c pass (ref real.c:108-132).  For h = N/2 whose c2c plan
 * ends in a later [8,8,8] pass with A == 1 (columns q < B, B % 16 == 0), output k = u*B + q
 * of that pass pairs with h - k = (P-1-u)*B + (B-q) (q > 0), so the lo tile of columns
 * [8j+1, 8j+9) and the hi tile [B-8j-8, B-8j) are closed under the pairing: a workgroup
 * computes both tiles, swaps the hi tile through LDS, and writes X[k], X[N-k], X[h-k] and
 * X[h+k] for every k of its lo tile.  Tile j == B/16 handles column 0 (u <-> P-u, X[0], X[h]).
 * a.in: pass-A output (row dist idist), a.out: X (row dist odist = N), a.saux: twiddle2. */
__device__ __forceinline__ void r2c_pair(double2 a, double2 c, double2 w, double &re, double &im)
{
    const double t1 = a.y + c.y, t2 = c.x - a.x;
    re = (a.x + c.x + (t1 * w.x) + (t2 * w.y)) / 2.0;
    im = (a.y - c.y + (t2 * w.x) - (t1 * w.y)) / 2.0;
}

#ifdef HSFFT_DEV_PROBES /* round 1's split kernel: development build only (HSFFT_R2C_FUSE=2) */
__global__ __launch_bounds__(512, 4) void k_r2c_last(Args a, long long h)
{
    constexpr int P = 512, TPG = 64, G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    unsigned blk = blockIdx.x;
    {
        const unsigned nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blk % 8;
        blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blk / 8;
    }
    const unsigned tiles = (unsigned)a.tiles, b = blk / tiles, j = blk % tiles;
    const int tid = threadIdx.x, g = tid % G, jt = tid / G;
    const long long B = a.B, N = 2 * h;
    const double2 *in = a.in + (long long)b * a.idist;
    double2 *X = a.out + (long long)b * a.odist;
    const double2 *w2 = a.saux;
    double xr[8], xi[8];
    if (j < tiles - 1) {
        const long long qlo = 8 * (long long)j + 1, qhi = B - 8 * (long long)j - 8;
        double hr[8], hi[8];
        tile888(hr, hi, a, in, qhi, jt, g, lds);
        tile888(xr, xi, a, in, qlo, jt, g, lds);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) lds[(jt + jj * TPG) * G + g] = make_double2(hr[jj], hi[jj]);
        __syncthreads();
        const long long q = qlo + g;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const int u = jt + jj * TPG;
            const long long k = u * B + q, hk = h - k;
            const double2 zk = make_double2(xr[jj], xi[jj]), zh = lds[(P - 1 - u) * G + (7 - g)];
            double re, im;
            r2c_pair(zk, zh, w2[k], re, im);
            X[k] = make_double2(re, im);
            X[N - k] = make_double2(re, -im);
            r2c_pair(zh, zk, w2[hk], re, im);
            X[hk] = make_double2(re, im);
            X[N - hk] = make_double2(re, -im);
        }
    } else { /* column 0: k = u*B pairs with (P-u)*B */
        tile888(xr, xi, a, in, 0, jt, g, lds);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) lds[(jt + jj * TPG) * G + g] = make_double2(xr[jj], xi[jj]);
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const int u = jt + jj * TPG;
            const long long k = u * B;
            const double2 zk = make_double2(xr[jj], xi[jj]);
            if (u == 0) {
                X[0] = make_double2(zk.x + zk.y, 0.0);
                X[h] = make_double2(zk.x - zk.y, 0.0);
            } else {
                const double2 zh = lds[(P - u) * G];
                double re, im;
                r2c_pair(zk, zh, w2[k], re, im);
                X[k] = make_double2(re, im);
                X[N - k] = make_double2(re, -im);
            }
        }
    }
}

inline int launch_r2c_last(const void *Z, long long zdist, void *X, long long xdist, const void *tw, const void *w2,
                           long long h, long long B, int batch, int sgn, hipStream_t st)
{
    if (B % 16 || B * 512 != h) return -1;
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
    a.sgn = sgn;
    a.batch = batch;
    a.tiles = a.tiles_q = B / 16 + 1;
    const long long grid = a.tiles * (long long)batch;
    if (grid <= 0 || grid > 0x7fffffffLL) return -1;
    hipLaunchKernelGGL(k_r2c_last, dim3((unsigned)grid), dim3(512), 512 * 8 * sizeof(double2), st, a, h);
    HCHK(hipGetLastError());
    return 0;
}
#endif

typedef void (*kfn)(Args);

struct Variant {
    int r0, n8, G, WQ;
    bool first, split, hook;
    kfn fn;
};

#define R8V(r0, n8, g, wq, f)                                                                        \
    {r0, n8, g, wq, f, false, false, k_pass<r0, n8, g, wq, f, false, false>},                        \
        {r0, n8, g, wq, f, true, false, k_pass<r0, n8, g, wq, f, true, false>},                      \
        {r0, n8, g, wq, f, false, true, k_pass<r0, n8, g, wq, f, false, true>},                      \
        {r0, n8, g, wq, f, true, true, k_pass<r0, n8, g, wq, f, true, true>}
static const Variant k_variants[] = {
    /* first passes (B == 1): WQ = 1, G = WM */
    R8V(4, 3, 1, 1, true), R8V(4, 3, 2, 1, true), R8V(4, 3, 4, 1, true),
    R8V(2, 3, 1, 1, true), R8V(2, 3, 2, 1, true), R8V(2, 3, 4, 1, true),
    R8V(8, 3, 1, 1, true), R8V(8, 3, 2, 1, true), R8V(2, 4, 1, 1, true), /* 8192 = [2,8,8,8,8] whole row */
    R8V(8, 2, 1, 1, true), R8V(8, 2, 2, 1, true), R8V(8, 2, 4, 1, true), R8V(8, 2, 8, 1, true),
    R8V(4, 2, 1, 1, true), R8V(4, 2, 4, 1, true), R8V(4, 2, 8, 1, true),
    R8V(2, 2, 1, 1, true), R8V(2, 2, 4, 1, true), R8V(2, 2, 8, 1, true),
    R8V(8, 1, 1, 1, true), R8V(8, 1, 8, 1, true), R8V(8, 1, 16, 1, true),
    R8V(4, 1, 1, 1, true), R8V(4, 1, 16, 1, true), R8V(4, 1, 32, 1, true),
    R8V(2, 1, 1, 1, true), R8V(2, 1, 16, 1, true),
    R8V(8, 0, 1, 1, true), R8V(8, 0, 16, 1, true),
    /* later passes: radix-8 only, WQ = G (tiles along q) */
    R8V(8, 2, 8, 8, false), R8V(8, 2, 4, 4, false), R8V(8, 2, 16, 16, false),
    R8V(8, 1, 8, 8, false), R8V(8, 1, 16, 16, false), R8V(8, 1, 32, 32, false),
    R8V(8, 0, 8, 8, false), R8V(8, 0, 32, 32, false),
};
#undef R8V

/* TWA first passes (G = 1, no hooks) for the small path's one-workgroup launches */
#define R8T(r0, n8) {r0, n8, 1, 1, true, false, false, k_pass<r0, n8, 1, 1, true, false, false, true>}, \
                    {r0, n8, 1, 1, true, true, false, k_pass<r0, n8, 1, 1, true, true, false, true>}
/* up to 2048 points (256 threads): at 4096 (512 threads, 150 VGPRs) measured slower, 23.28 vs
 * 22.86 us per fft_exec (profiles/r05l_c1_twa.txt) */
static const Variant k_twa[] = {R8T(2, 3), R8T(4, 3), R8T(2, 2), R8T(4, 2), R8T(8, 2), R8T(2, 1), R8T(4, 1), R8T(8, 1)};
#undef R8T

inline const Variant *find(int r0, int n8, int G, int WQ, bool first, bool split = false, bool hook = false)
{
    for (const Variant &v : k_variants)
        if (v.r0 == r0 && v.n8 == n8 && v.G == G && v.WQ == WQ && v.first == first && v.split == split &&
            v.hook == hook)
            return &v;
    return nullptr;
}

inline int split_mode(bool first)
{
    static int m = -1;
    if (m < 0) {
        const char *e = getenv("HSFFT_SPLIT");
        m = e ? atoi(e) : 1; /* split exchange for first passes only */
    }
    return first ? (m & 1) : ((m >> 1) & 1);
}

inline int launch(const hsd_pass *p, const hsd_launch *l, hipStream_t st)
{
    /* the pass's radices must be [r0, 8, 8, ...] with r0 in {2,4,8} */
    int n8 = p->nst - 1;
    const bool first = p->B == 1;
    const bool split = split_mode(first) && p->nst > 1;
    const bool hook = l->load_op != HS_LOAD_PLAIN || l->store_op != HS_STORE_PLAIN;
    static int tloop = -1;
    if (tloop < 0) {
        const char *e = getenv("HSFFT_BLOOP");
        tloop = e ? atoi(e) : 8;
    }
    if (!first && p->nst == 3 && p->radix[0] == 8 && p->G == 8 && p->Wq == 8 && p->A == 1 && p->B % 8 == 0 &&
        l->load_op == HS_LOAD_PLAIN && tloop > 1 && l->batch >= 2) {
        kfn fn = tloop >= 8 ? (kfn)k_pass_b512<8> : tloop >= 4 ? (kfn)k_pass_b512<4> : (kfn)k_pass_b512<2>;
        const int T = tloop >= 8 ? 8 : tloop >= 4 ? 4 : 2;
        Args a;
        memset(&a, 0, sizeof a);
        a.in = (const double2 *)l->in;
        a.out = (double2 *)l->out;
        a.tw = (const double2 *)l->tw;
        a.saux = (const double2 *)l->store_aux;
        a.idist = l->idist;
        a.odist = l->odist;
        a.A = 1;
        a.B = p->B;
        a.nsig = l->nsig;
        a.sgn = l->sgn;
        a.dir = l->dir;
        a.conj = l->conj;
        a.store_op = l->store_op;
        a.xcd_groups = 1;
        a.batch = l->batch;
        a.tiles = p->B / 8;
        a.tiles_q = a.tiles;
        const long long grid = a.tiles * ((l->batch + T - 1) / T);
        hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(512), 512 * 8 * sizeof(double2), st, a);
        HCHK(hipGetLastError());
        return 0;
    }
    const Variant *v = find(p->radix[0], n8, p->G, p->Wq, first, split, hook);
    for (int s = 1; s < p->nst; s++)
        if (p->radix[s] != 8) v = nullptr;
    if (!v || (first && !p->leaf) || p->Wm * p->Wq != p->G) {
        snprintf(g_err, sizeof g_err, "r8: no kernel variant for this pass (P=%d G=%d Wq=%d)", p->P, p->G, p->Wq);
        return -4;
    }
    Args a;
    a.in = (const double2 *)l->in;
    a.out = (double2 *)l->out;
    a.tw = (const double2 *)l->tw;
    a.laux = (const double2 *)l->load_aux;
    a.saux = (const double2 *)l->store_aux;
    a.idist = l->idist;
    a.odist = l->odist;
    a.A = p->A;
    a.B = p->B;
    a.nsig = l->nsig;
    a.sgn = l->sgn;
    a.dir = l->dir;
    a.conj = l->conj;
    a.load_op = l->load_op;
    a.store_op = l->store_op;
    /* measured on MI355X (profiles/): the XCD remap keeps neighbouring tiles of one row on
     * one L2; HSFFT_ORDER bit0/bit1 make the first / later passes tile-major */
    static int xcd = -1, order = -1;
    if (xcd < 0) {
        const char *e1 = getenv("HSFFT_XCD"), *e2 = getenv("HSFFT_ORDER");
        xcd = e1 ? atoi(e1) : 1;
        order = e2 ? atoi(e2) : 0;
    }
    a.xcd_groups = xcd;
    a.tile_major = first ? (order & 1) : ((order >> 1) & 1);
    a.batch = l->batch;
    const long long tm = (p->A + p->Wm - 1) / p->Wm, tq = (p->B + p->Wq - 1) / p->Wq;
    a.tiles_q = tq;
    a.tiles = tm * tq;
    const long long grid = a.tiles * l->batch;
    const int threads = (p->P / 8) * p->G;
    a.done = nullptr;
    a.done_val = 0;
    if (l->done && l->armed && grid == 1) { /* one workgroup: it can signal its own completion */
        a.done = l->done;
        a.done_val = l->done_val;
        *l->armed = 1;
        /* HSFFT_SMALL_TWA (default 1): the one-workgroup first pass with every stage's twiddles
         * loaded behind its inputs */
        const char *te = hs_getenv("HSFFT_SMALL_TWA");
        if (first && !hook && p->G == 1 && !(te && atoi(te) == 0))
            for (const Variant &t : k_twa)
                if (t.r0 == v->r0 && t.n8 == v->n8 && t.split == v->split) v = &t;
    }
    const size_t lds = (size_t)p->P * p->G * (split ? sizeof(double) : sizeof(double2));
    if (grid <= 0 || grid > 0x7fffffffLL || threads > 1024 || lds > 160 * 1024) {
        snprintf(g_err, sizeof g_err, "r8: bad geometry grid=%lld threads=%d lds=%zu", grid, threads, lds);
        return -1;
    }
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void *)v->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return set_err(e, "hipFuncSetAttribute");
    }
    hipLaunchKernelGGL(v->fn, dim3((unsigned)grid), dim3(threads), lds, st, a);
    HCHK(hipGetLastError());
    return 0;
}

}  // namespace r8
