/*
 * hsfft_pass_mr.h -- register-resident Stockham passes for mixed radix lists (radix 2, 3,
 * 4, 5, 7, 8 in any order, up to four stages per pass), e.g. 12600 = [3,3,5,5] + [7,8].
 *
 * Same data model as hsfft_pass_r8.h (a pass of P points at L = B views its input as
 * [t][m][q] and writes [m][u][q]; twiddles tw[L-1 + (R-1)k + i-1], k = q + B*kloc; ref
 * src/highSpeedFFT.c:731-741 and the per-radix combine loops :776-1561), but the radices
 * are template parameters, so every stage is unrolled with compile-time index math:
 *  - a column's P points are held by TPG threads; at a stage of radix R the P/R butterflies
 *    are dealt round-robin (butterfly b = jt + c*TPG), so a thread owns ceil(P/(R*TPG))
 *    butterflies -- stages whose count does not divide evenly leave some lanes idle;
 *  - stage-0 inputs come straight from global memory (clamped, unconditional loads), the
 *    stages exchange through one LDS image of P*G points, the last stage stores to global;
 *  - G columns per workgroup (consecutive m for first passes, consecutive q for later
 *    passes: G*16 contiguous bytes per row of the tile).
 * Included by hsfft_device.hip only.
 */
#pragma once

namespace mr {

template <int NST, int R0, int R1, int R2, int R3>
struct List {
    static constexpr int R(int s) { return s == 0 ? R0 : s == 1 ? R1 : s == 2 ? R2 : R3; }
    static constexpr int P = R0 * (NST > 1 ? R1 : 1) * (NST > 2 ? R2 : 1) * (NST > 3 ? R3 : 1);
    static constexpr int Lloc(int s)
    {
        return (s > 0 ? R0 : 1) * (s > 1 ? R1 : 1) * (s > 2 ? R2 : 1);
    }
};

struct MArgs {
    const double2 *in;
    double2 *out;
    const double2 *tw;
    long long idist, odist;
    int A, B, tiles_q, tiles, batch;
    int sgn, conj;
    int xcd; /* XCD-aware block remap */
    unsigned *dbg; /* k_row2 phase trace (HSFFT_ROW_DEBUG): 8 cumulative phase times per workgroup */
};

/* phase clock of the k_row2 trace: thread 0 adds the 100 MHz ticks since the last mark */
__device__ __forceinline__ void mark(const MArgs &a, unsigned &tp, int slot)
{
    if (a.dbg && threadIdx.x == 0) {
        const unsigned t = (unsigned)__builtin_amdgcn_s_memrealtime();
        a.dbg[blockIdx.x * 8 + slot] += t - tp;
        tp = t;
    }
}

constexpr int cdiv(int a, int b) { return (a + b - 1) / b; }

/* register slots per thread: the largest NB*R over the pass's stages */
template <int NST, int R0, int R1, int R2, int R3, int TPG>
constexpr int nmax()
{
    constexpr int P = List<NST, R0, R1, R2, R3>::P;
    int n = 0;
    for (int s = 0; s < NST; s++) {
        const int r = List<NST, R0, R1, R2, R3>::R(s), v = cdiv(P / r, TPG) * r;
        n = v > n ? v : n;
    }
    return n;
}

/* butterflies of one stage for this thread; x holds NB*R points (butterfly c at c*R) */
template <int R, int LLOC, int P, int TPG, bool LEAF>
__device__ __forceinline__ void stage(double *xr, double *xi, const MArgs &a, int jt, int q, bool valid)
{
    constexpr int NBF = P / R, NB = cdiv(NBF, TPG);
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int b = c * TPG + jt;
        if (NB * TPG != NBF && b >= NBF) continue; /* idle slot of an uneven stage */
        if constexpr (!LEAF) {
            const int kloc = b % LLOC;
            const long long L = (long long)a.B * LLOC;
            const long long k = valid ? q + (long long)a.B * kloc : 0;
            /* radix 4/5/7 combine loops start at k = 1 (ref :826, :904, :1062); 2, 3, 8 do not */
            const bool skip = (R == 4 || R == 5 || R == 7) && k == 0;
            if (!skip) {
                const double2 *w = a.tw + (L - 1 + (long long)(R - 1) * k);
                double2 t[R - 1];
#pragma unroll
                for (int i = 1; i < R; i++) t[i - 1] = w[i - 1];
#pragma unroll
                for (int i = 1; i < R; i++)
                    hsb::twmul(xr[c * R + i], xi[c * R + i], t[i - 1].x, a.conj ? -t[i - 1].y : t[i - 1].y);
            }
        }
        hsb::bfly<R>(&xr[c * R], &xi[c * R], a.sgn, LEAF);
    }
}

/* outputs of a stage (radix R, local L) -> LDS -> inputs of the next stage (radix R2) */
template <int R, int LLOC, int R2, int P, int TPG, int G>
__device__ __forceinline__ void exchange(double *xr, double *xi, double2 *lds, int jt, int g)
{
    constexpr int NBF = P / R, NB = cdiv(NBF, TPG);
    constexpr int L2 = LLOC * R, NBF2 = P / R2, NB2 = cdiv(NBF2, TPG), S2 = P / (L2 * R2);
    __syncthreads(); /* the previous exchange's reads are done */
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int b = c * TPG + jt;
        if (NB * TPG != NBF && b >= NBF) continue;
        const int ml = b / LLOC, kloc = b % LLOC;
#pragma unroll
        for (int jj = 0; jj < R; jj++)
            lds[(ml * LLOC * R + kloc + jj * LLOC) * G + g] = make_double2(xr[c * R + jj], xi[c * R + jj]);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NB2; c++) {
        int b = c * TPG + jt;
        if (NB2 * TPG != NBF2 && b >= NBF2) b = NBF2 - 1; /* idle slot: read something valid */
        const int ml = b / L2, kloc = b % L2;
#pragma unroll
        for (int i = 0; i < R2; i++) {
            const double2 v = lds[((ml + i * S2) * L2 + kloc) * G + g];
            xr[c * R2 + i] = v.x;
            xi[c * R2 + i] = v.y;
        }
    }
}

template <int NST, int R0, int R1, int R2, int R3, int TPG, int G, bool FIRST, bool LEAF>
__global__ __launch_bounds__(TPG * G) void k_pass(MArgs a)
{
    using LS = List<NST, R0, R1, R2, R3>;
    constexpr int P = LS::P;
    constexpr int NM = nmax<NST, R0, R1, R2, R3, TPG>();
    extern __shared__ __attribute__((aligned(16))) double2 lds[];

    unsigned blk = blockIdx.x;
    if (a.xcd) { /* consecutive tiles of a row on one XCD: they share the lines at tile edges */
        const unsigned nwg = gridDim.x, q8 = nwg / 8, r8_ = nwg % 8, xcd = blk % 8;
        blk = (xcd < r8_ ? xcd * (q8 + 1) : r8_ * (q8 + 1) + (xcd - r8_) * q8) + blk / 8;
    }
    const unsigned tiles = (unsigned)a.tiles;
    const unsigned b = blk / tiles, tile = blk % tiles;
    const int tid = threadIdx.x, g = tid % G, jt = tid / G;
    /* first passes (B == 1): G consecutive m; later passes (A == 1): G consecutive q */
    const int m = FIRST ? (int)tile * G + g : 0;
    const int q = FIRST ? 0 : (int)tile * G + g;
    const bool valid = FIRST ? m < a.A : q < a.B;
    const double2 *in = a.in + (long long)b * a.idist;
    double2 *out = a.out + (long long)b * a.odist;

    double xr[NM], xi[NM];
    {
        constexpr int NBF = P / R0, NB = cdiv(NBF, TPG);
#pragma unroll
        for (int c = 0; c < NB; c++) {
            int bf = c * TPG + jt;
            if (NB * TPG != NBF && bf >= NBF) bf = NBF - 1;
#pragma unroll
            for (int i = 0; i < R0; i++) {
                const long long t = bf + i * NBF;
                const long long n = valid ? (t * a.A + m) * a.B + q : 0;
                const double2 v = in[n];
                xr[c * R0 + i] = v.x;
                xi[c * R0 + i] = v.y;
            }
        }
    }
    stage<R0, 1, P, TPG, LEAF>(xr, xi, a, jt, q, valid);
    if constexpr (NST > 1) {
        exchange<R0, 1, R1, P, TPG, G>(xr, xi, lds, jt, g);
        stage<R1, LS::Lloc(1), P, TPG, false>(xr, xi, a, jt, q, valid);
    }
    if constexpr (NST > 2) {
        exchange<R1, LS::Lloc(1), R2, P, TPG, G>(xr, xi, lds, jt, g);
        stage<R2, LS::Lloc(2), P, TPG, false>(xr, xi, a, jt, q, valid);
    }
    if constexpr (NST > 3) {
        exchange<R2, LS::Lloc(2), R3, P, TPG, G>(xr, xi, lds, jt, g);
        stage<R3, LS::Lloc(3), P, TPG, false>(xr, xi, a, jt, q, valid);
    }
    /* last stage: butterfly b = kloc (ml == 0), output u = kloc + jj*LL to [m][u][q] */
    constexpr int RL = LS::R(NST - 1), LL = LS::Lloc(NST - 1), NBFL = P / RL, NBL = cdiv(NBFL, TPG);
    if (!valid) return;
#pragma unroll
    for (int c = 0; c < NBL; c++) {
        const int kloc = c * TPG + jt;
        if (NBL * TPG != NBFL && kloc >= NBFL) continue;
#pragma unroll
        for (int jj = 0; jj < RL; jj++) {
            const long long n = ((long long)m * P + kloc + jj * LL) * a.B + q;
            out[n] = make_double2(xr[c * RL + jj], xi[c * RL + jj]);
        }
    }
}

/* ------------------------------------------------------------------ whole-row kernel
 * All six stages of a row in one launch (12600 = [3,3,5,5,7,8]: 197 KB per row, more than
 * LDS but not more than a workgroup's registers): 1024 threads hold the row (<= 16 points
 * each), the exchanges go through an image of P doubles -- real parts, then imaginary
 * parts ("split", 98.4 KiB for 12600) -- and the row is read from and written to HBM once,
 * instead of once per pass.  One workgroup per CU (LDS-bound); the other resident rows are
 * simply the next workgroups.  Stage arithmetic is mr::stage's (same twiddles, operand
 * order, k == 0 skips), so results are bit-identical to the two-pass schedule. */
template <int R0, int R1, int R2, int R3, int R4, int R5>
struct List6 {
    static constexpr int R(int s)
    {
        return s == 0 ? R0 : s == 1 ? R1 : s == 2 ? R2 : s == 3 ? R3 : s == 4 ? R4 : R5;
    }
    static constexpr int P = R0 * R1 * R2 * R3 * R4 * R5;
    static constexpr int Lloc(int s)
    {
        int l = 1;
        for (int i = 0; i < s; i++) l *= R(i);
        return l;
    }
    template <int TPG>
    static constexpr int nmax()
    {
        int n = 0;
        for (int i = 0; i < 6; i++) {
            const int v = cdiv(P / R(i), TPG) * R(i);
            n = v > n ? v : n;
        }
        return n;
    }
};

/* exchange of one double per point (split image): stage (R, LLOC) outputs -> stage R2 inputs */
template <int R, int LLOC, int R2, int P, int TPG>
__device__ __forceinline__ void xchg1(double *x, double *ld, int jt)
{
    constexpr int NBF = P / R, NB = cdiv(NBF, TPG);
    constexpr int L2 = LLOC * R, NBF2 = P / R2, NB2 = cdiv(NBF2, TPG), S2 = P / (L2 * R2);
    __syncthreads(); /* the image's previous readers are done */
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int b = c * TPG + jt;
        if (NB * TPG != NBF && b >= NBF) continue;
        const int ml = b / LLOC, kloc = b % LLOC;
#pragma unroll
        for (int jj = 0; jj < R; jj++) ld[ml * LLOC * R + kloc + jj * LLOC] = x[c * R + jj];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NB2; c++) {
        int b = c * TPG + jt;
        if (NB2 * TPG != NBF2 && b >= NBF2) b = NBF2 - 1; /* idle slot: read something valid */
        const int ml = b / L2, kloc = b % L2;
#pragma unroll
        for (int i = 0; i < R2; i++) x[c * R2 + i] = ld[(ml + i * S2) * L2 + kloc];
    }
}

template <int R, int LLOC, int R2, int P, int TPG>
__device__ __forceinline__ void xchg_split(double *xr, double *xi, double *ld, int jt)
{
    xchg1<R, LLOC, R2, P, TPG>(xr, ld, jt);
    xchg1<R, LLOC, R2, P, TPG>(xi, ld, jt);
}

template <int R0, int R1, int R2, int R3, int R4, int R5, int TPG>
__global__ __launch_bounds__(TPG) void k_row(MArgs a)
{
    using LS = List6<R0, R1, R2, R3, R4, R5>;
    constexpr int P = LS::P;
    constexpr int NM = LS::template nmax<TPG>();
    extern __shared__ __attribute__((aligned(16))) double ldsd[];
    const unsigned b = blockIdx.x;
    const int jt = threadIdx.x;
    const double2 *in = a.in + (long long)b * a.idist;
    double2 *out = a.out + (long long)b * a.odist;
    double xr[NM], xi[NM];
    {
        constexpr int NBF = P / R0, NB = cdiv(NBF, TPG);
#pragma unroll
        for (int c = 0; c < NB; c++) {
            int bf = c * TPG + jt;
            if (NB * TPG != NBF && bf >= NBF) bf = NBF - 1;
#pragma unroll
            for (int i = 0; i < R0; i++) {
                const double2 v = in[bf + i * NBF];
                xr[c * R0 + i] = v.x;
                xi[c * R0 + i] = v.y;
            }
        }
    }
    stage<R0, 1, P, TPG, true>(xr, xi, a, jt, 0, true);
    xchg_split<R0, 1, R1, P, TPG>(xr, xi, ldsd, jt);
    stage<R1, LS::Lloc(1), P, TPG, false>(xr, xi, a, jt, 0, true);
    xchg_split<R1, LS::Lloc(1), R2, P, TPG>(xr, xi, ldsd, jt);
    stage<R2, LS::Lloc(2), P, TPG, false>(xr, xi, a, jt, 0, true);
    xchg_split<R2, LS::Lloc(2), R3, P, TPG>(xr, xi, ldsd, jt);
    stage<R3, LS::Lloc(3), P, TPG, false>(xr, xi, a, jt, 0, true);
    xchg_split<R3, LS::Lloc(3), R4, P, TPG>(xr, xi, ldsd, jt);
    stage<R4, LS::Lloc(4), P, TPG, false>(xr, xi, a, jt, 0, true);
    xchg_split<R4, LS::Lloc(4), R5, P, TPG>(xr, xi, ldsd, jt);
    stage<R5, LS::Lloc(5), P, TPG, false>(xr, xi, a, jt, 0, true);
    /* last stage: butterfly kloc, outputs u = kloc + jj*LL */
    constexpr int LL = LS::Lloc(5), NBFL = P / R5, NBL = cdiv(NBFL, TPG);
#pragma unroll
    for (int c = 0; c < NBL; c++) {
        const int kloc = c * TPG + jt;
        if (NBL * TPG != NBFL && kloc >= NBFL) continue;
#pragma unroll
        for (int jj = 0; jj < R5; jj++) out[kloc + jj * LL] = make_double2(xr[c * R5 + jj], xi[c * R5 + jj]);
    }
}

/* k_row2: k_row walking rows (grid = one workgroup per CU), with the twiddles of the
 * combine stages before the last ((R-1)*L entries at L-1: tw[0, Lloc(5)-1), 1574 for 12600,
 * 24.6 KiB) copied to LDS once per workgroup, so only the last stage reads global (L2)
 * twiddles; 32-bit index math; conjugation a template constant. */
template <int R, int LLOC, int P, int TPG, bool LEAF, bool CONJ, bool TR = false>
__device__ __forceinline__ void rstage(double *xr, double *xi, const double2 *tws, int jt, int sgn)
{
    /* tws = tw + (LLOC - 1): stage twiddles tw[L-1 + (R-1)k + i-1] (ref :776-1561) */
    constexpr int NBF = P / R, NB = cdiv(NBF, TPG);
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int b = c * TPG + jt;
        if (NB * TPG != NBF && b >= NBF) continue;
        if constexpr (!LEAF) {
            const unsigned k = (unsigned)b % (unsigned)LLOC;
            const bool skip = (R == 4 || R == 5 || R == 7) && k == 0;
            if (!skip) {
                double2 t[R - 1];
#pragma unroll
                for (int i = 1; i < R; i++) t[i - 1] = TR ? tws[(i - 1) * LLOC + k] : tws[(R - 1) * k + i - 1];
#pragma unroll
                for (int i = 1; i < R; i++) hsb::twmul(xr[c * R + i], xi[c * R + i], t[i - 1].x, CONJ ? -t[i - 1].y : t[i - 1].y);
            }
        }
        hsb::bfly<R>(&xr[c * R], &xi[c * R], sgn, LEAF);
    }
}

/* Stages 0 and 1 fused in registers (FUSE01): stage-1 butterfly (ml, kloc) reads output kloc
 * of the stage-0 butterflies ml + S*i (S = P/(R0*R1), i < R1), so the R0*R1 points of group
 * ml are closed under both stages -- a thread transforms whole groups and the first exchange
 * disappears.  Same butterflies, twiddles and operand order as the unfused stages. */
/* inputs of fused01's groups 0..PFG-1 (ml = g*TPG + jt) of a row, loaded ahead (k_row2 PF) */
template <int R0, int R1, int P, int TPG, int PFG>
__device__ __forceinline__ void f01_load0(double2 (&p0)[PFG * R0 * R1], const double2 *in, int jt)
{
    constexpr int S = P / (R0 * R1), NBF0 = P / R0;
#pragma unroll
    for (int g = 0; g < PFG; g++) {
        int ml = g * TPG + jt;
        if (ml >= S) ml = S - 1;
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++)
#pragma unroll
            for (int i = 0; i < R0; i++)
                p0[(g * R1 + j1) * R0 + i] = pf::ldg(in, (unsigned)(ml + S * j1 + i * NBF0) * 16u);
    }
}

template <int R0, int R1, int P, int TPG, bool CONJ, int HAS0 = 0>
__device__ __forceinline__ void fused01(double *xr, double *xi, const double2 *in, const double2 *ltw, double *ld,
                                        int jt, int sgn, const double2 *p0 = nullptr)
{
    constexpr int S = P / (R0 * R1), NG = cdiv(S, TPG), NBF0 = P / R0, Q = R0 * R1;
#pragma unroll
    for (int g = 0; g < NG; g++) {
        int ml = g * TPG + jt;
        if (NG * TPG != S && ml >= S) ml = S - 1; /* idle slot: compute on a valid group */
        double *yr = xr + g * Q, *yi = xi + g * Q;
        /* stage 0 (leaf): butterfly j1 of the group is b = ml + S*j1, inputs t = b + i*P/R0 */
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++)
#pragma unroll
            for (int i = 0; i < R0; i++) {
                const double2 v = g < HAS0 ? p0[(g * R1 + j1) * R0 + i] : pf::ldg(in, (unsigned)(ml + S * j1 + i * NBF0) * 16u);
                yr[j1 * R0 + i] = v.x;
                yi[j1 * R0 + i] = v.y;
            }
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++) hsb::bfly<R0>(&yr[j1 * R0], &yi[j1 * R0], sgn, true);
        /* stage 1 (L = R0): butterfly kloc takes output kloc of stage-0 butterfly i */
        double zr[Q], zi[Q];
#pragma unroll
        for (int kloc = 0; kloc < R0; kloc++) {
#pragma unroll
            for (int i = 0; i < R1; i++) {
                zr[kloc * R1 + i] = yr[i * R0 + kloc];
                zi[kloc * R1 + i] = yi[i * R0 + kloc];
            }
            const bool skip = (R1 == 4 || R1 == 5 || R1 == 7) && kloc == 0;
            if (!skip) {
#pragma unroll
                for (int i = 1; i < R1; i++) {
                    const double2 t = ltw[(R0 - 1) + (i - 1) * R0 + kloc]; /* transposed (k_row2) */
                    hsb::twmul(zr[kloc * R1 + i], zi[kloc * R1 + i], t.x, CONJ ? -t.y : t.y);
                }
            }
            hsb::bfly<R1>(&zr[kloc * R1], &zi[kloc * R1], sgn, false);
        }
#pragma unroll
        for (int q = 0; q < Q; q++) {
            yr[q] = zr[q];
            yi[q] = zi[q];
        }
    }
}

/* exchange after fused01: output jj of stage-1 butterfly (ml, kloc) goes to ml*Q + kloc +
 * jj*R0 (LLOC = R0), then stage R2's standard round-robin read (L2 = Q) */
template <int R0, int R1, int R2, int P, int TPG>
__device__ __forceinline__ void xchg1_f01(double *x, double *ld, int jt)
{
    constexpr int S = P / (R0 * R1), NG = cdiv(S, TPG), Q = R0 * R1;
    constexpr int NBF2 = P / R2, NB2 = cdiv(NBF2, TPG), S2 = P / (Q * R2);
    __syncthreads();
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int ml = g * TPG + jt;
        if (NG * TPG != S && ml >= S) continue;
#pragma unroll
        for (int kloc = 0; kloc < R0; kloc++)
#pragma unroll
            for (int jj = 0; jj < R1; jj++) ld[ml * Q + kloc + jj * R0] = x[g * Q + kloc * R1 + jj];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NB2; c++) {
        int b = c * TPG + jt;
        if (NB2 * TPG != NBF2 && b >= NBF2) b = NBF2 - 1;
        const int ml = b / Q, kloc = b % Q;
#pragma unroll
        for (int i = 0; i < R2; i++) x[c * R2 + i] = ld[(ml + i * S2) * Q + kloc];
    }
}

/* Two consecutive combine stages fused in registers (k_row2 F23): stage a (radix RA, local L)
 * and stage b (radix RB, local L*RA).  Group g (< NG2 = P/(RA*RB)) is (ml' = g / L, kloc =
 * g % L): stage-a butterflies ml' + i'*S' (S' = NG2/L, i' < RB) at kloc and stage-b
 * butterflies kloc + jj*L (jj < RA) at ml' -- closed under both stages (stage-b butterfly jj
 * takes output jj of every stage-a butterfly of the group), so the exchange between the two
 * stages disappears.  Same twiddles (LDS copy, transposed as rstage<TR>), skips and operand
 * order as the unfused stages, so the results are bit-identical.
 * Register layout: group c of this thread at x[c*Q ...], point i of stage-a butterfly i' at
 * x[c*Q + i'*RA + i] on entry; on exit output jj' of stage-b butterfly jj at x[c*Q + jj*RB + jj']. */
template <int RA, int RB, int L, int P, int TPG, bool CONJ>
__device__ __forceinline__ void fused_ab(double *xr, double *xi, const double2 *ltw, int jt, int sgn)
{
    constexpr int Q = RA * RB, NG2 = P / Q, NGT = cdiv(NG2, TPG), LB = L * RA;
    const double2 *twa = ltw + (L - 1), *twb = ltw + (LB - 1);
#pragma unroll
    for (int c = 0; c < NGT; c++) {
        int g = c * TPG + jt;
        if (NGT * TPG != NG2 && g >= NG2) g = NG2 - 1; /* idle slot: compute on a valid group */
        const unsigned kloc = (unsigned)g % (unsigned)L;
        double *yr = xr + c * Q, *yi = xi + c * Q;
        /* stage a: RB butterflies of radix RA, all at k = kloc */
        {
            const bool skip = (RA == 4 || RA == 5 || RA == 7) && kloc == 0;
            double2 t[RA - 1];
#pragma unroll
            for (int i = 1; i < RA; i++) t[i - 1] = twa[(i - 1) * L + kloc];
#pragma unroll
            for (int ib = 0; ib < RB; ib++) {
                if (!skip) {
#pragma unroll
                    for (int i = 1; i < RA; i++)
                        hsb::twmul(yr[ib * RA + i], yi[ib * RA + i], t[i - 1].x, CONJ ? -t[i - 1].y : t[i - 1].y);
                }
                hsb::bfly<RA>(&yr[ib * RA], &yi[ib * RA], sgn, false);
            }
        }
        /* stage b: butterfly jj (k = kloc + jj*L) takes output jj of stage-a butterfly ib */
        double zr[Q], zi[Q];
#pragma unroll
        for (int jj = 0; jj < RA; jj++) {
#pragma unroll
            for (int ib = 0; ib < RB; ib++) {
                zr[jj * RB + ib] = yr[ib * RA + jj];
                zi[jj * RB + ib] = yi[ib * RA + jj];
            }
            const unsigned k = kloc + (unsigned)jj * L;
            const bool skip = (RB == 4 || RB == 5 || RB == 7) && k == 0;
            if (!skip) {
#pragma unroll
                for (int i = 1; i < RB; i++) {
                    const double2 t = twb[(i - 1) * LB + k];
                    hsb::twmul(zr[jj * RB + i], zi[jj * RB + i], t.x, CONJ ? -t.y : t.y);
                }
            }
            hsb::bfly<RB>(&zr[jj * RB], &zi[jj * RB], sgn, false);
        }
#pragma unroll
        for (int q = 0; q < Q; q++) {
            yr[q] = zr[q];
            yi[q] = zi[q];
        }
    }
}

/* exchange fused01's outputs (stage-1 butterfly (ml, kloc) output jj at ml*Q0 + kloc + jj*R0)
 * into fused_ab's group inputs (point i of stage-a butterfly i' of group g at g + NG2*(i' + RB*i)) */
template <int R0, int R1, int RA, int RB, int P, int TPG>
__device__ __forceinline__ void xchg1_f01_ab(double *x, double *ld, int jt)
{
    constexpr int S = P / (R0 * R1), NG = cdiv(S, TPG), Q0 = R0 * R1;
    constexpr int Q = RA * RB, NG2 = P / Q, NGT = cdiv(NG2, TPG);
    __syncthreads();
#pragma unroll
    for (int g = 0; g < NG; g++) {
        const int ml = g * TPG + jt;
        if (NG * TPG != S && ml >= S) continue;
#pragma unroll
        for (int kloc = 0; kloc < R0; kloc++)
#pragma unroll
            for (int jj = 0; jj < R1; jj++) ld[ml * Q0 + kloc + jj * R0] = x[g * Q0 + kloc * R1 + jj];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NGT; c++) {
        int g = c * TPG + jt;
        if (NGT * TPG != NG2 && g >= NG2) g = NG2 - 1;
#pragma unroll
        for (int ib = 0; ib < RB; ib++)
#pragma unroll
            for (int i = 0; i < RA; i++) x[c * Q + ib * RA + i] = ld[g + NG2 * (ib + RB * i)];
    }
}

/* exchange fused_ab's outputs (output jj' of stage-b butterfly kloc + jj*L of group (ml', kloc)
 * at ml'*L*RA*RB + kloc + jj*L + jj'*L*RA) into the next stage's inputs (radix RN at local
 * LN = L*RA*RB: butterfly b reads (b/LN + i*SN)*LN + b%LN, SN = P/(LN*RN)) */
template <int RA, int RB, int L, int RN, int P, int TPG>
__device__ __forceinline__ void xchg1_ab_std(double *x, double *ld, int jt)
{
    constexpr int Q = RA * RB, NG2 = P / Q, NGT = cdiv(NG2, TPG), LN = L * Q;
    constexpr int NBF2 = P / RN, NB2 = cdiv(NBF2, TPG), SN = P / (LN * RN);
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NGT; c++) {
        const int g = c * TPG + jt;
        if (NGT * TPG != NG2 && g >= NG2) continue;
        const int mlp = g / L, kloc = g % L;
#pragma unroll
        for (int jj = 0; jj < RA; jj++)
#pragma unroll
            for (int jq = 0; jq < RB; jq++) ld[mlp * LN + kloc + jj * L + jq * L * RA] = x[c * Q + jj * RB + jq];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NB2; c++) {
        int b = c * TPG + jt;
        if (NB2 * TPG != NBF2 && b >= NBF2) b = NBF2 - 1;
        const int ml = b / LN, kloc = b % LN;
#pragma unroll
        for (int i = 0; i < RN; i++) x[c * RN + i] = ld[(ml + i * SN) * LN + kloc];
    }
}

/* k_row2 F45: the last two stages ([7, 8] at L = P/56) fused with TWO threads per group instead of
 * an exchange through the split image.  Group g (< G45 = P/56) is the 8 stage-4 butterflies
 * (ml = 0..7, kloc = g) and the 7 stage-5 butterflies kloc5 = g + jj*G45 (jj < 7): stage-5
 * butterfly jj takes output jj of every stage-4 butterfly of the group.  Thread pair (2g, 2g+1)
 * of one wave holds it: thread A (even) the stage-4 butterflies ml = 0..3, thread B (odd) ml =
 * 4..7; after stage 4 they swap, through one DPP lane swap per dword, the 16 outputs A's stage-5
 * butterflies (jj = 0..3) need from B and the 12 B's (jj = 4..6) need from A -- no LDS, no block
 * barrier.  Same twiddles (stage 4 from the transposed LDS copy, stage 5 from global), skips and
 * operand order as rstage, so the results are bit-identical. */
__device__ __forceinline__ double lane_swap(double v)
{
    int2 u;
    __builtin_memcpy(&u, &v, 8);
    u.x = __builtin_amdgcn_mov_dpp(u.x, 0xB1, 0xF, 0xF, false); /* quad_perm [1,0,3,2] */
    u.y = __builtin_amdgcn_mov_dpp(u.y, 0xB1, 0xF, 0xF, false);
    double r;
    __builtin_memcpy(&r, &u, 8);
    return r;
}

/* exchange fused_ab's outputs (as xchg1_ab_std writes them) into F45's stage-4 inputs: thread
 * (g, h) reads butterflies ml = 4h + c (c < 4) at kloc = g, point i at (ml + 8i)*G45 + g.
 * (A padded pitch of 260 doubles, conflict-free ds_read_b64 instead of ds_read2_b64, measured
 * 5.741 vs 5.749 ms in round 5 and removed.) */
template <int RA, int RB, int L, int P, int TPG>
__device__ __forceinline__ void xchg1_ab_g45(double *x, double *ld, int jt)
{
    constexpr int Q = RA * RB, NG2 = P / Q, NGT = cdiv(NG2, TPG), LN = L * Q, G45 = P / 56;
    static_assert(LN == G45, "F45 follows F23 at L = P / 56");
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NGT; c++) {
        const int g = c * TPG + jt;
        if (NGT * TPG != NG2 && g >= NG2) continue;
        const int mlp = g / L, kloc = g % L;
#pragma unroll
        for (int jj = 0; jj < RA; jj++)
#pragma unroll
            for (int jq = 0; jq < RB; jq++) ld[mlp * LN + kloc + jj * L + jq * L * RA] = x[c * Q + jj * RB + jq];
    }
    __syncthreads();
    const int h = jt & 1;
    int g = jt >> 1;
    if (g >= G45) g = G45 - 1; /* idle threads read a valid group */
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int i = 0; i < 7; i++) x[c * 7 + i] = ld[(4 * h + c + 8 * i) * G45 + g];
}

/* TWN 3: the stage-5 twiddles of steps d >= 1 (k-blocks jj = 1, 2, 3 of thread A and 5, 6 of
 * thread B, 225 k x 7 each) are copied into LDS before the first store of the row -- four blocks
 * into the free exchange image, the fifth behind the stage twiddle copy -- transposed to
 * [i-1][k - 225 jj]; step 0 reads its run from global as before (no store precedes it).  So no
 * twiddle load waits behind a store burst (vmcnt is in order). */
constexpr int F45_BLK = 1575; /* 225 k x 7 entries */
__device__ __forceinline__ const double2 *f45_slot(const double2 *img, const double2 *extra, int s)
{
    return s < 4 ? img + s * F45_BLK : extra;
}
template <int P, int TPG>
__device__ __forceinline__ void f45_tw_copy(const double2 *tw, double2 *img, double2 *extra, int jt)
{
    constexpr int G45 = P / 56, L5 = 7 * G45, NE = 5 * F45_BLK, NIT = (NE + TPG - 1) / TPG;
    static_assert(G45 * 7 == F45_BLK, "F45 block");
    double2 v[NIT];
#pragma unroll
    for (int it = 0; it < NIT; it++) {
        int e = it * TPG + jt;
        if (e >= NE) e = NE - 1;
        const int blk = e / F45_BLK, r = e % F45_BLK, jj = blk < 3 ? blk + 1 : blk + 2;
        v[it] = pf::ldg(tw, (unsigned)(L5 - 1 + 7 * G45 * jj + r) * 16u);
    }
#pragma unroll
    for (int it = 0; it < NIT; it++) {
        const int e = it * TPG + jt;
        if (e >= NE) continue;
        const int blk = e / F45_BLK, r = e % F45_BLK;
        const_cast<double2 *>(f45_slot(img, extra, blk))[(r % 7) * G45 + r / 7] = v[it];
    }
}

/* stages 4 (radix 7) and 5 (radix 8) of the pair's group, then the row's stores */
template <int P, int TPG, bool CONJ, int TWN = 0>
__device__ __forceinline__ void fused45_pair(double *xr, double *xi, const double2 *ltw, const double2 *tw,
                                             double2 *out, int jt, int sgn, const double2 *timg = nullptr,
                                             const double2 *textra = nullptr)
{
    constexpr int G45 = P / 56, L4 = G45, L5 = 7 * G45;
    const int h = jt & 1, g0 = jt >> 1;
    const bool live = g0 < G45;
    const unsigned g = live ? (unsigned)g0 : (unsigned)(G45 - 1);
    /* stage 4: butterflies ml = 4h + c at k = g (radix 7 skips k == 0) */
    {
        const double2 *twa = ltw + (L4 - 1);
        double2 t[6];
#pragma unroll
        for (int i = 1; i < 7; i++) t[i - 1] = twa[(i - 1) * L4 + g];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            if (g != 0) {
#pragma unroll
                for (int i = 1; i < 7; i++) hsb::twmul(xr[c * 7 + i], xi[c * 7 + i], t[i - 1].x, CONJ ? -t[i - 1].y : t[i - 1].y);
            }
            hsb::bfly<7>(&xr[c * 7], &xi[c * 7], sgn, false);
        }
    }
    /* stage 5, one butterfly per step d: this thread's is jj = d (A) or 4 + d (B, d < 3; B's
     * d = 3 is idle), k = g + jj*G45.  Per step the pair swaps 4 values: A sends output 4 + d of
     * its butterflies (B's inputs 0..3), B sends output d of its butterflies (A's inputs 4..7) */
    const double2 *twb = tw + (L5 - 1);
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int jj = h ? 4 + d : d, da = d < 3 ? 4 + d : 6;
        double zr[8], zi[8];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const double sr = lane_swap(h ? xr[i * 7 + d] : xr[i * 7 + da]);
            const double si = lane_swap(h ? xi[i * 7 + d] : xi[i * 7 + da]);
            zr[i] = h ? sr : xr[i * 7 + d];
            zi[i] = h ? si : xi[i * 7 + d];
            zr[4 + i] = h ? xr[i * 7 + da] : sr;
            zi[4 + i] = h ? xi[i * 7 + da] : si;
        }
        const unsigned k = g + (unsigned)(h && d == 3 ? 0 : jj) * G45; /* B's d = 3 is idle: a valid k */
#pragma unroll
        for (int i = 1; i < 8; i++) {
            /* TWN 2 (timing probe, development builds): constant twiddles, results wrong */
            double2 t;
            if constexpr (TWN == 2) t = make_double2(0.5, 0.25 * i);
            else if constexpr (TWN == 3) {
                /* slots 0-2: A's d = 1..3; 3, 4: B's d = 1, 2 (B's idle d = 3 reads slot 2) */
                const int sl = h ? (d == 3 ? 2 : d + 2) : d - 1;
                t = d == 0 ? pf::ldg(twb, (7 * k + i - 1) * 16u) : f45_slot(timg, textra, sl)[(i - 1) * G45 + g];
            } else if constexpr (TWN == 4) {
                /* the plan's transposed copy of this stage's block at tw + P ([i-1][k]) */
                t = pf::ldg(tw + P, ((i - 1) * L5 + k) * 16u);
            } else t = pf::ldg(twb, (7 * k + i - 1) * 16u);
            hsb::twmul(zr[i], zi[i], t.x, CONJ ? -t.y : t.y);
        }
        hsb::bfly<8>(zr, zi, sgn, false);
        if (live && (h == 0 || d < 3)) {
#pragma unroll
            for (int j5 = 0; j5 < 8; j5++) pf::stg(out, (k + (unsigned)j5 * L5) * 16u, make_double2(zr[j5], zi[j5]));
        }
    }
}

/* fused01 for a row whose points [0, 2*P/R0) were prefetched into `pre` by LDS-DMA (k_row2
 * PRE): the remaining leaf inputs (i = R0-1) are loaded from global first, then one barrier
 * behind every wave's vmcnt(0) (all LDS-DMA has landed), then the prefetched inputs are read
 * from LDS.  Same values, same butterflies as fused01. */
template <int R0, int R1, int P, int TPG, bool CONJ>
__device__ __forceinline__ void fused01p(double *xr, double *xi, const double2 *in, const double2 *ltw,
                                         const double2 *pre, int jt, int sgn)
{
    constexpr int S = P / (R0 * R1), NG = cdiv(S, TPG), NBF0 = P / R0, Q = R0 * R1;
    static_assert(R0 == 3, "prefetch layout assumes a radix-3 leaf");
#pragma unroll
    for (int g = 0; g < NG; g++) {
        int ml = g * TPG + jt;
        if (NG * TPG != S && ml >= S) ml = S - 1;
        double *yr = xr + g * Q, *yi = xi + g * Q;
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++) {
            const double2 v = pf::ldg(in, (unsigned)(ml + S * j1 + (R0 - 1) * NBF0) * 16u);
            yr[j1 * R0 + R0 - 1] = v.x;
            yi[j1 * R0 + R0 - 1] = v.y;
        }
    }
    /* every wave's LDS-DMA has landed: an explicit vmcnt(0) per wave, then the barrier
     * (__syncthreads alone does not order the DMA: hipcc puts its vmcnt(0) after s_barrier) */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int g = 0; g < NG; g++) {
        int ml = g * TPG + jt;
        if (NG * TPG != S && ml >= S) ml = S - 1;
        double *yr = xr + g * Q, *yi = xi + g * Q;
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++)
#pragma unroll
            for (int i = 0; i < R0 - 1; i++) {
                const double2 v = pre[ml + S * j1 + i * NBF0];
                yr[j1 * R0 + i] = v.x;
                yi[j1 * R0 + i] = v.y;
            }
    }
#pragma unroll
    for (int g = 0; g < NG; g++) {
        double *yr = xr + g * Q, *yi = xi + g * Q;
#pragma unroll
        for (int j1 = 0; j1 < R1; j1++) hsb::bfly<R0>(&yr[j1 * R0], &yi[j1 * R0], sgn, true);
        double zr[Q], zi[Q];
#pragma unroll
        for (int kloc = 0; kloc < R0; kloc++) {
#pragma unroll
            for (int i = 0; i < R1; i++) {
                zr[kloc * R1 + i] = yr[i * R0 + kloc];
                zi[kloc * R1 + i] = yi[i * R0 + kloc];
            }
            const bool skip = (R1 == 4 || R1 == 5 || R1 == 7) && kloc == 0;
            if (!skip) {
#pragma unroll
                for (int i = 1; i < R1; i++) {
                    const double2 t = ltw[(R0 - 1) + (i - 1) * R0 + kloc];
                    hsb::twmul(zr[kloc * R1 + i], zi[kloc * R1 + i], t.x, CONJ ? -t.y : t.y);
                }
            }
            hsb::bfly<R1>(&zr[kloc * R1], &zi[kloc * R1], sgn, false);
        }
#pragma unroll
        for (int q = 0; q < Q; q++) {
            yr[q] = zr[q];
            yi[q] = zi[q];
        }
    }
}

/* one 16-B-per-lane LDS-DMA: lane l copies g[l] to lds_base + 16 l (lds_base wave-uniform) */
__device__ __forceinline__ void glds16(const double2 *g, double2 *lds_base)
{
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)lds_base, 16, 0, 0);
}

/* points of the next row prefetched by k_row2<..., PRE>: 132 wave-instructions of 64 */
constexpr int ROW_PRE_PTS = 8448;

/* PF: the inputs of the next row's first PF 9-point groups (37 % of a row per group at
 * TPG = 512) are loaded into registers right after this row's first exchange, so their
 * latency overlaps this row's remaining stages (needs the VGPRs of TPG = 512: 256 per thread) */
template <int R0, int R1, int R2, int R3, int R4, int R5, int TPG, bool CONJ, bool F01, bool PRE = false, int PF = 0,
          bool F23 = false, bool F45 = false, int TWN = 0>
__global__ __launch_bounds__(TPG) void k_row2(MArgs a)
{
    static_assert(!F45 || (F23 && R4 == 7 && R5 == 8 && 2 * (R0 * R1 * R2 * R3) <= TPG), "F45: [7,8] after F23");
    static_assert(PF == 0 || (F01 && !PRE), "PF prefetches fused01's first groups");
    static_assert(!F23 || (F01 && !PRE), "F23 follows fused01");
    using LS = List6<R0, R1, R2, R3, R4, R5>;
    constexpr int P = LS::P, NT = LS::Lloc(5) - 1; /* LDS twiddles tw[0, NT) */
    constexpr int NM0 = LS::template nmax<TPG>(), NMF = cdiv(P / (R0 * R1), TPG) * R0 * R1;
    constexpr int NM1 = F01 && NMF > NM0 ? NMF : NM0, NM23 = cdiv(P / (R2 * R3), TPG) * R2 * R3;
    constexpr int NM = F23 && NM23 > NM1 ? NM23 : NM1;
    extern __shared__ __attribute__((aligned(16))) double ldsd[];
    /* PRE: [ltw | exchange image + prefetch area]; else [exchange image | ltw] */
    static_assert(!PRE || (F01 && NT % 2 == 0 && 2 * NT * 8 + ROW_PRE_PTS * 16 <= 160 * 1024 &&
                           ROW_PRE_PTS >= 2 * (P / R0) && P * 8 <= ROW_PRE_PTS * 16),
                  "row prefetch layout");
    double2 *ltw = PRE ? reinterpret_cast<double2 *>(ldsd) : reinterpret_cast<double2 *>(ldsd + P + (P & 1));
    double *img = PRE ? ldsd + 2 * NT : ldsd;
    const int jt0 = threadIdx.x, sgn = a.sgn;
    /* LDS copy of the stage-1..4 twiddles, transposed within each stage's block [L-1, RL-1):
     * entry (k, i) at L-1 + (i-1)*L + k, so the lanes of a wave (consecutive k) read
     * consecutive 16-B words instead of words (R-1)*16 B apart (LDS bank conflicts) */
    for (int e = LS::Lloc(1) - 1 + jt0; e < NT; e += TPG) { /* [0, R0-1): the leaf's, unused */
        int L = LS::Lloc(1), R = R1;
        if (e >= LS::Lloc(4) - 1) {
            L = LS::Lloc(4);
            R = R4;
        } else if (e >= LS::Lloc(3) - 1) {
            L = LS::Lloc(3);
            R = R3;
        } else if (e >= LS::Lloc(2) - 1) {
            L = LS::Lloc(2);
            R = R2;
        }
        const int loc = e - (L - 1), k = loc / (R - 1), i1 = loc % (R - 1);
        ltw[L - 1 + i1 * L + k] = a.tw[e];
    }
    /* fused01 reads the stage-1 entries before the first exchange's barrier, so the copy
     * needs a barrier of its own (once per workgroup) */
    __syncthreads();
    unsigned tp = (unsigned)__builtin_amdgcn_s_memrealtime();
    bool pre = false; /* PRE: this row's points [0, ROW_PRE_PTS) are in the image area */
    double2 p0[(PF > 0 ? PF : 1) * R0 * R1]; /* PF: the next row's first PF groups of inputs */
    if constexpr (PF > 0) f01_load0<R0, R1, P, TPG, PF>(p0, a.in + (long long)blockIdx.x * a.idist, jt0);
#pragma unroll 1
    for (unsigned b = blockIdx.x; b < (unsigned)a.batch; b += gridDim.x) {
        int jt = jt0;
        asm volatile("" : "+v"(jt)); /* keep per-row index math (and twiddle reads) in the loop */
        const double2 *in = a.in + (long long)b * a.idist;
        double2 *out = a.out + (long long)b * a.odist;
        double xr[NM], xi[NM];
        if constexpr (F01) {
            if (PRE && pre)
                fused01p<R0, R1, P, TPG, CONJ>(xr, xi, in, ltw, reinterpret_cast<const double2 *>(img), jt, sgn);
            else
                fused01<R0, R1, P, TPG, CONJ, PF>(xr, xi, in, ltw, img, jt, sgn, p0);
            if (a.dbg) {
                r8::pin(*reinterpret_cast<double(*)[8]>(xr));
                mark(a, tp, 0); /* loads + stages 0-1 */
            }
            if constexpr (F23) {
                xchg1_f01_ab<R0, R1, R2, R3, P, TPG>(xr, img, jt);
                xchg1_f01_ab<R0, R1, R2, R3, P, TPG>(xi, img, jt);
            } else {
                xchg1_f01<R0, R1, R2, P, TPG>(xr, img, jt);
                xchg1_f01<R0, R1, R2, P, TPG>(xi, img, jt);
            }
            if constexpr (PF > 0) { /* unconditional: the last row of a workgroup reloads itself */
                const unsigned bn = b + gridDim.x < (unsigned)a.batch ? b + gridDim.x : b;
                f01_load0<R0, R1, P, TPG, PF>(p0, a.in + (long long)bn * a.idist, jt);
            }
            mark(a, tp, 1);
        } else {
            {
                constexpr int NBF = P / R0, NB = cdiv(NBF, TPG);
#pragma unroll
                for (int c = 0; c < NB; c++) {
                    int bf = c * TPG + jt;
                    if (NB * TPG != NBF && bf >= NBF) bf = NBF - 1;
#pragma unroll
                    for (int i = 0; i < R0; i++) {
                        const double2 v = pf::ldg(in, (unsigned)(bf + i * NBF) * 16u);
                        xr[c * R0 + i] = v.x;
                        xi[c * R0 + i] = v.y;
                    }
                }
            }
            rstage<R0, 1, P, TPG, true, CONJ>(xr, xi, ltw, jt, sgn);
            xchg_split<R0, 1, R1, P, TPG>(xr, xi, img, jt);
            rstage<R1, LS::Lloc(1), P, TPG, false, CONJ, true>(xr, xi, ltw + (LS::Lloc(1) - 1), jt, sgn);
            xchg_split<R1, LS::Lloc(1), R2, P, TPG>(xr, xi, img, jt);
        }
        if constexpr (F45) { /* stages 2-3 fused, then 4-5 fused over thread pairs: two exchanges */
            fused_ab<R2, R3, LS::Lloc(2), P, TPG, CONJ>(xr, xi, ltw, jt, sgn);
            mark(a, tp, 2);
            xchg1_ab_g45<R2, R3, LS::Lloc(2), P, TPG>(xr, img, jt);
            xchg1_ab_g45<R2, R3, LS::Lloc(2), P, TPG>(xi, img, jt);
            mark(a, tp, 3);
            if constexpr (TWN == 3) {
                __syncthreads(); /* every wave has read the image */
                f45_tw_copy<P, TPG>(a.tw, reinterpret_cast<double2 *>(img), ltw + NT, jt);
                __syncthreads();
            }
            fused45_pair<P, TPG, CONJ, TWN>(xr, xi, ltw, a.tw, out, jt, sgn, reinterpret_cast<const double2 *>(img),
                                            ltw + NT);
            mark(a, tp, 6);
            if (a.dbg && threadIdx.x == 0) a.dbg[blockIdx.x * 8 + 7] += 1;
            continue;
        }
        if constexpr (F23) { /* stages 2 and 3 fused in registers: one exchange fewer */
            fused_ab<R2, R3, LS::Lloc(2), P, TPG, CONJ>(xr, xi, ltw, jt, sgn);
            mark(a, tp, 2);
            xchg1_ab_std<R2, R3, LS::Lloc(2), R4, P, TPG>(xr, img, jt);
            xchg1_ab_std<R2, R3, LS::Lloc(2), R4, P, TPG>(xi, img, jt);
            mark(a, tp, 3);
        } else {
            rstage<R2, LS::Lloc(2), P, TPG, false, CONJ, true>(xr, xi, ltw + (LS::Lloc(2) - 1), jt, sgn);
            xchg_split<R2, LS::Lloc(2), R3, P, TPG>(xr, xi, img, jt);
            mark(a, tp, 2);
            rstage<R3, LS::Lloc(3), P, TPG, false, CONJ, true>(xr, xi, ltw + (LS::Lloc(3) - 1), jt, sgn);
            xchg_split<R3, LS::Lloc(3), R4, P, TPG>(xr, xi, img, jt);
            mark(a, tp, 3);
        }
        rstage<R4, LS::Lloc(4), P, TPG, false, CONJ, true>(xr, xi, ltw + (LS::Lloc(4) - 1), jt, sgn);
        xchg_split<R4, LS::Lloc(4), R5, P, TPG>(xr, xi, img, jt);
        mark(a, tp, 4);
        rstage<R5, LS::Lloc(5), P, TPG, false, CONJ>(xr, xi, a.tw + (LS::Lloc(5) - 1), jt, sgn);
        if (a.dbg) {
            r8::pin(*reinterpret_cast<double(*)[8]>(xr));
            mark(a, tp, 5); /* last stage (global twiddles) */
        }
        if constexpr (PRE) {
            /* the image is free once every wave has read its last exchange: prefetch the next
             * row's first ROW_PRE_PTS points into it by LDS-DMA while this row is stored */
            const unsigned bn = b + gridDim.x;
            pre = bn < (unsigned)a.batch;
            if (pre) {
                __syncthreads();
                const double2 *inn = a.in + (long long)bn * a.idist;
                const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
                double2 *dst = reinterpret_cast<double2 *>(img);
#pragma unroll 1
                for (unsigned j = wave; j < (unsigned)ROW_PRE_PTS / 64; j += TPG / 64)
                    glds16(inn + j * 64 + lane, dst + j * 64);
            }
        }
        constexpr int LL = LS::Lloc(5), NBFL = P / R5, NBL = cdiv(NBFL, TPG);
#pragma unroll
        for (int c = 0; c < NBL; c++) {
            const int kloc = c * TPG + jt;
            if (NBL * TPG != NBFL && kloc >= NBFL) continue;
#pragma unroll
            for (int jj = 0; jj < R5; jj++)
                pf::stg(out, (unsigned)(kloc + jj * LL) * 16u, make_double2(xr[c * R5 + jj], xi[c * R5 + jj]));
        }
        mark(a, tp, 6); /* stores issued */
        if (a.dbg && threadIdx.x == 0) a.dbg[blockIdx.x * 8 + 7] += 1;
    }
}

typedef void (*kfn)(MArgs);

struct Variant {
    int nst, r[6], tpg, G;
    bool first, leaf;
    kfn fn;
    bool row; /* k_row: the whole row (A == B == 1) in one launch */
};

#define MRV(n, a, b, c, d, tpg, g, f, l) {n, {a, b, c, d, 1, 1}, tpg, g, f, l, k_pass<n, a, b, c, d, tpg, g, f, l>, false}
static const Variant k_variants[] = {
    /* 12600 = [3,3,5,5] + [7,8] (BASELINE config 3) */
    MRV(4, 3, 3, 5, 5, 45, 8, true, true),
    MRV(2, 7, 8, 1, 1, 8, 45, false, false),
    MRV(2, 7, 8, 1, 1, 8, 15, false, false),
    MRV(2, 7, 8, 1, 1, 8, 16, false, false),
    /* 12600 whole-row (HSFFT_MR_ROW=0: the two passes above); launched as k_row2 */
    {6, {3, 3, 5, 5, 7, 8}, 512, 1, true, true, nullptr, true},
};
#undef MRV

/* picks a variant for a pass of the generic schedule; fills the tile geometry */
inline const Variant *select(hsd_pass *p)
{
    if (p->nst == 6) { /* whole-row variants */
        if (p->B != 1 || p->A != 1) return nullptr;
        for (const Variant &v : k_variants) {
            if (!v.row || v.leaf != (p->leaf != 0)) continue;
            bool same = true;
            for (int s = 0; s < 6; s++) same &= v.r[s] == p->radix[s];
            if (!same) continue;
            p->G = p->Wm = p->Wq = 1;
            return &v;
        }
        return nullptr;
    }
    if (p->nst < 1 || p->nst > 4) return nullptr;
    const bool first = p->B == 1;
    if (!first && p->A != 1) return nullptr;
    const Variant *best = nullptr;
    long long best_waste = -1;
    for (const Variant &v : k_variants) {
        if (v.row || v.nst != p->nst || v.first != first || v.leaf != (p->leaf != 0)) continue;
        bool same = true;
        for (int s = 0; s < p->nst; s++) same &= v.r[s] == p->radix[s];
        if (!same) continue;
        const long long ext = first ? p->A : p->B; /* columns the tiles cover */
        const long long waste = (ext + v.G - 1) / v.G * v.G - ext;
        if (!best || waste < best_waste) {
            best = &v;
            best_waste = waste;
        }
    }
    if (!best) return nullptr;
    p->G = best->G;
    p->Wm = first ? best->G : 1;
    p->Wq = first ? 1 : best->G;
    return best;
}

inline int launch(const hsd_pass *p, const hsd_launch *l, hipStream_t st)
{
    hsd_pass tmp = *p;
    const Variant *v = select(&tmp);
    if (!v || l->load_op != HS_LOAD_PLAIN || l->store_op != HS_STORE_PLAIN) {
        snprintf(g_err, sizeof g_err, "mr: no kernel variant for this pass (P=%d)", p->P);
        return -4;
    }
    MArgs a;
    memset(&a, 0, sizeof a);
    a.in = (const double2 *)l->in;
    a.out = (double2 *)l->out;
    a.tw = (const double2 *)l->tw;
    a.idist = l->idist;
    a.odist = l->odist;
    a.A = (int)p->A;
    a.B = (int)p->B;
    a.sgn = l->sgn;
    a.conj = l->conj;
    a.batch = l->batch;
    {
        const char *e = getenv("HSFFT_MR_XCD");
        a.xcd = e ? atoi(e) : 1; /* c3: 78-80 -> 84-88 GSamples/s */
    }
    if (v->row) { /* 12600 = [3,3,5,5,7,8]: k_row2 (the only whole-row variant) */
        constexpr int P = 12600, NT = 1574;
        const size_t lds0 = (size_t)P * sizeof(double) + (size_t)NT * sizeof(double2);
        if (l->batch <= 0) {
            snprintf(g_err, sizeof g_err, "mr: bad row batch=%d", l->batch);
            return -1;
        }
        /* 512 threads (8 waves, 256 VGPRs per thread) with the next row's first input group
         * (37 % of the row) loaded into registers during this row's stages 2-5: 113.5 -> 123.5
         * GSamples/s over the 1024-thread kernel.  Measured and removed: 768 /
         * 1024-thread kernels, prefetching ones that spill, an LDS-DMA prefetch of the next row,
         * the unfused stage 0/1 form. */
        /* F23 (HSFFT_ROW_F23, default 1): stages 2 and 3 ([5,5], 504 groups of 25 points)
         * fused in registers as stages 0 and 1 are -- three exchanges per row instead of four */
        const char *e23 = getenv("HSFFT_ROW_F23");
        const bool f23 = e23 ? atoi(e23) != 0 : true;
        /* F45 (HSFFT_ROW_F45, default 1 since round 4): stages 4 and 5 ([7,8], 225 groups of 56
         * points) fused over thread pairs (DPP lane swaps): two exchanges per row; in-process A/B
         * 5.97 vs 6.08 ms per 65536 rows (profiles/r04i_i_c3_f45.txt) */
        const char *e45 = getenv("HSFFT_ROW_F45");
        const bool f45 = f23 && (e45 ? atoi(e45) != 0 : true);
        kfn fn = f23 ? (a.conj ? k_row2<3, 3, 5, 5, 7, 8, 512, true, true, false, 1, true>
                               : k_row2<3, 3, 5, 5, 7, 8, 512, false, true, false, 1, true>)
                     : (a.conj ? k_row2<3, 3, 5, 5, 7, 8, 512, true, true, false, 1>
                               : k_row2<3, 3, 5, 5, 7, 8, 512, false, true, false, 1>);
        /* F45's stage-5 twiddles (default since round 4) from the plan's transposed copy of the
         * stage's block (d_tw + P: one 16-B word per lane, lanes on consecutive k, where the
         * table's own layout puts a lane's 7 entries 112 B from its neighbour's): 5.77 vs 5.87 ms
         * per 65536 rows in-process (profiles/r04r_c3_stage5_transposed.txt) */
        /* The transposed copy exists only when the plan's device state built it (l->tw_t, set
         * for exactly this schedule); without it the table is read as laid out (TWN 0, also
         * HSFFT_ROW_TWN=0) */
        const char *etwn = getenv("HSFFT_ROW_TWN");
        const bool twn4 = l->tw_t && !(etwn && atoi(etwn) == 0);
        if (f45)
            fn = twn4 ? (a.conj ? k_row2<3, 3, 5, 5, 7, 8, 512, true, true, false, 1, true, true, 4>
                                : k_row2<3, 3, 5, 5, 7, 8, 512, false, true, false, 1, true, true, 4>)
                      : (a.conj ? k_row2<3, 3, 5, 5, 7, 8, 512, true, true, false, 1, true, true, 0>
                                : k_row2<3, 3, 5, 5, 7, 8, 512, false, true, false, 1, true, true, 0>);
        /* the next row's first group loaded before this row's first exchange instead of after
         * it: 6.11 vs 5.98 ms (round 4, removed) */
        size_t lds = lds0;
#ifdef HSFFT_DEV_PROBES
        /* round 5, measured and removed: the stage-5 twiddles of steps 1-2 / 1-3 copied by LDS-DMA
         * into the free exchange image before the row's stores, 5.83 / 6.17 vs 5.68 ms
         * (profiles/r05e_c3_twn_c4_ul_ab.txt); the F45 exchange image with a padded pitch (no bank
         * conflicts, no ds_read2_b64), 5.741 vs 5.749 ms (profiles/r05b_c3_xp_ab_and_cu_mask.txt) */
        /* development build only (measurement): HSFFT_ROW_TWN=2 constant stage-5 twiddles, results
         * wrong (5.46-5.49 ms: what the twiddle loads cost); 3 those of steps 1-3 copied into LDS
         * before the row's stores (6.20 vs 5.89 ms).  Loading step d+1's run before step d's
         * stores in registers spills 17 dwords: 7.01 vs 5.93 ms (removed) */
        if (f45 && etwn && atoi(etwn) == 2 && !a.conj) fn = k_row2<3, 3, 5, 5, 7, 8, 512, false, true, false, 1, true, true, 2>;
        if (f45 && etwn && atoi(etwn) == 3) {
            fn = a.conj ? k_row2<3, 3, 5, 5, 7, 8, 512, true, true, false, 1, true, true, 3>
                        : k_row2<3, 3, 5, 5, 7, 8, 512, false, true, false, 1, true, true, 3>;
            lds = lds0 + (size_t)F45_BLK * sizeof(double2);
        }
#endif
        /* measured slower and removed (round 4): non-temporal row stores 6.32 vs 5.96 ms; the
         * next row's remaining groups copied into LDS by LDS-DMA before this row's stores, 6.15
         * vs 5.94 (the load wait moves into the store phase: profiles/r04n_c3_dma_*) */
        const int threads = 512;
        int ncu = 0, dev = 0;
        HCHK(hipGetDevice(&dev));
        HCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        const int grid = l->batch < ncu ? l->batch : (ncu > 0 ? ncu : 256);
        a.tiles = a.tiles_q = 1;
        static unsigned *s_dbg = nullptr;
        const char *de = getenv("HSFFT_ROW_DEBUG");
        if (de && atoi(de) && grid <= 4096) {
            if (!s_dbg) HCHK(hipMalloc((void **)&s_dbg, 4096 * 8 * sizeof(unsigned)));
            HCHK(hipMemsetAsync(s_dbg, 0, (size_t)grid * 8 * sizeof(unsigned), st));
            a.dbg = s_dbg;
        }
        HCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3((unsigned)threads), lds, st, a);
        HCHK(hipGetLastError());
        if (a.dbg) {
            static unsigned h[4096 * 8];
            HCHK(hipStreamSynchronize(st));
            HCHK(hipMemcpy(h, s_dbg, (size_t)grid * 8 * sizeof(unsigned), hipMemcpyDeviceToHost));
            double ph[8] = {0};
            for (int g = 0; g < grid; g++)
                for (int k = 0; k < 8; k++) ph[k] += h[g * 8 + k];
            const double rows = ph[7] > 0 ? ph[7] : 1;
            fprintf(stderr, "k_row2 per row (us): load+st01 %.2f x01 %.2f st2+x %.2f st3+x %.2f st4+x %.2f st5 %.2f store %.2f | rows %.0f\n",
                    ph[0] / rows / 100, ph[1] / rows / 100, ph[2] / rows / 100, ph[3] / rows / 100, ph[4] / rows / 100,
                    ph[5] / rows / 100, ph[6] / rows / 100, rows);
        }
        return 0;
    }
    const long long ext = v->first ? p->A : p->B;
    a.tiles = (int)((ext + v->G - 1) / v->G);
    a.tiles_q = v->first ? 1 : a.tiles;
    const long long grid = (long long)a.tiles * l->batch;
    const int threads = v->tpg * v->G;
    const size_t lds = (size_t)p->P * v->G * sizeof(double2);
    if (grid <= 0 || grid > 0x7fffffffLL || threads > 1024 || lds > 65536 || p->A > 0x7fffffff ||
        p->B > 0x7fffffff || (long long)p->A * p->B * p->P > 0x7fffffffLL) {
        snprintf(g_err, sizeof g_err, "mr: bad geometry grid=%lld threads=%d lds=%zu", grid, threads, lds);
        return -1;
    }
    hipLaunchKernelGGL(v->fn, dim3((unsigned)grid), dim3(threads), lds, st, a);
    HCHK(hipGetLastError());
    return 0;
}

}  // namespace mr
