/*
 * hsfft_pass_wl.h -- "wave-local" register passes for 2^20 = [4,8,8,8 | 8,8,8] (BASELINE
 * config 2): one workgroup barrier pair per tile instead of one per stage.
 *
 * A pass of P points whose first stages form sub-FFTs of P' points over a decimated input
 * (t = ml + (P/P')*t') runs those stages inside ONE wave: the P' x G points of sub-FFT ml
 * live in that wave's registers and its exchanges go through the wave's own slice of LDS,
 * ordered by the wave's in-order LDS queue (no s_barrier).  Only the last stage, whose
 * butterflies combine the sub-FFTs of all waves, exchanges across the workgroup.
 *
 *   pass A [4,8,8 | 8]  (P = 2048, G = 2 columns): wave ml does the 256-point sub-FFT of the
 *                       rows t = ml (mod 8) of its two columns (stages L = 1, 4, 32; ref
 *                       :804-900 leaf, :1310-1474), then stage L = 256 across waves.
 *   pass B [8,8 | 8]    (P = 512 at L = 2048, G = 8 q-columns): wave ml does the 64-point
 *                       sub-FFT of t = ml (mod 8) (stages L = 2048, 16384), then L = 131072.
 *
 * The sub-FFT is the same Stockham computation restricted to one residue class: stage s of
 * the sub-FFT reads exactly the points stage s of the full pass reads for that class, and
 * its twiddles tw[L-1 + 7k + i-1] depend on (L, k) only, which are the same in both views
 * (derivation in DESIGN.md §4).  Butterflies and twiddles are those of pf::stage, so the
 * results are bit-identical to pf::k_firstq / pf::k_b512 and the reference.
 */
#pragma once

namespace wl {

using r8::Args;

/* orders this wave's LDS writes before its later reads (and the reads before later writes):
 * one wave's LDS operations execute in order, so only the compiler must be kept from
 * moving them across */
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* r8::exchange (non-split) on one wave's image wl[P*G] */
template <int R, int LLOC, int R2, int TPG, int P, int G>
__device__ __forceinline__ void wexchange(double (&xr)[8], double (&xi)[8], double2 *wl, unsigned jt, unsigned g)
{
    constexpr int NB = 8 / R, NB2 = 8 / R2, L2 = LLOC * R, S2 = P / (L2 * R2);
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const unsigned b = c * TPG + jt;
        const unsigned kloc = b & (LLOC - 1), ml = b / LLOC;
#pragma unroll
        for (int jj = 0; jj < R; jj++) {
            const unsigned p = r8::lds_slot<R, LLOC, G>(ml * LLOC * R + kloc + jj * LLOC);
            wl[p * G + g] = make_double2(xr[c * R + jj], xi[c * R + jj]);
        }
    }
    wave_sync();
#pragma unroll
    for (int c = 0; c < NB2; c++) {
        const unsigned b = c * TPG + jt;
        const unsigned kloc = b & (L2 - 1), ml = b / L2;
#pragma unroll
        for (int i = 0; i < R2; i++) {
            const unsigned p = r8::lds_slot<R, LLOC, G>((ml + i * S2) * L2 + kloc);
            const double2 v = wl[p * G + g];
            xr[c * R2 + i] = v.x;
            xi[c * R2 + i] = v.y;
        }
    }
    r8::pin(xr);
    r8::pin(xi);
    wave_sync();
}

/* ------------------------------------------------------------------ pass A
 * input [t][m] (t < 2048, m < A), output [m][u]; a workgroup walks 2-column tiles tg,
 * tg + groups, ... of one row (pf::k_first's walk).  LDS: 8 wave images of 512 entries
 * (64 KiB; the stage-3 exchange reuses them), then tw[0, 256) (stages L = 4, 32). */
template <int SGN, bool CONJ>
__device__ __forceinline__ void aw_load(double (&xr)[8], double (&xi)[8], const double2 *row, unsigned A,
                                        unsigned m0, unsigned ml, unsigned jt, unsigned g)
{
    /* sub-FFT butterfly c*32 + jt of residue ml: rows t = ml + 8*(c*32 + jt + 64*i) */
    const unsigned lane = ((ml + 8 * jt) * A + m0 + g) * 16u;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const double2 v = pf::ldg(row + (size_t)(256 * c + 512 * i) * A, lane);
            xr[c * 4 + i] = v.x;
            xi[c * 4 + i] = v.y;
        }
}

template <int SGN, bool CONJ>
__device__ __forceinline__ void aw_body(double (&xr)[8], double (&xi)[8], const double2 (&w3)[7], double2 *lds,
                                        const double2 *ltw, double2 *orow, unsigned m0, unsigned tid)
{
    constexpr int PW = 256, TPGW = 32, G = 2;
    const unsigned wv = tid >> 6, lane = tid & 63, g = lane & 1, jt = lane >> 1;
    double2 *wimg = lds + wv * (PW * G);
    double2 w[7];
    pf::stage<4, SGN>(xr, xi, w, true);
    wexchange<4, 1, 8, TPGW, PW, G>(xr, xi, wimg, jt, g);
    pf::tw8_lds<CONJ>(w, ltw, 4, jt & 3);
    pf::stage<8, SGN>(xr, xi, w, false);
    wexchange<8, 4, 8, TPGW, PW, G>(xr, xi, wimg, jt, g);
    pf::tw8_lds<CONJ>(w, ltw, 32, jt & 31);
    pf::stage<8, SGN>(xr, xi, w, false);
    /* sub-FFT outputs u' = jt + 32 jj -> this wave's image as [g][u'] */
#pragma unroll
    for (int jj = 0; jj < 8; jj++) wimg[g * PW + jt + 32 * jj] = make_double2(xr[jj], xi[jj]);
    __syncthreads();
    /* stage L = 256: butterfly k3 takes output u' = k3 of every residue's sub-FFT */
    const unsigned k3 = tid & 255, g3 = tid >> 8;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const double2 v = lds[i * (PW * G) + g3 * PW + k3];
        xr[i] = v.x;
        xi[i] = v.y;
    }
    r8::pin(xr);
    r8::pin(xi);
    __syncthreads(); /* every image read before the next tile's wave-local writes */
    pf::stage<8, SGN>(xr, xi, w3, false);
#pragma unroll
    for (int jj = 0; jj < 8; jj++) pf::stg(orow, ((m0 + g3) * 2048u + k3 + 256u * jj) * 16u, make_double2(xr[jj], xi[jj]));
}

template <int SGN, bool CONJ, bool PREF>
__global__ __launch_bounds__(512, 4) void k_aw(Args a)
{
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + 4096;
    const unsigned blk = a.xcd_groups > 0 ? pf::xcd_remap(blockIdx.x) : blockIdx.x;
    const unsigned groups = (unsigned)a.tiles_q;
    const unsigned b = blk / groups, tg = blk % groups;
    const unsigned tid0 = threadIdx.x;
    const unsigned A = (unsigned)a.A, ntiles = A / 2;
    const double2 *row = a.in + (long long)b * a.idist;
    double2 *orow = a.out + (long long)b * a.odist;
    for (int i = tid0; i < 255; i += 512) ltw[i] = a.tw[i];
    /* stage L = 256 twiddles of this thread's butterfly k3 = tid & 255 (the same for every
     * tile): tw[255 + 7 k3 + i] */
    double2 w3[7];
    pf::tw8<CONJ>(w3, a.tw, 256, tid0 & 255);
    const int nit = (int)((ntiles - 1 - tg) / groups + 1);
    const unsigned wv = tid0 >> 6, lane = tid0 & 63;
    double pr[8], pi[8];
    if constexpr (PREF) aw_load<SGN, CONJ>(pr, pi, row, A, tg * 2, wv, lane >> 1, lane & 1);
    __syncthreads();
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned m0 = (tg + it * groups) * 2;
        double xr[8], xi[8];
        if constexpr (PREF) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                xr[i] = pr[i];
                xi[i] = pi[i];
            }
            /* next tile (clamped to the last one: no branch around the loads) */
            const unsigned mn = it + 1 < nit ? m0 + groups * 2 : m0;
            aw_load<SGN, CONJ>(pr, pi, row, A, mn, tid >> 6, (tid & 63) >> 1, tid & 1);
        } else {
            aw_load<SGN, CONJ>(xr, xi, row, A, m0, tid >> 6, (tid & 63) >> 1, tid & 1);
        }
        aw_body<SGN, CONJ>(xr, xi, w3, lds, ltw, orow, m0, tid);
    }
}

/* ------------------------------------------------------------------ pass B
 * [8,8 | 8] at L = B (P = 512, A = 1): input [t][q], output [u][q]; a workgroup owns 8
 * adjacent q-columns and walks T rows (pf::k_b512's walk).  Stage-0/1 twiddles as LDS runs
 * (k_b512 layout), stage-2 twiddles in registers.  LDS: 8 wave images of 512 entries
 * (64 KiB, reused by the stage-2 exchange), then the 504 run entries. */
template <int SGN>
__device__ __forceinline__ void bw_body(double (&xr)[8], double (&xi)[8], const double2 (&w2)[7], double2 *lds,
                                        const double2 *ltw, double2 *orow, unsigned B, unsigned q0, unsigned tid)
{
    constexpr int PW = 64, TPGW = 8, G = 8;
    const unsigned wv = tid >> 6, lane = tid & 63, g = lane & 7, jt = lane >> 3;
    double2 *wimg = lds + wv * (PW * G);
    double2 w[7];
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ltw[7 * g + i];
    pf::stage<8, SGN>(xr, xi, w, false);
    wexchange<8, 1, 8, TPGW, PW, G>(xr, xi, wimg, jt, g);
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = ltw[56 * (1 + jt) + 7 * g + i];
    pf::stage<8, SGN>(xr, xi, w, false);
    /* sub-FFT outputs u' = jt + 8 jj -> image entry [u'][g] */
#pragma unroll
    for (int jj = 0; jj < 8; jj++) wimg[(jt + 8 * jj) * G + g] = make_double2(xr[jj], xi[jj]);
    __syncthreads();
    const unsigned g2 = tid & 7, k2 = tid >> 3;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const double2 v = lds[i * (PW * G) + k2 * G + g2];
        xr[i] = v.x;
        xi[i] = v.y;
    }
    r8::pin(xr);
    r8::pin(xi);
    __syncthreads();
    pf::stage<8, SGN>(xr, xi, w2, false);
    const unsigned lane2 = (k2 * B + q0 + g2) * 16u;
#pragma unroll
    for (int jj = 0; jj < 8; jj++) pf::stg(orow + (size_t)jj * 64 * B, lane2, make_double2(xr[jj], xi[jj]));
}

template <int T, int SGN, bool CONJ>
__global__ __launch_bounds__(512, 4) void k_bw(Args a)
{
    constexpr int G = 8;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *ltw = lds + 4096;
    const unsigned blk = a.xcd_groups > 0 ? pf::xcd_remap(blockIdx.x) : blockIdx.x;
    const unsigned tiles = (unsigned)a.tiles;
    const unsigned bg = blk / tiles, tile = blk % tiles;
    const unsigned tid0 = threadIdx.x;
    const unsigned B = (unsigned)a.B;
    const unsigned q0 = tile * G;
    const unsigned b0 = bg * T, nb = (unsigned)a.batch;
    /* stage-2 twiddles (k = q + B*k2, k2 = tid >> 3): coalesced runs redistributed through
     * the (idle) image, as pf::k_b512 */
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
    const int nit = (int)min((unsigned)T, nb - b0);
#pragma unroll 1
    for (int it = 0; it < nit; it++) {
        unsigned tid = tid0;
        asm volatile("" : "+v"(tid));
        const unsigned lane = tid & 63, g = lane & 7, jt = lane >> 3, ml = tid >> 6;
        const unsigned b = b0 + it;
        const double2 *row = a.in + (long long)b * a.idist;
        /* sub-FFT butterfly jt of residue ml: rows t = ml + 8*(jt + 8 i) */
        const unsigned ofs = ((ml + 8 * jt) * B + q0 + g) * 16u;
        double xr[8], xi[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = pf::ldg(row + (size_t)i * 64 * B, ofs);
            xr[i] = v.x;
            xi[i] = v.y;
        }
        bw_body<SGN>(xr, xi, w2, lds, ltw, a.out + (long long)b * a.odist, B, q0, tid);
    }
}

/* launch helpers: the pass shapes pf::pick recognises */
inline Args make_args(const hsd_pass *p, const hsd_launch *l)
{
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
    a.xcd_groups = 1;
    a.batch = l->batch;
    return a;
}

inline int env(const char *name, int dflt)
{
    const char *s = getenv(name);
    return s ? atoi(s) : dflt;
}

/* returns 1 if no wave-local kernel applies (or HSFFT_WL does not select it), 0 on launch */
inline int launch(const hsd_pass *p, const hsd_launch *l, hipStream_t st)
{
    const int mask = env("HSFFT_WL", 0);
    if (!mask || l->load_op != HS_LOAD_PLAIN || l->store_op != HS_STORE_PLAIN || (l->sgn != 1 && l->sgn != -1))
        return 1;
    for (int s = 1; s < p->nst; s++)
        if (p->radix[s] != 8) return 1;
    typedef void (*kfn)(Args);
    Args a = make_args(p, l);
    kfn fn = nullptr;
    long long grid = 0;
    size_t lds = 0;
    if ((mask & 1) && p->B == 1 && p->leaf && p->nst == 4 && p->radix[0] == 4 && p->A % 2 == 0 && p->P == 2048) {
        const int tl = env("HSFFT_WL_T", 4);
        const long long ntiles = p->A / 2, groups = (ntiles + tl - 1) / tl;
        a.tiles_q = a.tiles = groups;
        grid = groups * l->batch;
        lds = (4096 + 256) * sizeof(double2);
        const bool pref = env("HSFFT_WL_PREF", 0) != 0;
        if (l->sgn == 1)
            fn = l->conj ? (pref ? k_aw<1, true, true> : k_aw<1, true, false>)
                         : (pref ? k_aw<1, false, true> : k_aw<1, false, false>);
        else
            fn = l->conj ? (pref ? k_aw<-1, true, true> : k_aw<-1, true, false>)
                         : (pref ? k_aw<-1, false, true> : k_aw<-1, false, false>);
    } else if ((mask & 2) && p->B > 1 && p->nst == 3 && p->radix[0] == 8 && p->A == 1 && p->B % 8 == 0 &&
               p->B * 512 < 0x10000000LL) {
        a.tiles = a.tiles_q = p->B / 8;
        grid = a.tiles * ((l->batch + 7) / 8);
        lds = (4096 + 504) * sizeof(double2);
        if (l->sgn == 1) fn = l->conj ? k_bw<8, 1, true> : k_bw<8, 1, false>;
        else fn = l->conj ? k_bw<8, -1, true> : k_bw<8, -1, false>;
    } else {
        return 1;
    }
    if (grid <= 0 || grid > 0x7fffffffLL) {
        snprintf(g_err, sizeof g_err, "wl: bad grid %lld", grid);
        return -1;
    }
    HCHK(hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(512), lds, st, a);
    HCHK(hipGetLastError());
    return 0;
}

}  // namespace wl
