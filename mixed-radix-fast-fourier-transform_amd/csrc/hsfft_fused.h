/*
 * hsfft_fused.h -- both passes of 2^20 = [4,8,8,8 | 8,8,8] (BASELINE config 2) in ONE
 * persistent launch, with the pass-A -> pass-B intermediate handed over inside the launch.
 *
 * Why: as two launches each pass reads and writes the whole batch in HBM (64 B per sample
 * in total); both already run at ~85-95 % of a stream copy, so the second HBM round trip is
 * the cost left.  Here pass B of a row group starts as soon as that group's pass-A tiles are
 * done, a few groups behind pass A, so the in-flight intermediate (lag+1 groups of R rows,
 * 16 MiB each) stays in the 256 MiB Infinity Cache and HBM sees ~32 B per sample.
 *
 * Work decomposition.  Rows are taken in groups of R.  A row has 256 pass-A tiles (2 of its
 * 512 columns, 2048 points each; as k_pass / pf::k_first) and 256 pass-B tiles (8 of its 2048
 * q-columns, 512 points; pass-B tiles walk the R rows of their group so the stage twiddles
 * are loaded once per R rows, as pf::k_b512).  Tiles are dealt to NQ = 8 ticket queues by
 * column range (queue x: tiles [32x, 32x+32) of every row), a persistent workgroup serves
 * queue blockIdx % 8 (under round-robin dispatch: one queue per XCD, so the workgroups
 * sharing a pass-A input line sit on one L2; placement is never needed for correctness).
 * Queue order: A(0) .. A(lag-1), then A(g) followed by B(g-lag), then the last B groups.
 *
 * Deadlock freedom: a workgroup only takes a ticket while running, pass-A tiles never wait,
 * and in every queue A(g) precedes B(g) and B(g') (g' >= g), so the pass-A tiles a waiting
 * pass-B tile needs were all dequeued by running workgroups (every queue has workers: the
 * grid is a multiple of 8, all resident).  Waits are bounded anyway (spin_max polls, then
 * the sticky error word is set and the call reports an error instead of hanging).
 *
 * Hand-off (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md visibility table row
 * 1): every intermediate byte is stored with 16-B sc1 buffer stores; each storing wave
 * waits vmcnt(0), a workgroup barrier, then one lane adds 1 (relaxed, agent scope) to the
 * group's counter.  The consumer polls that counter with relaxed agent loads (sc1), one
 * barrier, and reads the intermediate ONLY with 16-B sc1 buffer loads.  Inputs and
 * twiddles are never written in the launch (plain loads); pass B writes its output in
 * place over the columns it alone read.
 *
 * Arithmetic: hsfft_butterfly.h via pf::stage, the plan's own twiddles -- bit-identical to
 * the two-launch path and to the CPU reference.
 */
#pragma once

namespace fz {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int NQ = 8;      /* ticket queues */
constexpr int AT = 256;    /* pass-A tiles per row */
constexpr int BT = 256;    /* pass-B tiles per row */
constexpr unsigned ROW_BYTES = (1u << 20) * 16u;

struct FArgs {
    const double2 *in;
    double2 *out;
    const double2 *tw;
    long long idist, odist;
    unsigned *head; /* [NQ] ticket counters (zeroed per call) */
    unsigned *done; /* [ngroups] finished pass-A tiles per group (zeroed per call) */
    unsigned *err;  /* sticky: a wait gave up */
    unsigned ngroups, lag, spin_max;
    unsigned *dbg;  /* optional per-workgroup trace: tickets, last ticket, A items, B items, spins */
};

__device__ __forceinline__ double2 as_d2(u32x4 v)
{
    double2 d;
    __builtin_memcpy(&d, &v, 16);
    return d;
}
__device__ __forceinline__ u32x4 as_u4(double2 d)
{
    u32x4 v;
    __builtin_memcpy(&v, &d, 16);
    return v;
}

/* pass A, one tile: columns m = 2*tile + {0,1} of `row`, [4,8,8,8] (ref :1310-1474 stages
 * L = 1, 4, 32, 256), results stored write-through (sc1) into the output row */
template <int SGN, bool CONJ>
__device__ __forceinline__ void a_item(const FArgs &a, unsigned row, unsigned tile, double2 *lds, int tid)
{
    constexpr int P = 2048, TPG = 256, G = 2;
    const int g = tid & 1, jt = tid >> 1;
    const unsigned m = tile * 2 + g;
    const double2 *in = a.in + (long long)row * a.idist;
    double xr[8], xi[8];
    {
        const unsigned lane = (jt * 512u + m) * 16u;
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const double2 v = pf::ldg(in + (size_t)(c * TPG + i * 512) * 512, lane);
                xr[c * 4 + i] = v.x;
                xi[c * 4 + i] = v.y;
            }
    }
    unsigned long long tph = 0;
    if (a.dbg) { /* trace: load latency (issue -> landed) */
        tph = __builtin_amdgcn_s_memrealtime();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) a.dbg[blockIdx.x * 16 + 8] += (unsigned)(t1 - tph);
        tph = t1;
    }
    double2 w[7];
    pf::stage<4, SGN>(xr, xi, w, true);
    r8::exchange<4, 1, 8, TPG, P, G, true>(xr, xi, lds, jt, g);
    pf::tw8<CONJ>(w, a.tw, 4, jt & 3);
    pf::stage<8, SGN>(xr, xi, w, false);
    r8::exchange<8, 4, 8, TPG, P, G, true>(xr, xi, lds, jt, g);
    pf::tw8<CONJ>(w, a.tw, 32, jt & 31);
    pf::stage<8, SGN>(xr, xi, w, false);
    r8::exchange<8, 32, 8, TPG, P, G, true>(xr, xi, lds, jt, g);
    pf::tw8<CONJ>(w, a.tw, 256, jt & 255);
    pf::stage<8, SGN>(xr, xi, w, false);
    if (a.dbg) { /* trace: compute (stages + exchanges) */
        const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
        if (tid == 0) a.dbg[blockIdx.x * 16 + 9] += (unsigned)(t2 - tph);
    }
    /* [m][u], u = jt + 256*jj */
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(a.out + (long long)row * a.odist, 0, (int)ROW_BYTES, 0x00020000);
    const unsigned lane = (m * 2048u + jt) * 16u;
#pragma unroll
    for (int jj = 0; jj < 8; jj++)
        __builtin_amdgcn_raw_buffer_store_b128(as_u4(make_double2(xr[jj], xi[jj])), rs, lane, jj * 4096, 16);
}

/* pass A, two tiles ta, tb of `row` with the second tile's loads in flight during the first
 * tile's stages (pf::k_first's body: split exchange in [0, 32 KiB), the first-pass twiddles
 * tw[0, 2048) copied to [32, 64 KiB) per item), results stored write-through (sc1) */
template <int SGN, bool CONJ>
__device__ __forceinline__ void a_item2(const FArgs &a, unsigned row, unsigned ta, unsigned tb, double2 *lds, unsigned tid)
{
    constexpr int G = 2;
    double2 *ltw = lds + 2048;
    const double2 *in = a.in + (long long)row * a.idist;
    double2 *orow = a.out + (long long)row * a.odist;
    const unsigned g0 = tid & 1, jt0 = tid >> 1;
    double xr[8], xi[8];
    pf::first_load<4, 3, G>(xr, xi, in, 512u, ta * G + g0, jt0);
#pragma unroll
    for (int i = tid; i < 2047; i += 512) ltw[i] = a.tw[i];
    __syncthreads();
    double pr[8], pi[8];
    pf::first_load<4, 3, G>(pr, pi, in, 512u, tb * G + g0, jt0);
    {
        unsigned t = tid;
        asm volatile("" : "+v"(t));
        const unsigned g = t & 1, jt = t >> 1;
        pf::first_body<4, 3, G, SGN, CONJ, true>(xr, xi, lds, ltw, orow, ta * G + g, jt, g);
    }
    pf::first_body<4, 3, G, SGN, CONJ, true>(pr, pi, lds, ltw, orow, tb * G + g0, jt0, g0);
}

/* pass A, one 4-column group m0 .. m0+3 of `row` (two 2-column tiles) with the 64-B paired
 * loads of pf::k_firstq, results stored write-through (sc1) */
template <int SGN, bool CONJ>
__device__ __forceinline__ void a_itemq(const FArgs &a, unsigned row, unsigned m0, double2 *lds, unsigned tid)
{
    constexpr int P = 2048, TPG = 256;
    double2 *ltw = lds + 2048;
    const double2 *in = a.in + (long long)row * a.idist;
    double2 *orow = a.out + (long long)row * a.odist;
    const unsigned h = tid & 1, jt = tid >> 1, odd = jt & 1;
    const unsigned offA = ((jt - odd) * 512u + m0 + h + 2 * odd) * 16u;
    const unsigned offB = ((jt + 1 - odd) * 512u + m0 + h + 2 - 2 * odd) * 16u;
    double2 va[8], vb[8];
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const double2 *rb = in + (size_t)(c * TPG + i * (P / 4)) * 512;
            va[c * 4 + i] = pf::ldg(rb, offA);
            vb[c * 4 + i] = pf::ldg(rb, offB);
        }
#pragma unroll
    for (int i = tid; i < P - 1; i += 512) ltw[i] = a.tw[i];
    __syncthreads();
    unsigned t = tid;
    asm volatile("" : "+v"(t));
    const unsigned hh = t & 1, jj = t >> 1;
    double xr[8], xi[8], yr[8], yi[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const double2 own = odd ? vb[k] : va[k], oth = odd ? va[k] : vb[k];
        xr[k] = own.x;
        xi[k] = own.y;
        yr[k] = pf::pair_swap<2>(oth.x);
        yi[k] = pf::pair_swap<2>(oth.y);
    }
    pf::first_body<4, 3, 2, SGN, CONJ, true>(xr, xi, lds, ltw, orow, m0 + hh, jj, hh);
    pf::first_body<4, 3, 2, SGN, CONJ, true>(yr, yi, lds, ltw, orow, m0 + 2 + hh, jj, hh);
}

/* pass B, one tile (q-columns 8*qt .. 8*qt+7) over the R rows of group grp, reading the
 * intermediate with sc1 loads; output written in place with plain stores */
template <int R, int SGN, bool CONJ>
__device__ __forceinline__ void b_item(const FArgs &a, unsigned grp, unsigned qt, double2 *lds, unsigned tid)
{
    constexpr int P = 512, TPG = 64, G = 8;
    constexpr unsigned B = 2048;
    double2 *ltw = lds + P * G;
    const unsigned q0 = qt * G;
    const unsigned row0 = grp * R;
    const unsigned g0 = tid & 7, jt0 = tid >> 3;
    const unsigned lane0 = (jt0 * B + q0 + g0) * 16u;
    /* twiddles: stage 2 in registers (coalesced run + redistribution through the image),
     * stages 0/1 as LDS runs (pf::k_b512 layout) */
    r8::Args ta;
    ta.tw = a.tw;
    ta.B = B;
    double2 w2[7];
    r8::load_tw_co<64>(w2, ta, jt0, q0);
    if (tid < 504) {
        const int r = tid / 56, e = tid % 56;
        const long long src = r == 0 ? (long long)B - 1 + 7LL * q0 + e : 8LL * B - 1 + 7LL * (q0 + (long long)B * (r - 1)) + e;
        double2 v = a.tw[src];
        if (CONJ) v.y = -v.y;
        ltw[tid] = v;
    }
    r8::redistribute_tw(w2, lds);
    if (CONJ) {
#pragma unroll
        for (int i = 0; i < 7; i++) w2[i].y = -w2[i].y;
    }
    __syncthreads();
    /* no row prefetch (as pf::k_b512's default): 32 fewer live VGPRs */
#pragma unroll 1
    for (int it = 0; it < R; it++) {
        unsigned t = tid;
        asm volatile("" : "+v"(t));
        const unsigned g = t & 7, jt = t >> 3;
        const unsigned lane = (jt * B + q0 + g) * 16u;
        double xr[8], xi[8];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            a.out + (long long)(row0 + it) * a.odist, 0, (int)ROW_BYTES, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const double2 v = as_d2(__builtin_amdgcn_raw_buffer_load_b128(rs, lane, i * TPG * B * 16, 16));
            xr[i] = v.x;
            xi[i] = v.y;
        }
        pf::b512_body<SGN>(xr, xi, w2, lds, ltw, a.out + (long long)(row0 + it) * a.odist, B, lane, jt, g);
    }
}

/* ticket t of a queue -> (pass, group, index within the group's slice of this queue) */
template <int R>
__device__ __forceinline__ void decode(unsigned t, unsigned ng, unsigned lag, bool &isA, unsigned &grp, unsigned &i)
{
    constexpr unsigned nA = R * AT / NQ / 2, nB = BT / NQ;
    const unsigned L = lag < ng ? lag : ng;
    if (t < L * nA) {
        isA = true;
        grp = t / nA;
        i = t % nA;
        return;
    }
    t -= L * nA;
    const unsigned mid = (ng - L) * (nA + nB);
    if (t < mid) {
        const unsigned p = L + t / (nA + nB), r = t % (nA + nB);
        isA = r < nA;
        grp = isA ? p : p - L;
        i = isA ? r : r - nA;
        return;
    }
    t -= mid;
    isA = false;
    grp = ng - L + t / nB;
    i = t % nB;
}

template <int R, int SGN, bool CONJ, bool QA = false>
__global__ __launch_bounds__(512, 4) void k_fused(FArgs a)
{
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    unsigned *sticket = reinterpret_cast<unsigned *>(lds + 4096 + 504);
    const unsigned tid = threadIdx.x;
    const unsigned x = blockIdx.x % NQ;
    constexpr unsigned nA = R * AT / NQ / 2, nB = BT / NQ, AQ = AT / NQ; /* A item = 2 tiles */
    const unsigned total = a.ngroups * (nA + nB);
    unsigned ntk = 0, na = 0, nb = 0, nspin = 0;
    /* last line of defence against a hang: a workgroup older than ~10 s (100 MHz real-time
     * counter) stops taking work and flags the call as failed */
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    constexpr unsigned long long T_LIMIT = 1ull << 30;
    if (tid == 0) *sticket = __hip_atomic_fetch_add(&a.head[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    unsigned t = __builtin_amdgcn_readfirstlane(*sticket);
    __syncthreads();
    while (t < total) {
        /* the next ticket is fetched while this one is processed (its latency hidden); a
         * fetched-but-unstarted A ticket cannot deadlock: every item waits only on items of
         * an earlier queue phase, and this workgroup's current item precedes its next one */
        unsigned tnext = 0;
        if (tid == 0) tnext = __hip_atomic_fetch_add(&a.head[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_s_memrealtime() - t_start > T_LIMIT) {
            if (tid == 0) __hip_atomic_fetch_or(a.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        if (++ntk > total) { /* cannot happen with a working counter: never loop forever */
            if (tid == 0) __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        if (a.dbg && tid == 0) {
            a.dbg[blockIdx.x * 16 + 0] = ntk;
            a.dbg[blockIdx.x * 16 + 1] = t;
        }
        bool isA;
        unsigned grp, i;
        decode<R>(t, a.ngroups, a.lag, isA, grp, i);
        const unsigned long long t_item = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
        if (isA) {
            const unsigned row = grp * R + i / (AQ / 2), k = i % (AQ / 2);
            if constexpr (QA) /* tiles 2k', 2k'+1 as one 4-column group (64-B loads) */
                a_itemq<SGN, CONJ>(a, row, (x * AQ + 2 * k) * 2, lds, tid);
            else
                a_item2<SGN, CONJ>(a, row, x * AQ + k, x * AQ + k + AQ / 2, lds, tid);
            const unsigned long long t_st = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* every storing wave: payload landed */
            if (a.dbg && tid == 0) a.dbg[blockIdx.x * 16 + 10] += (unsigned)(__builtin_amdgcn_s_memrealtime() - t_st);
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(&a.done[grp], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.dbg && tid == 0) {
                a.dbg[blockIdx.x * 16 + 2] = ++na;
                a.dbg[blockIdx.x * 16 + 5] += (unsigned)(__builtin_amdgcn_s_memrealtime() - t_item);
            }
        } else {
            if (tid == 0) {
                const unsigned target = R * AT / 2; /* A items (2 tiles each) of the group */
                unsigned spins = 0;
                while (__hip_atomic_load(&a.done[grp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(2);
                    if (a.dbg) a.dbg[blockIdx.x * 16 + 4] = ++nspin;
                    if (++spins >= a.spin_max || __builtin_amdgcn_s_memrealtime() - t_start > T_LIMIT ||
                        __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keep the sc1 loads below the poll */
            const unsigned long long t_b = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
            if (a.dbg && tid == 0) a.dbg[blockIdx.x * 16 + 7] += (unsigned)(t_b - t_item);
            b_item<R, SGN, CONJ>(a, grp, x * (BT / NQ) + i, lds, tid);
            if (a.dbg && tid == 0) {
                a.dbg[blockIdx.x * 16 + 3] = ++nb;
                a.dbg[blockIdx.x * 16 + 6] += (unsigned)(__builtin_amdgcn_s_memrealtime() - t_b);
            }
        }
        const unsigned long long t_tk = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0;
        if (tid == 0) *sticket = tnext;
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(*sticket);
        __syncthreads();
        if (a.dbg && tid == 0) a.dbg[blockIdx.x * 16 + 11] += (unsigned)(__builtin_amdgcn_s_memrealtime() - t_tk);
    }
}

typedef void (*ffn)(FArgs);

template <int R>
inline ffn fused_fn(int sgn, int conj, bool qa)
{
    if (qa) {
        if (sgn == 1) return conj ? k_fused<R, 1, true, true> : k_fused<R, 1, false, true>;
        return conj ? k_fused<R, -1, true, true> : k_fused<R, -1, false, true>;
    }
    if (sgn == 1) return conj ? k_fused<R, 1, true> : k_fused<R, 1, false>;
    return conj ? k_fused<R, -1, true> : k_fused<R, -1, false>;
}

constexpr size_t LDS_BYTES = (4096 + 504) * sizeof(double2) + 16;

}  // namespace fz
