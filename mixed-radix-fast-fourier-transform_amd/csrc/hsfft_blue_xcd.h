/*
 * hsfft_blue_xcd.h -- Bluestein M = 2^18 = [8,8,8 | 8,8,8] (BASELINE config 4) as ONE
 * persistent launch in which a group of 64 workgroups carries a row through all three of
 * bpf's kernels (hsfft_blue_pf.h: chirped forward first pass, fused middle, chirp-store last
 * pass), handing the two M-point intermediates over inside the launch.
 *
 * Why (measured, round 2, c4 = 99991 x 8192): the three row-looped kernels take 1.24 / 2.11 /
 * 1.52 ms per 1024 rows with the intermediates in HBM, 0.91 / 1.29 / 1.17 ms with every row
 * aliased to one on-die image (HSFFT_DEV_ALIAS=2, timing only) -- 21 vs 31 GSamples/s.  A
 * group holds ONE row in flight (two 4 MiB images), so the eight groups' intermediates (64 MiB)
 * stay in the 256 MiB Infinity Cache instead of crossing HBM twice per row.
 *
 * Geometry: grid = NG x 64 workgroups of 512 threads, two per CU (81.7 KiB LDS each), all
 * co-resident (checked on the host with the occupancy API).  Workgroup w is tile w / NG of
 * group w % NG (under round-robin dispatch group x lives on XCD x when NG == 8: speed only);
 * group x transforms rows x, x + NG, ...  Per row:
 *   P1  columns m0 .. m0+7 of the chirped, zero-padded input  -> image 1 rows m0 .. m0+7
 *   --  group barrier A (all 64 tiles of image 1 written)
 *   P2  q-columns q0 .. q0+7 of image 1: forward second pass, hk product, inverse first pass
 *       -> image 2 rows q0 .. q0+7
 *   --  group barrier B
 *   P3  q-columns of image 2: inverse second pass, chirp product -> output row (n < N)
 * P1 of the next row overwrites image 1 only after barrier B (every P2 read of it is done) and
 * P2 of the next row overwrites image 2 only after the next barrier A (every P3 read is done).
 *
 * The twiddles are loaded once per launch: tw[0, 511) (P1's stages and P2's inverse first
 * pass) and the tile's forward runs (P2; conjugated for P3) in LDS, the tile's stage-2
 * twiddles in registers.
 *
 * Hand-off (cdna_hip_programming.md Guideline 16, recipe R1 -- valid at any number of
 * workgroups per CU): images are written with 16-B sc1 (write-through) stores, every wave
 * waits vmcnt(0), a workgroup barrier, then ONE lane adds 1 (relaxed, agent scope) to the
 * group's counter.  The consumer's lane 0 polls that counter (relaxed agent loads, bounded by
 * a ~1.3 s real-time deadline that sets the sticky error word), then ONE agent-scope acquire
 * (buffer_inv sc1) + vmcnt(0), then the workgroup barrier, then the image loads (sc1 loads,
 * L2-served).  Round 2 ran without the acquire, relying on sc1 loads alone; that form is
 * validated only for one workgroup per CU (MI355X_MICROARCH.md, Valid forms, row 1), and this
 * launch runs two, so the acquire is back.
 *
 * Residency: every workgroup of a group waits on the others, so the whole grid must be
 * resident.  The host checks the occupancy API and refuses a grid that does not fit (its rows
 * run on the three-launch path).  The kernel then PROVES residency with an arrival census
 * (round 6): a group's hand-offs only ever wait on the same group, so every workgroup counts
 * itself into its GROUP's census counter and waits until all 64 tiles of the group have
 * arrived before its first hand-off wait.  The census gives up only when no new member has
 * arrived for `climit` ticks.  Synchronous calls (which re-run a failed launch's rows on the
 * three-launch path themselves) use ~2 ms: a group the occupancy API over-promised
 * (MI355X_MICROARCH.md: the API can report one block per CU too many at some SGPR counts) then
 * fails in ~2 ms instead of after the ~1.3 s hand-off bound.  Asynchronous calls, which cannot
 * re-run, keep the ~1.3 s bound, so a group waiting for slots that a complete group (or a short
 * kernel of another stream) will free is delayed, not failed.  A group whose 64 members are all
 * resident never waits in the census beyond their dispatch, and once its census is complete no
 * hand-off wait of that group can be a residency deadlock.  A failed census or a timed-out wait
 * sets the error word and the kernel exits: a synchronous call re-runs the rows through the
 * three-launch path (hsfft_exec.c run_bluestein), an asynchronous one reports the error at the
 * caller's next hsfft_synchronize().
 *
 * Uneven-load testing: a.jitter > 0 adds a pseudo-random s_sleep (0 .. jitter-1 units of
 * ~4 us) to each workgroup before its arrive and after its wait, per phase -- results are
 * unchanged, the order in which workgroups hand over is scrambled.
 *
 * Arithmetic: the exact operation sequence of k_bfirst / k_bmid / k_blast (pf::stage,
 * r8::exchange, spec, chirp_out) -- bit-identical to them and to the CPU reference
 * (ref src/highSpeedFFT.c:1735-1907).
 */
#pragma once

namespace bxc {

constexpr unsigned long long T_LIMIT = 1ull << 27; /* bounded waits: ~1.3 s of the 100 MHz real-time counter */
constexpr unsigned long long C_LIMIT = 200000;   /* census of a synchronous call: ~2 ms without a new arrival */

constexpr unsigned NTILE = 64;  /* 8-column tiles of the 512 x 512 image = workgroups per group */
constexpr unsigned CS = 32;     /* counter stride (128-B line per counter) */
constexpr unsigned IMG = 512u * 512u; /* points per M-point image */
constexpr unsigned NIMG = 4;          /* images per group: image 1 and image 2, double-buffered */
constexpr size_t LDS_BYTES = (size_t)(512 * 8 + 511 + 504) * 16 + 16;

struct XArgs {
    const double2 *in;
    double2 *out;
    const double2 *tw;    /* plan twiddles of M */
    const double2 *chirp; /* N chirp values */
    const double2 *hk;    /* M transformed chirp values */
    double2 *img;         /* [ng][NIMG][IMG] */
    long long idist, odist;
    unsigned *cnt;        /* [ng][2] hand-off counters, then [ng] census counters, each on its own line (CS apart) */
    unsigned *err;        /* sticky error word (set on a timed-out wait; every wait gives up once it is set) */
    unsigned long long tlimit; /* wait bound in ticks of the 100 MHz real-time counter (T_LIMIT; tests lower it) */
    unsigned long long climit; /* census bound: ticks without a new arrival (C_LIMIT sync, T_LIMIT async) */
    unsigned batch, ng, nsig, sleep;
    unsigned jitter;      /* > 0: pseudo-random per-phase delays (uneven-load tests; results unchanged) */
    unsigned xmap;        /* 1: a group spans the XCDs (XCD x owns tiles [8x, 8x+8) of every group) */
    unsigned *dbg;        /* optional per-workgroup trace (8 words): rows, P1, wait A, P2, wait B, P3 */
};

typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st_sc1(const __amdgpu_buffer_rsrc_t &rs, unsigned voff, unsigned soff, double x, double y)
{
    const double2 v = make_double2(x, y);
    u4 u;
    __builtin_memcpy(&u, &v, 16);
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, voff, soff, 16); /* aux 16 = sc1: write-through */
}

__device__ __forceinline__ double2 ld_sc1(const __amdgpu_buffer_rsrc_t &rs, unsigned voff, unsigned soff)
{
    const u4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 16);
    double2 d;
    __builtin_memcpy(&d, &u, 16);
    return d;
}

/* uneven-load test delay: 0 .. jitter-1 units of s_sleep 64 (~4 us at 1 GHz..2.4 GHz clocks
 * it is 2.7-6.5 us), chosen per (workgroup, phase, row) by a hash; thread 0 sleeps, the
 * barrier that follows holds the rest of the workgroup */
__device__ __forceinline__ void jitter_sleep(const XArgs &a, unsigned k, unsigned ph)
{
    if (a.jitter == 0 || threadIdx.x != 0) return;
    unsigned h = (blockIdx.x * 0x9E3779B1u) ^ (k * 0x85EBCA77u) ^ (ph * 0xC2B2AE3Du);
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    for (unsigned n = h % a.jitter; n; n--) __builtin_amdgcn_s_sleep(64);
}

/* this workgroup's image stores are done: count it in (R1 producer: every storing wave drains
 * its sc1 stores, the barrier, then one lane adds) */
__device__ __forceinline__ void arrive(const XArgs &a, unsigned *c, unsigned k, unsigned ph)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    jitter_sleep(a, k, ph);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* wait until the group's counter c reaches `target` (R1 consumer: one lane polls relaxed, then
 * ONE agent-scope acquire and its vmcnt(0), then the barrier every wave joins before loading);
 * false on timeout (~1.3 s without progress of this one wait) or sticky error.  (Round 4's
 * merged form -- one acquire per iteration when both counters were already complete -- measured
 * +3.9 % slower and was removed in round 6.) */
__device__ __forceinline__ bool await(const XArgs &a, unsigned *c, unsigned target, unsigned *sflag, unsigned k,
                                      unsigned ph)
{
    if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime(); /* deadline per wait */
        unsigned st = 0;
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            for (unsigned n = 0; n < a.sleep; n++) __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.tlimit ||
                __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                st = 1;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); /* buffer_inv sc1: drop this CU's stale L1 lines */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   /* the invalidate has completed */
        *sflag = st;
    }
    jitter_sleep(a, k, ph + 8);
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*sflag) == 0;
}

/* Arrival census of one group: thread 0 counts the workgroup in, then polls the group's census
 * until all `n` members have arrived; false (error word bit 4 set) when no member arrived for
 * climit ticks, or when the error word is set (a workgroup gave up, possibly before this one was
 * dispatched).  Relaxed atomics: the census orders no data (the hand-offs acquire their own). */
__device__ __forceinline__ bool census(const XArgs &a, unsigned *cs, unsigned n, unsigned *sflag)
{
    if (threadIdx.x == 0) {
        unsigned st = 0;
        unsigned seen = __hip_atomic_fetch_add(cs, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (seen < n) {
            for (unsigned n = 0; n < a.sleep; n++) __builtin_amdgcn_s_sleep(2);
            if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                st = 1;
                break;
            }
            const unsigned now = __hip_atomic_load(cs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if (now != seen) { /* progress: the bound restarts */
                seen = now;
                t0 = t;
            } else if (t - t0 > a.climit) {
                __hip_atomic_fetch_or(a.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                st = 1;
                break;
            }
        }
        if (!st && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) st = 1;
        *sflag = st;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*sflag) == 0;
}

/* Round 5: every load of P1 (input row, chirp) and P3 (chirp) is issued unconditionally at a
 * clamped index, the zero padding / the n < N store condition applied to the VALUES -- with the
 * n < nsig test around the loads hipcc branched around each one and waited vmcnt(0) after it
 * (cdna_hip_programming.md, the per-element "register or load" trap): P3's eight chirp loads
 * each waited for the previous element's store, P1's row loads one by one.  Same arithmetic on
 * the same values (bit-identical); in-process A/B on two boxes 32.40 vs 32.62 and 32.08 vs 32.35
 * ms per 8192 rows (profiles/r05e_*, r05f_*). */
template <int S>
__global__ __launch_bounds__(512, 4) void k_bxcd(XArgs a)
{
    constexpr int P = 512, TPG = 64, G = 8;
    constexpr unsigned A = 512, B = 512;
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    double2 *t0 = lds + P * G; /* tw[0, 511): stages L = 8, 64 of a first pass */
    double2 *run = t0 + 511;   /* the tile's forward runs at L = B and 8B (bpf::runs_to_lds) */
    unsigned *sflag = reinterpret_cast<unsigned *>(run + 504);
    /* block -> (group, tile).  xmap 0: group = blockIdx % ng (ng == 8: one XCD per group under
     * round-robin dispatch).  xmap 1: 64 consecutive blocks form a group and XCD x = blockIdx % 8
     * owns tiles [8x, 8x+8) of every group, so the hk / chirp slices an XCD reads are 1/8 of
     * them (L2-resident) while the images cross the fabric either way.  Speed only. */
    const unsigned ng = a.ng;
    unsigned grp, tile;
    if (a.xmap) {
        const unsigned x = blockIdx.x % 8, r = blockIdx.x / 8;
        tile = x * 8 + r % 8;
        grp = r / 8;
    } else {
        grp = blockIdx.x % ng;
        tile = blockIdx.x / ng;
    }
    const unsigned tid = threadIdx.x, q0 = tile * G;
    const unsigned nsig = a.nsig;

    /* per-launch state: the tile's stage-2 twiddles (redistributed through the image); the
     * chirp and hk values are re-read per row (L2 / Infinity-Cache hits; in registers they
     * would spill) */
    double2 w2[7];
    {
        r8::Args ta;
        ta.tw = a.tw;
        ta.B = B;
        r8::load_tw_co<64>(w2, ta, (int)(tid / G), q0);
    }
    if (tid < 511) t0[tid] = a.tw[tid];
    bpf::runs_to_lds<false>(run, a.tw, B, q0, tid);
    r8::redistribute_tw(w2, lds);
    __syncthreads();

    double2 *imgs = a.img + (size_t)grp * NIMG * IMG; /* image 1 [2], image 2 [2] */
    unsigned *cA = a.cnt + (size_t)grp * 2 * CS, *cB = cA + CS;
    const unsigned R = grp < a.batch ? (a.batch - grp + ng - 1) / ng : 0; /* this group's rows */
    if (R && !census(a, a.cnt + (size_t)(2 * ng + grp) * CS, NTILE, sflag)) return;
    unsigned tr[8] = {0, 0, 0, 0, 0, 0, 0, 0}; /* debug: rows, P1, wait A, P2, wait B, P3, P1 / P2 store drain (10 ns) */

    /* skewed pipeline: iteration k runs P3 of row k-2, P2 of row k-1, P1 of row k, so every
     * barrier a phase waits for was signalled one phase earlier (the group has had a whole
     * phase to arrive).  Images are double-buffered by row parity:
     *   P1(k) overwrites image 1 [k&1], last read by P2(k-2): done once B(k-2) is complete,
     *     which this workgroup awaited before P3(k-2) in this iteration;
     *   P2(k-1) overwrites image 2 [(k-1)&1], last read by P3(k-3): every workgroup counts
     *     itself into A(k-1) only after its P3(k-3), so A(k-1) -- awaited before P2(k-1) --
     *     covers it.
     * (Measured: the image stores take ~2.4 us per phase to drain before the arrive; deferring
     * the arrive behind the next phase's loads did not hide it -- 24.6 vs 25.5 GSamples/s.) */
#pragma unroll 1
    for (unsigned k = 0; k < R + 2; k++) {
        unsigned tk = a.dbg ? (unsigned)__builtin_amdgcn_s_memrealtime() : 0;
#define BX_MARK(i)                                                              \
    if (a.dbg) {                                                                \
        const unsigned tn = (unsigned)__builtin_amdgcn_s_memrealtime();         \
        tr[i] += tn - tk;                                                       \
        tk = tn;                                                                \
    }
        double xr[8], xi[8];
        double2 w[7];
        if (k >= 2) { /* ---- P3 of row k-2: k_blast's body on image 2 [k&1], chirp store */
            if (!await(a, cB, (k - 1) * NTILE, sflag, k, 0)) return;
            BX_MARK(4)
            /* per-thread indices from an opaque copy of threadIdx in every phase, so the
             * compiler does not hoist all three phases' addresses out of the loop (spills) */
            unsigned tt = tid;
            asm volatile("" : "+v"(tt));
            const unsigned g = tt % G, jt = tt / G, q = q0 + g;
            const unsigned col = (jt * B + q) * 16u;
            const __amdgpu_buffer_rsrc_t r2 =
                __builtin_amdgcn_make_buffer_rsrc(imgs + (2 + (k & 1)) * (size_t)IMG, 0, (int)(IMG * 16u), 0x00020000);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = ld_sc1(r2, col, i * TPG * B * 16);
                xr[i] = v.x;
                xi[i] = v.y;
            }
#pragma unroll
            for (int i = 0; i < 7; i++) {
                const double2 v = run[7 * g + i];
                w[i] = make_double2(v.x, -v.y);
            }
            pf::stage<8, -S>(xr, xi, w, false);
            r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
#pragma unroll
            for (int i = 0; i < 7; i++) {
                const double2 v = run[56 * (1 + (jt & 7)) + 7 * g + i];
                w[i] = make_double2(v.x, -v.y);
            }
            pf::stage<8, -S>(xr, xi, w, false);
            r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
#pragma unroll
            for (int i = 0; i < 7; i++) w[i] = make_double2(w2[i].x, -w2[i].y);
            pf::stage<8, -S>(xr, xi, w, false);
            double2 *orow = a.out + (long long)(grp + (k - 2) * ng) * a.odist;
            /* the chirp values of four outputs at a time, loaded together */
#pragma unroll
            for (int h4 = 0; h4 < 8; h4 += 4) {
                double2 ch[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const unsigned n = (jt + (h4 + u) * TPG) * B + q;
                    ch[u] = a.chirp[n < nsig ? n : nsig - 1];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const unsigned n = (jt + (h4 + u) * TPG) * B + q;
                    if (n < nsig) orow[n] = bpf::chirp_out<S>(xr[h4 + u], xi[h4 + u], ch[u]);
                }
            }
            BX_MARK(5)
            tr[0]++;
        }
        if (k >= 1 && k <= R) { /* ---- P2 of row k-1: k_bmid's body, image 1 -> image 2 [(k-1)&1] */
            if (!await(a, cA, k * NTILE, sflag, k, 1)) return;
            BX_MARK(2)
            unsigned tt = tid;
            asm volatile("" : "+v"(tt));
            const unsigned g = tt % G, jt = tt / G, q = q0 + g;
            const unsigned col = (jt * B + q) * 16u, rowo = (q * P + jt) * 16u;
            const unsigned par = (k - 1) & 1;
            const __amdgpu_buffer_rsrc_t r1 =
                __builtin_amdgcn_make_buffer_rsrc(imgs + par * (size_t)IMG, 0, (int)(IMG * 16u), 0x00020000);
            const __amdgpu_buffer_rsrc_t r2 =
                __builtin_amdgcn_make_buffer_rsrc(imgs + (2 + par) * (size_t)IMG, 0, (int)(IMG * 16u), 0x00020000);
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = ld_sc1(r1, col, i * TPG * B * 16);
                xr[i] = v.x;
                xi[i] = v.y;
            }
#pragma unroll
            for (int i = 0; i < 7; i++) w[i] = run[7 * g + i];
            pf::stage<8, S>(xr, xi, w, false);
            r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
            double2 hko[8]; /* issued after the first exchange: fewer live registers */
#pragma unroll
            for (int i = 0; i < 8; i++) hko[i] = pf::ldg(a.hk + (size_t)i * TPG * B, col);
#pragma unroll
            for (int i = 0; i < 7; i++) w[i] = run[56 * (1 + (jt & 7)) + 7 * g + i];
            pf::stage<8, S>(xr, xi, w, false);
            r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
            pf::stage<8, S>(xr, xi, w2, false);
#pragma unroll
            for (int jj = 0; jj < 8; jj++) bpf::spec<S>(xr[jj], xi[jj], hko[jj]);
            pf::stage<8, -S>(xr, xi, w, true);
            r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
            pf::tw8_lds<true>(w, t0, 8, jt & 7);
            pf::stage<8, -S>(xr, xi, w, false);
            r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
            pf::tw8_lds<true>(w, t0, 64, jt & 63);
            pf::stage<8, -S>(xr, xi, w, false);
#pragma unroll
            for (int jj = 0; jj < 8; jj++) st_sc1(r2, rowo, jj * TPG * 16, xr[jj], xi[jj]);
            BX_MARK(3)
            arrive(a, cB, k, 2);
            BX_MARK(7)
        }
        if (k < R) { /* ---- P1 of row k: k_bfirst's body (columns m = q) -> image 1 [k&1] */
            unsigned tt = tid;
            asm volatile("" : "+v"(tt));
            const unsigned g = tt % G, jt = tt / G, q = q0 + g;
            const unsigned rowo = (q * P + jt) * 16u;
            const __amdgpu_buffer_rsrc_t r1 =
                __builtin_amdgcn_make_buffer_rsrc(imgs + (k & 1) * (size_t)IMG, 0, (int)(IMG * 16u), 0x00020000);
            const double2 *row = a.in + (long long)(grp + k * ng) * a.idist;
            double2 hin[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const unsigned n = (jt + i * TPG) * A + q;
                hin[i] = a.chirp[n < nsig ? n : 0];
            }
            /* every row load issued, the padding applied to the values */
            double2 x4[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const unsigned n = (jt + i * TPG) * A + q;
                x4[i] = row[n < nsig ? n : nsig - 1];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const unsigned n = (jt + i * TPG) * A + q;
                const double2 x = x4[i];
                double2 v;
                if (S == 1) v = make_double2(x.x * hin[i].x + x.y * hin[i].y, -x.x * hin[i].y + x.y * hin[i].x);
                else v = make_double2(x.x * hin[i].x - x.y * hin[i].y, x.x * hin[i].y + x.y * hin[i].x);
                const bool inside = n < nsig;
                xr[i] = inside ? v.x : 0.0;
                xi[i] = inside ? v.y : 0.0;
                xr[i + 4] = 0.0;
                xi[i + 4] = 0.0;
            }
            pf::stage<8, S>(xr, xi, w, true);
            r8::exchange<8, 1, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
#pragma unroll
            for (int i = 0; i < 7; i++) w[i] = t0[7 + 7 * (jt & 7) + i];
            pf::stage<8, S>(xr, xi, w, false);
            r8::exchange<8, 8, 8, TPG, P, G, false>(xr, xi, lds, jt, g);
#pragma unroll
            for (int i = 0; i < 7; i++) w[i] = t0[63 + 7 * (jt & 63) + i];
            pf::stage<8, S>(xr, xi, w, false);
#pragma unroll
            for (int jj = 0; jj < 8; jj++) st_sc1(r1, rowo, jj * TPG * 16, xr[jj], xi[jj]);
            BX_MARK(1)
            arrive(a, cA, k, 3);
            BX_MARK(6)
        }
    }
#undef BX_MARK
    if (a.dbg && threadIdx.x == 0) {
        unsigned *d = a.dbg + blockIdx.x * 8;
        for (int i = 0; i < 8; i++) d[i] = tr[i];
    }
}

}  // namespace bxc
