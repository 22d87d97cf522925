/*
 * hsfft_fused2.h -- 2^20 = [4,8,8,8 | 8,8,8] (BASELINE config 2) as ONE persistent launch
 * with fixed workgroup roles, the pass-A -> pass-B intermediate handed over inside the
 * launch so that it stays in the 256 MiB Infinity Cache and HBM sees ~32 B per sample.
 *
 * Why fixed roles (measured, round 2, 4096 x 2^20, every row aliased to one 16 MiB buffer so
 * nothing waits on HBM): pass A (pf::k_firstq, 64-B paired column loads) is held by its
 * column-segment request rate -- 22.4 ms with two workgroups per CU, 24.7 ms with ONE;
 * pass B (pf::k_b512) is held by on-die bandwidth -- 15.1 ms with two, 13.4 ms with one.
 * The two limits are different units, so one pass-A workgroup and one pass-B workgroup per
 * CU can overlap where two workgroups of the same pass cannot.
 *
 *   A role (blockIdx < na): keeps tw[0, 2047) in LDS for the whole launch and takes pass-A
 *     items (one 4-column group of one row, pf::k_firstq's body) from NQ = 8 ticket queues;
 *     queue x serves column groups [16x, 16x + 16) of every row in row order, so the
 *     workgroups sharing a 128-B input line take their items together (one XCD under
 *     round-robin dispatch: speed only).  Results are stored write-through (sc1).
 *   B role (blockIdx >= na): owns q-tiles b, b + nb, ... (8 q-columns each) for the whole
 *     launch, so its stage twiddles are loaded once, and walks the rows in order: waits
 *     until the row's 128 pass-A items are done, reads its columns with sc1 loads,
 *     transforms them ([8,8,8], pf::k_b512's body) and writes the output in place.
 *
 * Hand-off (MI355X_MICROARCH.md visibility table, row 1): every storing wave waits
 * vmcnt(0), a workgroup barrier, then one lane adds 1 (relaxed, agent scope) to the row's
 * counter; the consumer polls it with relaxed agent loads, joins a barrier, and reads the
 * intermediate only with 16-B sc1 loads.
 *
 * Progress: A-role workgroups never wait on anything but a bounded throttle (they stay at
 * most `lag` rows ahead of the B roles to keep the intermediate on die; the throttle gives
 * up after spin_max polls), so every pass-A item completes; they have the lower block ids,
 * so they are dispatched first.  B waits are bounded by a ~10 s real-time deadline that
 * sets a sticky error word (the call then fails instead of hanging).
 *
 * Arithmetic: pf::stage / hsfft_butterfly.h, the plan's own twiddles -- bit-identical to the
 * two-launch path and to the CPU reference.
 */
#pragma once

namespace fz2 {

constexpr int NQ = 8;                 /* A ticket queues */
constexpr unsigned AG = 128;          /* 4-column pass-A groups per row */
constexpr unsigned QT = 256;          /* 8-column pass-B tiles per row */
constexpr unsigned ROW_BYTES = (1u << 20) * 16u;
constexpr unsigned long long T_LIMIT = 1ull << 30; /* ~10 s of the 100 MHz real-time counter */
constexpr unsigned CS = 32;           /* counter stride: every counter on a 128-B line of its own */

struct F2Args {
    const double2 *in;
    double2 *out;
    const double2 *tw;
    long long idist, odist;
    unsigned *head;  /* [NQ * CS] ticket heads */
    unsigned *err;   /* sticky error word */
    unsigned *adone; /* [batch * CS] finished pass-A items per row */
    unsigned *bdone; /* [batch * CS] finished pass-B tiles per row (throttle only) */
    unsigned batch, na, nb, lag, spin_max, sleep;
    unsigned *dbg;   /* optional per-workgroup trace (8 words): items, busy, wait, first, last */
};

constexpr size_t LDS_BYTES = (4096 + 504) * sizeof(double2) + 16;

/* The kernels below are compiled in their own translation unit (hsfft_device_fz2.hip, which
 * defines HSFFT_FZ2_KERNELS): instantiated next to the production passes in
 * hsfft_device.hip, they changed the register allocation of pf::k_firstq<4,3,2> (128 VGPRs
 * + 4 dwords of spill instead of none). */
#ifdef HSFFT_FZ2_KERNELS
__device__ __forceinline__ unsigned now32() { return (unsigned)__builtin_amdgcn_s_memrealtime(); }

/* polling pause: `n` x s_sleep 4 (~4 x 64 clocks each) */
__device__ __forceinline__ void nap(unsigned n)
{
    for (unsigned k = 0; k < n; k++) __builtin_amdgcn_s_sleep(4);
}

__device__ __forceinline__ double2 as_d2(fz::u32x4 v)
{
    double2 d;
    __builtin_memcpy(&d, &v, 16);
    return d;
}

template <int SGN, bool CONJ, bool ASC1 = true, bool NTL = false>
__device__ __forceinline__ void a_role(const F2Args &a, double2 *lds, unsigned *sticket)
{
    constexpr int P = 2048, TPG = 256;
    double2 *ltw = lds + 2048; /* after the 32 KiB split exchange image */
    const unsigned tid = threadIdx.x, x = blockIdx.x % NQ;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (int i = tid; i < P - 1; i += 512) ltw[i] = a.tw[i];
    const unsigned total = a.batch * (AG / NQ);
    if (tid == 0) *sticket = __hip_atomic_fetch_add(&a.head[x * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    unsigned t = __builtin_amdgcn_readfirstlane(*sticket);
    __syncthreads();
    unsigned guard = 0;
#pragma unroll 1
    while (t < total && ++guard <= total) {
        unsigned tnext = 0;
        if (tid == 0) tnext = __hip_atomic_fetch_add(&a.head[x * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned row = t / (AG / NQ), m0 = (x * (AG / NQ) + t % (AG / NQ)) * 4;
        const unsigned ti = a.dbg ? now32() : 0;
        unsigned tw_ = ti;
        if (row >= a.lag && tid == 0) { /* throttle: stay within `lag` rows of pass B */
            unsigned spins = 0;
            while (__hip_atomic_load(&a.bdone[(row - a.lag) * CS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < QT &&
                   ++spins < a.spin_max)
                nap(a.sleep);
            if (a.dbg) tw_ = now32();
        }
        /* pf::k_firstq's item: 64-B paired loads of columns m0 .. m0+3 */
        unsigned tt = tid;
        asm volatile("" : "+v"(tt));
        const unsigned h = tt & 1, jt = tt >> 1, odd = jt & 1;
        const double2 *in = a.in + (long long)row * a.idist;
        double2 *orow = a.out + (long long)row * a.odist;
        const unsigned offA = ((jt - odd) * 512u + m0 + h + 2 * odd) * 16u;
        const unsigned offB = ((jt + 1 - odd) * 512u + m0 + h + 2 - 2 * odd) * 16u;
        double2 va[8], vb[8];
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const double2 *rb = in + (size_t)(c * TPG + i * (P / 4)) * 512;
                va[c * 4 + i] = NTL ? pf::ldg_nt(rb, offA) : pf::ldg(rb, offA);
                vb[c * 4 + i] = NTL ? pf::ldg_nt(rb, offB) : pf::ldg(rb, offB);
            }
        __syncthreads(); /* the throttle poll (lane 0) and the previous item's LDS use are done */
        double xr[8], xi[8], yr[8], yi[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const double2 own = odd ? vb[k] : va[k], oth = odd ? va[k] : vb[k];
            xr[k] = own.x;
            xi[k] = own.y;
            yr[k] = pf::pair_swap<2>(oth.x);
            yi[k] = pf::pair_swap<2>(oth.y);
        }
        pf::first_body<4, 3, 2, SGN, CONJ, ASC1>(xr, xi, lds, ltw, orow, m0 + h, jt, h);
        pf::first_body<4, 3, 2, SGN, CONJ, ASC1>(yr, yi, lds, ltw, orow, m0 + 2 + h, jt, h);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* this wave's write-through stores landed */
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(&a.adone[row * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *sticket = tnext;
            if (a.dbg) { /* items, throttle wait, item time, first start, last end */
                unsigned *d = a.dbg + blockIdx.x * 8;
                const unsigned te = now32();
                d[0] += 1;
                d[1] += tw_ - ti;
                d[2] += te - tw_;
                if (d[0] == 1) d[3] = ti;
                d[4] = te;
            }
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(*sticket);
        if (__builtin_amdgcn_s_memrealtime() - t0 > T_LIMIT) {
            if (tid == 0) __hip_atomic_fetch_or(a.err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        __syncthreads();
    }
}

template <int SGN, bool CONJ, bool BSC1 = true, bool NTS = false>
__device__ __forceinline__ void b_role(const F2Args &a, double2 *lds, unsigned *sflag)
{
    constexpr int TPG = 64, G = 8;
    constexpr unsigned B = 2048;
    double2 *ltw = lds + 4096; /* after the 64 KiB exchange image */
    const unsigned tid = threadIdx.x, bid = blockIdx.x - a.na;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (unsigned qt = bid; qt < QT; qt += a.nb) {
        const unsigned q0 = qt * G;
        /* stage-2 twiddles in registers, stage-0/1 runs in LDS (pf::k_b512) */
        r8::Args ta;
        ta.tw = a.tw;
        ta.B = B;
        double2 w2[7];
        __syncthreads(); /* the previous tile's image readers are done */
        r8::load_tw_co<64>(w2, ta, (int)(tid / G), q0);
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
#pragma unroll 1
        for (unsigned row = 0; row < a.batch; row++) {
            const unsigned ti = a.dbg ? now32() : 0;
            if (tid == 0) {
                unsigned bad = 0;
                while (__hip_atomic_load(&a.adone[row * CS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < AG) {
                    nap(a.sleep);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > T_LIMIT ||
                        __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        bad = 1;
                        break;
                    }
                }
                *sflag = bad;
            }
            __syncthreads();
            const unsigned tw_ = a.dbg ? now32() : 0;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); /* keep the sc1 loads below the poll */
            if (__builtin_amdgcn_readfirstlane(*sflag)) return;
            unsigned tt = tid;
            asm volatile("" : "+v"(tt));
            const unsigned g = tt & 7, jt = tt >> 3;
            const unsigned lane = (jt * B + q0 + g) * 16u;
            double2 *orow = a.out + (long long)row * a.odist;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(orow, 0, (int)ROW_BYTES, 0x00020000);
            double xr[8], xi[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const double2 v = as_d2(__builtin_amdgcn_raw_buffer_load_b128(rs, lane, i * TPG * B * 16, BSC1 ? 16 : 0));
                xr[i] = v.x;
                xi[i] = v.y;
            }
            pf::b512_body<SGN, NTS>(xr, xi, w2, lds, ltw, orow, B, lane, jt, g);
            if (tid == 0) __hip_atomic_fetch_add(&a.bdone[row * CS], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.dbg && tid == 0) { /* rows, wait for pass A, row time, first start, last end */
                unsigned *d = a.dbg + blockIdx.x * 8;
                const unsigned te = now32();
                d[0] += 1;
                d[1] += tw_ - ti;
                d[2] += te - tw_;
                if (d[0] == 1) d[3] = ti;
                d[4] = te;
            }
        }
    }
}

/* PLAIN: timing probe only (HSFFT_FZ2_PLAIN): bit 0 pass-A stores, bit 1 pass-B loads
 * without sc1 -- NOT a valid hand-off across XCDs */
template <int SGN, bool CONJ, int PLAIN = 0, int NT = 0>
__global__ __launch_bounds__(512, 4) void k_fused2(F2Args a)
{
    extern __shared__ __attribute__((aligned(16))) double2 lds[];
    unsigned *scal = reinterpret_cast<unsigned *>(lds + 4096 + 504);
    if (blockIdx.x < a.na) a_role<SGN, CONJ, !(PLAIN & 1), (NT & 1) != 0>(a, lds, scal);
    else b_role<SGN, CONJ, !(PLAIN & 2), (NT & 2) != 0>(a, lds, scal);
}

typedef void (*ffn)(F2Args);

inline ffn fused2_fn(int sgn, int conj, int plain = 0, int nt = 0)
{
    /* NT (HSFFT_FZ2_NT): bit 0 pass-A input loads, bit 1 pass-B output stores non-temporal */
    if (nt == 1) return sgn == 1 ? (conj ? k_fused2<1, true, 0, 1> : k_fused2<1, false, 0, 1>)
                                 : (conj ? k_fused2<-1, true, 0, 1> : k_fused2<-1, false, 0, 1>);
    if (nt == 2) return sgn == 1 ? (conj ? k_fused2<1, true, 0, 2> : k_fused2<1, false, 0, 2>)
                                 : (conj ? k_fused2<-1, true, 0, 2> : k_fused2<-1, false, 0, 2>);
    if (nt == 3) return sgn == 1 ? (conj ? k_fused2<1, true, 0, 3> : k_fused2<1, false, 0, 3>)
                                 : (conj ? k_fused2<-1, true, 0, 3> : k_fused2<-1, false, 0, 3>);
    if (plain == 3) return sgn == 1 ? k_fused2<1, false, 3> : k_fused2<-1, false, 3>;
    if (plain == 2) return sgn == 1 ? k_fused2<1, false, 2> : k_fused2<-1, false, 2>;
    if (plain == 1) return sgn == 1 ? k_fused2<1, false, 1> : k_fused2<-1, false, 1>;
    if (sgn == 1) return conj ? k_fused2<1, true> : k_fused2<1, false>;
    return conj ? k_fused2<-1, true> : k_fused2<-1, false>;
}

#endif /* HSFFT_FZ2_KERNELS */

}  // namespace fz2
