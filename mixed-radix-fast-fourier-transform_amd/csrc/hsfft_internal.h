/*
 * hsfft_internal.h -- internal interface between the C host side (planner, drop-in API,
 * scheduler) and the HIP/CDNA4 device layer (hsfft_device.hip).  Not installed.
 *
 * Execution model: the reference recursion is replaced by a
 * Stockham autosort schedule.  Stage s (innermost first) has radix r_s and global
 * L_s = r_0...r_{s-1}; after it, sub-transform m (of length L_s*r_s) sits at
 * [m*L_s*r_s, (m+1)*L_s*r_s).  Consecutive stages are fused into passes; a pass of P points
 * with L0 = B at its start views its input as [t][m][q] (P x A x B, A = M/(B*P)) and writes
 * [m][u][q]: a P-point sub-FFT along t for every (m, q), using the plan's global twiddles
 * tw[L-1 + (r-1)*k + i-1] with k = q + B*k_local.
 */
#ifndef HSFFT_INTERNAL_H_
#define HSFFT_INTERNAL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HS_MAX_STAGES 64
#define HS_MAX_PASS_STAGES 12
#define HS_MAX_PASSES 16
#define HS_MAX_DEV 16

/* kernel variants */
#define HS_KV_GENERIC 0   /* runtime radix list, LDS ping-pong */
#define HS_KV_R8X3 1      /* specialised: 8*8*8 or tails, register butterflies */
#define HS_KV_MR 2        /* specialised mixed radix list (hsfft_pass_mr.h), else generic */

/* load / store hooks of a pass (Bluestein fusion) */
#define HS_LOAD_PLAIN 0
#define HS_LOAD_CHIRP 1   /* x[n]*conj-chirp for n < nsig, 0 for n >= nsig (:1803-1827) */
#define HS_STORE_PLAIN 0
#define HS_STORE_SPEC 1   /* y[n]*hk[n] (:1838-1855) */
#define HS_STORE_CHIRP 2  /* y[n]*chirp for n < nsig only (:1871-1886) */

typedef struct {
    int nst;                        /* stages fused in this pass */
    int radix[HS_MAX_PASS_STAGES];  /* innermost first */
    int gcs_off[HS_MAX_PASS_STAGES];/* generic-radix constant offsets (doubles) or -1 */
    int P;                          /* points per group */
    int leaf;                       /* first stage is the reference leaf (global L == 1) */
    long long B;                    /* L at pass start */
    long long A;                    /* M / (B*P) */
    int Wm, Wq, G;                  /* tile: Wm m-values x Wq q-values, G = Wm*Wq groups */
    int variant;                    /* HS_KV_* */
} hsd_pass;

typedef struct {
    const void *in;
    void *out;
    long long idist, odist;         /* batch strides in complex elements */
    int batch;
    int sgn;                        /* butterfly sign of this transform */
    int dir;                        /* Bluestein transform_direction for the hooks */
    int conj;                       /* negate twiddle imaginary parts */
    const void *tw;
    const double *gcs;
    int load_op, store_op;
    const void *load_aux, *store_aux;
    long long nsig;
    int tw_t;                       /* 1: tw + M holds the last stage's block transposed ([i-1][k]) */
    /* completion word (small host-buffer calls): a kernel that runs as ONE workgroup stores
     * done_val into *done (page-locked host memory) after every wave published its output at
     * system scope, and the device layer sets *armed; other launches ignore it */
    unsigned *done;
    unsigned done_val;
    int *armed;
} hsd_launch;

/* device layer (hsfft_device.hip) */
int hsd_device_count(void);
int hsd_set_device(int dev);
int hsd_get_device(void);
void *hsd_malloc(size_t bytes);
int hsd_free(void *p);
int hsd_h2d(void *d, const void *h, size_t bytes);
int hsd_d2h(void *h, const void *d, size_t bytes);
int hsd_d2d_async(void *d, const void *s, size_t bytes);
int hsd_memset_async(void *d, int v, size_t bytes);
int hsd_sync(void);               /* wait for the library stream (a pending launch error stays pending) */
int hsd_sync_report(void);        /* the same, then report this thread's pending persistent-launch error */
/* release every device object of the device layer on the current device (streams, events,
 * persistent-launch counters, this thread's error words); re-created on demand */
int hsd_finalize_device(void);
int hsd_select_stream(int idx);   /* 0 library stream, 1 pipeline / H2D, 2 D2H, 3 this thread's own stream */
int hsd_stream_index(void);       /* the calling thread's selected stream */
int hsd_h2d_async(void *d, const void *h, size_t bytes);   /* on the selected stream */
int hsd_d2h_async(void *h, const void *d, size_t bytes);
int hsd_stream_sync(void);        /* the selected stream */
/* completion of the selected stream's work through a page-locked word the host polls
 * (flag from hsd_host_alloc, v a fresh value), stream wait as the fallback */
int hsd_stream_signal_wait(unsigned *flag, unsigned v);
/* the same for a word a kernel stores itself (hsd_launch.done) */
int hsd_host_word_wait(unsigned *flag, unsigned v);
int hsd_host_register(void *p, size_t bytes);
int hsd_host_unregister(void *p);
void *hsd_host_alloc(size_t bytes);  /* page-locked, device-accessible host memory */
int hsd_host_free(void *p);
/* Per-thread resources of one device, recycled (round 6).  A thread's own stream and
 * persistent-launch error words (device layer) and its page-locked staging slots and completion
 * word (host side, `hsd_tset`) form one set per device.  At thread exit the set is PARKED in the
 * device's pool -- no HIP call: the exit destructor runs when the runtime's (and a profiler's)
 * per-thread state may be gone (round 5: rocprofv3 aborted the process there).  A thread's first
 * use of a device ADOPTS a parked set, again without a HIP call, so threads that come and go
 * (thread pools, hsfft_exec_multi's shard threads) reuse streams and pinned memory instead of
 * creating and destroying them on a live caller's path.  Sets are destroyed only by
 * hsd_pool_drain (hsfft_release_scratch, hsfft_finalize). */
typedef struct {
    void *pin[2];     /* page-locked in / out slots of the small path (hsd_host_alloc) */
    size_t pin_sz;    /* bytes of each slot */
    unsigned *flag;   /* page-locked completion word (hsd_host_alloc) */
    unsigned seq;     /* the last value the word was set to (the next owner continues after it) */
} hsd_tset;
void hsd_thread_park(int dev, const hsd_tset *h); /* thread exit: this thread's set of `dev` */
int hsd_thread_adopt(int dev, hsd_tset *h);       /* 1: a parked set was taken (host part in *h) */
int hsd_pool_drain(void); /* destroy every parked set, every device (streams waited first); returns the count */
long long hsd_thread_streams_created(void); /* per-thread streams created so far (diagnostics) */
int hsd_event_record(int i);      /* event ring (64 slots) on the selected stream */
int hsd_event_wait(int i);
void *hsd_stream(void);
int hsd_is_device_ptr(const void *p);
const char *hsd_errstr(void);
/* host side (hsfft_exec.c): getenv, served from a per-call snapshot inside the small fft_exec path */
const char *hs_getenv(const char *name);
void hs_env_begin(void); /* (the snapshot's scope; tests/sanitize checks its semantics) */
void hs_env_end(void);

int hsd_run_pass(const hsd_pass *p, const hsd_launch *l);
/* 1 if the register kernel has an instantiation for [r0, 8^n8] with this tile */
int r8_has_variant(int r0, int n8, int G, int Wq, int first);
int mr_has_variant(const hsd_pass *p);
/* r2c: last c2c pass ([8,8,8], A == 1) + the real.c split in one kernel; compact: rows of
 * h+1 bins (hsfft_r2c_batched_compact) instead of the mirrored N */
int hsd_r2c_last(const void *Z, long long zdist, void *X, long long xdist, const void *tw, const void *w2, long long h,
                 long long B, int batch, int sgn, int compact);
/* Bluestein M = 2^18 in one persistent launch (hsfft_blue_xcd.h); sync 0 asynchronous, 1
 * synchronous, 2 deferred (asynchronous, the outcome read later by hsd_blue_deferred_take):
 * 0 queued / done, 1 not applicable, 2 (sync) in-launch waits timed out, 3 grid not co-resident
 * (re-run the rows elsewhere in both), < 0 HIP error.  Asynchronous: a timed-out wait is
 * reported by the launching thread's next hsd_sync_report. */
int hsd_blue_xcd(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                 const void *hk, void *img, size_t img_bytes, long long nsig, int batch, int sgn, int ng, int sync);
/* 1 if a deferred launch (sync 2) of this thread on the current device timed out since the last
 * call (call after waiting for the library stream); clears the word */
int hsd_blue_deferred_take(void);
/* Bluestein M = 2^18: forward last pass + hk product + inverse first pass in one kernel */
int hsd_blue_mid(const void *in, void *out, long long dist, const void *tw, const void *hk, int batch, int sgn,
                 int conj, int dir, int sgn2, int conj2); /* hsfft_pass_mr.h has a kernel for this pass */
/* Bluestein M = 2^18: inverse last pass stored through the chirp (rows of M -> rows of N);
 * 1 if the row-looped kernel is disabled (caller runs the generic pass) */
int hsd_blue_last(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                  long long nsig, int batch, int dir);
/* Bluestein M = 2^18: forward first pass on the chirped input (rows of N -> rows of M) */
int hsd_blue_first(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                   long long nsig, int batch, int dir);
int hsd_fill_complex(void *d, int64_t count, uint64_t seed, uint64_t offset);
int hsd_fill_real(void *d, int64_t count, uint64_t seed, uint64_t offset);
/* r2c split (real.c:108-132): Z rows of h complex -> X rows of 2h complex */
int hsd_r2c_post(const void *Z, const void *tw2, void *X, int h, int batch, long long zdist, long long xdist);
/* the same split writing bins 0..h only: X rows of h+1 complex */
int hsd_r2c_post_compact(const void *Z, const void *tw2, void *X, int h, int batch, long long zdist, long long xdist);
/* c2r pre-twiddle (real.c:169-179): X rows (>= h+1 complex) -> Zin rows of h complex */
int hsd_c2r_pre(const void *X, const void *tw2, void *Zin, int h, int batch, long long xdist, long long zdist);
/* convolution helpers (convolve.c:147-160) */
int hsd_cmul(const void *A, const void *Bv, void *C, long long n, int batch, long long dist);
/* convolution: spectral product fused into the c2r pre-twiddle; scale fused into the window copy */
int hsd_c2r_pre_mul(const void *A, const void *Bv, const void *tw2, void *Zin, int h, int batch, long long xdist,
                    long long zdist);
int hsd_copy_rows_div(const void *src, long long sdist, long long soff, void *dst, long long ddist, long long n,
                      int batch, double divisor);
int hsd_scale_real(void *x, long long n, int batch, long long dist, double divisor);
int hsd_copy_rows(const void *src, long long sdist, long long soff, long long ncopy, void *dst, long long ddist,
                  long long dlen, int batch);

int hsd_cu_count(void);
/* differing 8-byte words of two device buffers (synchronous) */
int hsd_count_diff(const void *a, const void *b, long long nwords, unsigned long long *count);

/* timing on the library stream */
int hsd_timer_start(void);
int hsd_copy_bench(const void *src, void *dst, long long n16, int iters, float *ms);
int hsd_timer_stop(float *ms);
int hsd_pass_timer_begin(int i);
int hsd_pass_timer_end(int i);
int hsd_pass_timer_read(int n, float *ms);

#ifdef __cplusplus
}
#endif

#endif
