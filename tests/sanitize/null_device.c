/*
 * null_device.c -- TEST INFRASTRUCTURE ONLY: a host-memory stand-in for the device layer
 * (csrc/hsfft_internal.h's hsd_* functions) so that the host C of libhsfft.so (planner,
 * registry, pass scheduler, chunking, real / convolution drivers) can be built and run under
 * -fsanitize=address,undefined on a machine without a GPU (SURVEY.md §5 "Race detection /
 * sanitizers").  It computes nothing: every "launch" checks the geometry the host chose and
 * touches the first and last element of every row it would read or write, so an undersized
 * scratch buffer or a wrong row stride is an AddressSanitizer report.  It is never linked
 * into the product.
 */
#include <stdint.h>
#include <stdio.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "hsfft_internal.h"

static __thread char err[256];
static __thread int sidx;
static __thread volatile double sink; /* per thread: launches on different null devices run concurrently */

/* HSFFT_NULL_NDEV (default 1) null devices, so that the multi-device paths
 * (hsfft_exec_multi: one host thread per device, per-device state, locks and scratch) run
 * under the sanitizers on a machine with no GPU; the current device is per thread and starts
 * at 0, as in HIP */
static __thread int cur_dev;
int hsd_device_count(void)
{
    const char *e = getenv("HSFFT_NULL_NDEV");
    const int n = e ? atoi(e) : 1;
    return n < 1 ? 1 : n > 16 ? 16 : n;
}
int hsd_set_device(int dev)
{
    if (dev < 0 || dev >= hsd_device_count()) return -1;
    cur_dev = dev;
    return 0;
}
int hsd_get_device(void) { return cur_dev; }
void *hsd_malloc(size_t bytes) { return malloc(bytes ? bytes : 16); }
int hsd_free(void *p)
{
    free(p);
    return 0;
}
int hsd_h2d(void *d, const void *h, size_t bytes)
{
    memcpy(d, h, bytes);
    return 0;
}
int hsd_d2h(void *h, const void *d, size_t bytes)
{
    memcpy(h, d, bytes);
    return 0;
}
int hsd_d2d_async(void *d, const void *s, size_t bytes)
{
    memmove(d, s, bytes);
    return 0;
}
int hsd_memset_async(void *d, int v, size_t bytes)
{
    memset(d, v, bytes);
    return 0;
}
/* this thread's pending error of an asynchronous persistent Bluestein launch (null_bx_timeout
 * = 1): kept by hsd_sync, reported once by hsd_sync_report -- the device layer's contract */
static __thread int pl_pending;
int hsd_sync(void) { return 0; }
int hsd_sync_report(void)
{
    if (!pl_pending) return 0;
    pl_pending = 0;
    snprintf(err, sizeof err, "null device: persistent launch timed out");
    return -2;
}
int null_finalized;
static __thread void *own_tok[16]; /* this thread's own stream per device (hsd_thread_park) */
int hsd_finalize_device(void)
{
    free(own_tok[cur_dev]); /* the calling thread's own stream */
    own_tok[cur_dev] = NULL;
    __atomic_fetch_add(&null_finalized, 1, __ATOMIC_RELAXED);
    return hsd_sync_report();
}
int hsd_select_stream(int idx)
{
    sidx = idx;
    return 0;
}
int hsd_stream_index(void) { return sidx; }
int hsd_h2d_async(void *d, const void *h, size_t bytes) { return hsd_h2d(d, h, bytes); }
int hsd_d2h_async(void *h, const void *d, size_t bytes) { return hsd_d2h(h, d, bytes); }
int hsd_stream_sync(void) { return 0; }
int hsd_host_word_wait(unsigned *flag, unsigned v)
{
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != v) {
        snprintf(err, sizeof err, "null device: completion word %u, awaited %u", *flag, v);
        return -1;
    }
    return 0;
}
int hsd_stream_signal_wait(unsigned *flag, unsigned v)
{
    __atomic_store_n(flag, v, __ATOMIC_RELEASE); /* the null device completes at once */
    return 0;
}
int hsd_host_register(void *p, size_t bytes) { return 0; }
int hsd_host_unregister(void *p) { return 0; }
int null_host_allocs; /* page-locked blocks allocated (counted by the driver) */
void *hsd_host_alloc(size_t bytes)
{
    __atomic_fetch_add(&null_host_allocs, 1, __ATOMIC_RELAXED);
    return malloc(bytes ? bytes : 16);
}
int hsd_host_free(void *p)
{
    free(p);
    return 0;
}
int hsd_event_record(int i) { return i < 0 ? -1 : 0; }
int hsd_event_wait(int i) { return i < 0 ? -1 : 0; }
void *hsd_stream(void) { return NULL; }
/* per-thread sets (hsd_tset + the thread's own stream, modelled as a heap token created on
 * the thread's first launch on its own stream): parked at thread exit, adopted by a new thread's
 * first use of the device, freed by hsd_pool_drain -- so ASan reports a set that is lost (leak)
 * or freed while still in use, and the driver counts the streams and page-locked blocks
 * created (they must stay at the number of threads alive at once) */
#define NULL_POOL 256
typedef struct {
    void *tok;
    hsd_tset h;
} null_set;
static pthread_mutex_t null_pool_mtx = PTHREAD_MUTEX_INITIALIZER;
static null_set null_pool[16][NULL_POOL];
static int null_pool_n[16];
int null_parks, null_adopts, null_drained;
long long null_streams_created;
static void own_stream_used(void)
{
    if (sidx == 3 && !own_tok[cur_dev]) {
        own_tok[cur_dev] = malloc(1);
        __atomic_fetch_add(&null_streams_created, 1, __ATOMIC_RELAXED);
    }
}
long long hsd_thread_streams_created(void) { return __atomic_load_n(&null_streams_created, __ATOMIC_RELAXED); }
void hsd_thread_park(int dev, const hsd_tset *h)
{
    if (dev < 0 || dev >= 16) return;
    null_set s = {own_tok[dev], {{NULL, NULL}, 0, NULL}};
    if (h) s.h = *h;
    own_tok[dev] = NULL;
    if (!s.tok && !s.h.pin[0] && !s.h.pin[1] && !s.h.flag) return;
    pthread_mutex_lock(&null_pool_mtx);
    if (null_pool_n[dev] < NULL_POOL) null_pool[dev][null_pool_n[dev]++] = s;
    else { /* (never in the driver: it would show as a lower adopt count) */
        free(s.tok);
        free(s.h.pin[0]);
        free(s.h.pin[1]);
        free(s.h.flag);
    }
    pthread_mutex_unlock(&null_pool_mtx);
    __atomic_fetch_add(&null_parks, 1, __ATOMIC_RELAXED);
}
int hsd_thread_adopt(int dev, hsd_tset *h)
{
    if (dev < 0 || dev >= 16 || own_tok[dev]) return 0;
    pthread_mutex_lock(&null_pool_mtx);
    const int have = null_pool_n[dev] > 0;
    null_set s = {NULL, {{NULL, NULL}, 0, NULL}};
    if (have) s = null_pool[dev][--null_pool_n[dev]];
    pthread_mutex_unlock(&null_pool_mtx);
    if (!have) return 0;
    own_tok[dev] = s.tok;
    if (h) *h = s.h;
    __atomic_fetch_add(&null_adopts, 1, __ATOMIC_RELAXED);
    return 1;
}
int hsd_pool_drain(void)
{
    int n = 0;
    pthread_mutex_lock(&null_pool_mtx);
    for (int d = 0; d < 16; d++) {
        for (int i = 0; i < null_pool_n[d]; i++) {
            null_set *s = &null_pool[d][i];
            free(s->tok);
            free(s->h.pin[0]);
            free(s->h.pin[1]);
            free(s->h.flag);
            n++;
        }
        null_pool_n[d] = 0;
    }
    pthread_mutex_unlock(&null_pool_mtx);
    __atomic_fetch_add(&null_drained, n, __ATOMIC_RELAXED);
    return n;
}
/* "device" memory is host memory here: pointers the tests pass as device buffers are
 * malloc'd, so every pointer counts as a device pointer -- except the buffers a test marks
 * as host buffers (null_mark_host), which take the host-pointer paths of fft_exec (the
 * concurrent small path among them) */
#define NULL_NHOST 64
static const void *null_host[NULL_NHOST];
void null_mark_host(const void *p, int on)
{
    for (int i = 0; i < NULL_NHOST; i++) {
        const void *want = on ? NULL : p;
        if (__atomic_load_n(&null_host[i], __ATOMIC_ACQUIRE) == want) {
            const void *exp = want;
            if (__atomic_compare_exchange_n(&null_host[i], &exp, on ? p : NULL, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
                return;
        }
    }
}
int hsd_is_device_ptr(const void *p)
{
    if (p == NULL) return 0;
    for (int i = 0; i < NULL_NHOST; i++)
        if (__atomic_load_n(&null_host[i], __ATOMIC_ACQUIRE) == p) return 0;
    return 1;
}
const char *hsd_errstr(void) { return err; }
int hsd_cu_count(void) { return 256; }
int hsd_count_diff(const void *a, const void *b, long long nwords, unsigned long long *count)
{
    unsigned long long c = 0;
    for (long long i = 0; i < nwords; i++) c += ((const uint64_t *)a)[i] != ((const uint64_t *)b)[i];
    *count = c;
    return 0;
}

/* read the first and last element of `rows` rows of `len` complex, `dist` apart */
static void touch_rows_r(const void *base, long long dist, long long len, long long rows, size_t esz)
{
    if (!base || rows <= 0 || len <= 0) return;
    const char *b = base;
    for (long long r = 0; r < rows; r++) {
        sink += *(const double *)(b + (size_t)(r * dist) * esz);
        sink += *(const double *)(b + (size_t)(r * dist + len - 1) * esz + esz - sizeof(double));
    }
}

static void touch_rows_w(void *base, long long dist, long long len, long long rows, size_t esz)
{
    if (!base || rows <= 0 || len <= 0) return;
    char *b = base;
    for (long long r = 0; r < rows; r++) {
        memset(b + (size_t)(r * dist) * esz, 0, esz);
        memset(b + (size_t)(r * dist + len - 1) * esz, 0, esz);
    }
}

int hsd_run_pass(const hsd_pass *p, const hsd_launch *l)
{
    if (p->P <= 0 || p->A <= 0 || p->B <= 0 || l->batch <= 0) {
        snprintf(err, sizeof err, "null device: bad pass geometry");
        return -1;
    }
    /* a launch on a thread's own stream (the concurrent small fft_exec path) "runs" a little
     * later, as a queued kernel would: the window in which another thread could free what it
     * reads (tests the device-state pinning) */
    if (sidx == 3) {
        own_stream_used();
        usleep(20);
    }
    /* a one-workgroup launch that stores its completion word itself (the small path): the word
     * must not ALREADY hold the awaited value -- the host would see "done" before the kernel ran
     * (a recycled word must continue its previous owner's sequence) */
    if (l->done) {
        if (__atomic_load_n(l->done, __ATOMIC_ACQUIRE) == l->done_val) {
            snprintf(err, sizeof err, "null device: completion word already holds the awaited value %u", l->done_val);
            return -1;
        }
        __atomic_store_n(l->done, l->done_val, __ATOMIC_RELEASE);
        if (l->armed) *l->armed = 1;
    }
    const long long M = (long long)p->P * p->A * p->B;
    const long long in_len = l->load_op == HS_LOAD_CHIRP ? l->nsig : M;
    const long long out_len = l->store_op == HS_STORE_CHIRP ? l->nsig : M;
    touch_rows_r(l->in, l->idist, in_len, l->batch, 16);
    touch_rows_r(l->tw, 0, M > 1 ? M - 1 : 1, 1, 16);
    if (l->load_op == HS_LOAD_CHIRP) touch_rows_r(l->load_aux, 0, l->nsig, 1, 16);
    if (l->store_op == HS_STORE_SPEC) touch_rows_r(l->store_aux, 0, M, 1, 16);
    if (l->store_op == HS_STORE_CHIRP) touch_rows_r(l->store_aux, 0, l->nsig, 1, 16);
    touch_rows_w(l->out, l->odist, out_len, l->batch, 16);
    return 0;
}

/* the null device has every specialised variant the host may ask for */
int r8_has_variant(int r0, int n8, int G, int Wq, int first) { return 1; }
int mr_has_variant(const hsd_pass *p) { return 1; }

int hsd_r2c_last(const void *Z, long long zdist, void *X, long long xdist, const void *tw, const void *w2, long long h,
                 long long B, int batch, int sgn, int compact)
{
    touch_rows_r(Z, zdist, h, batch, 16);
    touch_rows_r(w2, 0, h, 1, 16);
    touch_rows_w(X, xdist, compact ? h + 1 : 2 * h, batch, 16);
    return 0;
}
int hsd_blue_mid(const void *in, void *out, long long dist, const void *tw, const void *hk, int batch, int sgn,
                 int conj, int dir, int sgn2, int conj2)
{
    touch_rows_r(in, dist, dist, batch, 16);
    touch_rows_r(hk, 0, dist, 1, 16);
    touch_rows_w(out, dist, dist, batch, 16);
    return 0;
}
int hsd_blue_last(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                  long long nsig, int batch, int dir)
{
    touch_rows_r(in, idist, idist, batch, 16);
    touch_rows_w(out, odist, nsig, batch, 16);
    return 0;
}
int hsd_blue_first(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                   long long nsig, int batch, int dir)
{
    touch_rows_r(in, idist, nsig, batch, 16);
    touch_rows_r(chirp, 0, nsig, 1, 16);
    touch_rows_w(out, odist, odist, batch, 16);
    return 0;
}
/* null_bx_timeout = 1: the persistent Bluestein launch's waits time out -- a synchronous call
 * gets 2 (it re-runs the rows), an asynchronous one leaves the error pending for the thread's
 * next hsd_sync_report; 2: the grid is refused as not co-resident (3) -- the host's three-launch
 * path runs */
int null_bx_timeout;
static __thread int deferred_pending;
int hsd_blue_deferred_take(void)
{
    const int v = deferred_pending;
    deferred_pending = 0;
    return v;
}

int hsd_blue_xcd(const void *in, long long idist, void *out, long long odist, const void *tw, const void *chirp,
                 const void *hk, void *img, size_t img_bytes, long long nsig, int batch, int sgn, int ng, int sync)
{
    touch_rows_r(in, idist, nsig, batch, 16);
    touch_rows_r(chirp, 0, nsig, 1, 16);
    touch_rows_r(hk, 0, 512 * 512, 1, 16);
    touch_rows_w(img, 0, (long long)(img_bytes / 16), 1, 16);
    if (null_bx_timeout == 2) return 3;
    if (null_bx_timeout == 1) {
        if (sync == 1) return 2;
        if (sync == 2) deferred_pending = 1; /* read by hsd_blue_deferred_take */
        else pl_pending = 1;
        return 0;
    }
    touch_rows_w(out, odist, nsig, batch, 16);
    return 0;
}
int hsd_fill_complex(void *d, int64_t count, uint64_t seed, uint64_t offset)
{
    memset(d, 0, (size_t)count * 16);
    return 0;
}
int hsd_fill_real(void *d, int64_t count, uint64_t seed, uint64_t offset)
{
    memset(d, 0, (size_t)count * 8);
    return 0;
}
int hsd_r2c_post(const void *Z, const void *tw2, void *X, int h, int batch, long long zdist, long long xdist)
{
    touch_rows_r(Z, zdist, h, batch, 16);
    touch_rows_w(X, xdist, 2LL * h, batch, 16);
    return 0;
}
int hsd_r2c_post_compact(const void *Z, const void *tw2, void *X, int h, int batch, long long zdist, long long xdist)
{
    touch_rows_r(Z, zdist, h, batch, 16);
    touch_rows_w(X, xdist, h + 1LL, batch, 16);
    return 0;
}
int hsd_c2r_pre(const void *X, const void *tw2, void *Zin, int h, int batch, long long xdist, long long zdist)
{
    touch_rows_r(X, xdist, h + 1LL, batch, 16);
    touch_rows_w(Zin, zdist, h, batch, 16);
    return 0;
}
int hsd_cmul(const void *A, const void *Bv, void *C, long long n, int batch, long long dist)
{
    touch_rows_r(A, dist, n, batch, 16);
    touch_rows_r(Bv, dist, n, batch, 16);
    touch_rows_w(C, dist, n, batch, 16);
    return 0;
}
int hsd_c2r_pre_mul(const void *A, const void *Bv, const void *tw2, void *Zin, int h, int batch, long long xdist,
                    long long zdist)
{
    touch_rows_r(A, xdist, h + 1LL, batch, 16);
    touch_rows_r(Bv, xdist, h + 1LL, batch, 16);
    touch_rows_w(Zin, zdist, h, batch, 16);
    return 0;
}
int hsd_copy_rows_div(const void *src, long long sdist, long long soff, void *dst, long long ddist, long long n,
                      int batch, double divisor)
{
    touch_rows_r((const double *)src + soff, sdist, n, batch, 8);
    touch_rows_w(dst, ddist, n, batch, 8);
    return 0;
}
int hsd_scale_real(void *x, long long n, int batch, long long dist, double divisor)
{
    touch_rows_w(x, dist, n, batch, 8);
    return 0;
}
int hsd_copy_rows(const void *src, long long sdist, long long soff, long long ncopy, void *dst, long long ddist,
                  long long dlen, int batch)
{
    touch_rows_r((const double *)src + soff, sdist, ncopy, batch, 8);
    touch_rows_w(dst, ddist, dlen, batch, 8);
    return 0;
}
int hsd_timer_start(void) { return 0; }
int hsd_copy_bench(const void *src, void *dst, long long n16, int iters, float *ms)
{
    *ms = 0.0f;
    return 0;
}
int hsd_timer_stop(float *ms)
{
    *ms = 0.0f;
    return 0;
}
int hsd_pass_timer_begin(int i) { return 0; }
int hsd_pass_timer_end(int i) { return 0; }
int hsd_pass_timer_read(int n, float *ms)
{
    for (int i = 0; i < n; i++) ms[i] = 0.0f;
    return 0;
}
