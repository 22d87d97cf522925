/*
 * hsfft_exec.c -- execution side of libhsfft.so (host C): plan registry, Stockham pass
 * scheduling, the drop-in fft_exec (ref src/highSpeedFFT.c:1920-1942), the Bluestein
 * orchestration (ref :1735-1907) and the batched / device-pointer extension API.
 *
 * There is no CPU compute path: every transform runs on the GPU through the device layer.
 * Without a usable GPU the compute entry points fail loudly (stderr + exit for the drop-in
 * functions, the reference's error convention; an error code for the extension API).
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include "hsfft_gpu.h"
#include "hsfft_host.h"

static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER; /* the plan registry */
static hs_entry *g_entries;
static __thread char g_errbuf[512];

/* > 0 while this thread is inside a synchronous entry point (fft_exec, the drop-in real and
 * convolution calls, hsfft_exec_batched_host, hsfft_exec_multi's shards): the persistent
 * Bluestein launch then runs synchronously and re-runs the rows of a timed-out launch itself,
 * instead of leaving the error for a later hsfft_synchronize() */
static __thread int t_sync_call;

void hs_sync_call(int enter) { t_sync_call += enter ? 1 : -1; }

/* > 0 inside hsfft_exec_batched_host's pipeline: its persistent Bluestein launches
 * stay asynchronous -- so chunk k+1's upload overlaps chunk k's transform -- and record a
 * timed-out wait in the thread's DEFERRED error word, which the pipeline reads once after its
 * final stream wait; a set word re-runs the whole batch on the three-launch path (t_no_xcd) */
static __thread int t_deferred_call;
static __thread int t_no_xcd;

/* per-device API locks (recursive: public entry points call each other) */
static pthread_mutex_t g_dev_mtx[HS_MAX_DEV];
static pthread_once_t g_dev_once = PTHREAD_ONCE_INIT;

static void dev_mtx_init(void)
{
    pthread_mutexattr_t at;
    pthread_mutexattr_init(&at);
    pthread_mutexattr_settype(&at, PTHREAD_MUTEX_RECURSIVE);
    for (int d = 0; d < HS_MAX_DEV; d++) pthread_mutex_init(&g_dev_mtx[d], &at);
    pthread_mutexattr_destroy(&at);
}

int hs_lock_device(void)
{
    pthread_once(&g_dev_once, dev_mtx_init);
    int d = hsd_get_device();
    if (d < 0 || d >= HS_MAX_DEV) d = 0;
    pthread_mutex_lock(&g_dev_mtx[d]);
    return d;
}

void hs_unlock_device(int dev) { pthread_mutex_unlock(&g_dev_mtx[dev]); }

void hs_seterr(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_errbuf, sizeof g_errbuf, fmt, ap);
    va_end(ap);
}

const char *hsfft_last_error(void) { return g_errbuf; }

static void fatal(const char *what)
{
    fprintf(stderr, "Error: %s (%s)\n", what, g_errbuf[0] ? g_errbuf : hsd_errstr());
    exit(EXIT_FAILURE);
}

static int g_ndev = -1;
static pthread_once_t g_ndev_once = PTHREAD_ONCE_INIT;
static void ndev_init(void) { g_ndev = hsd_device_count(); }

int hs_require_gpu(void)
{
    pthread_once(&g_ndev_once, ndev_init);
    if (g_ndev <= 0) {
        hs_seterr("no HIP device available: libhsfft has no CPU execution path");
        return HSFFT_ERR_DEVICE;
    }
    return 0;
}

/* ------------------------------------------------------------------ scheduling */
static int is_leaf_len(int n) { return n == 2 || n == 3 || n == 4 || n == 5 || n == 7 || n == 8; }

/* Effective stage list of the reference recursion: descend with data_length = M taking
 * factors[fi]; a data_length in {2,3,4,5,7,8} is a leaf butterfly of that size (ref
 * :332-713 dispatch on data_length before radix).  Returns stages innermost first. */
static int effective_stages(int M, const int *fac, int lf, int *out, int *first_leaf)
{
    int outer[HS_MAX_STAGES], n = 0, len = M, fi = 0;
    *first_leaf = 0;
    while (len > 1) {
        if (is_leaf_len(len)) {
            outer[n++] = len;
            *first_leaf = 1;
            break;
        }
        if (fi >= lf || fac[fi] <= 1 || len % fac[fi] != 0 || n >= HS_MAX_STAGES) return -1;
        outer[n++] = fac[fi];
        len /= fac[fi++];
    }
    for (int i = 0; i < n; i++) out[i] = outer[n - 1 - i];
    return n;
}

static int pass_pmax(void)
{
    const char *s = getenv("HSFFT_PMAX");
    const int v = s ? atoi(s) : 512;
    return v < 8 ? 8 : v;
}

/* Knob lookups of the small drop-in path (round 6).  fft_exec of N = 1024 on host buffers reads
 * five HSFFT_* knobs per call, and getenv scans the whole environment each time: measured on the
 * box, 500 extra environment variables made that call 5.5 us slower (11.6 -> 17.1 us; with the
 * snapshot +0.2 us, profiles/r06d_c1_getenv.txt).  The small path therefore takes one snapshot of the HSFFT_*
 * entries per call (hs_env_begin), rebuilt only when the environment changed -- the signature
 * is the `environ` array and the addresses of its strings: setenv / putenv / unsetenv (and
 * Python's os.environ) replace or move entries, so a changed value changes an address -- and
 * the lookups inside that call search the snapshot.  Outside such a call hs_getenv is getenv. */
extern char **environ;
#define HS_ENV_MAX 64
static __thread struct {
    uintptr_t sig;
    int valid, active, n;
    const char *kv[HS_ENV_MAX];
} t_env;

static uintptr_t env_signature(void)
{
    uintptr_t h0 = (uintptr_t)environ, h1 = 0;
    char **e = environ;
    for (int i = 0; e && e[i]; i++) {
        if (i & 1) h1 = h1 * 0x9E3779B97F4A7C15ull + (uintptr_t)e[i];
        else h0 = h0 * 0xC2B2AE3D27D4EB4Full + (uintptr_t)e[i];
    }
    return h0 ^ (h1 * 31 + 7);
}

void hs_env_begin(void)
{
    const uintptr_t sig = env_signature();
    if (!t_env.valid || sig != t_env.sig) {
        t_env.n = 0;
        for (char **e = environ; e && *e; e++)
            if (!strncmp(*e, "HSFFT_", 6)) {
                if (t_env.n == HS_ENV_MAX) { /* more knobs than the table holds: plain getenv */
                    t_env.valid = 0;
                    return;
                }
                t_env.kv[t_env.n++] = *e;
            }
        t_env.sig = sig;
        t_env.valid = 1;
    }
    t_env.active = 1;
}

void hs_env_end(void) { t_env.active = 0; }

const char *hs_getenv(const char *name)
{
    if (!t_env.active) return getenv(name);
    const size_t len = strlen(name);
    for (int i = 0; i < t_env.n; i++)
        if (!strncmp(t_env.kv[i], name, len) && t_env.kv[i][len] == '=') return t_env.kv[i] + len + 1;
    return NULL;
}

static int env_int(const char *name, int dflt)
{
    const char *s = hs_getenv(name);
    return s ? atoi(s) : dflt;
}

/* Register-kernel schedule for radix lists [r0, 8, 8, ...] (r0 in {2,4,8}; hsfft_pass_r8.h):
 * first pass [r0, 8^k1] with P <= 2048, then passes of 8^k (k <= 3), as few passes as
 * possible and as even as possible.  Tiles come from the variant table of the kernel. */
static int build_passes_pow2(hs_entry *e)
{
    const int r0 = e->stage_r[0];
    if (!e->first_leaf || !(r0 == 2 || r0 == 4 || r0 == 8)) return -1;
    for (int s = 1; s < e->nst; s++)
        if (e->stage_r[s] != 8) return -1;
    if (env_int("HSFFT_GENERIC", 0)) return -1;
    int n8 = e->nst - 1;            /* radix-8 stages after stage 0 */
    /* at most 4 stages per pass; P <= 2048 unless r0 == 8 and a 4096-point first pass
     * saves a whole pass (2^21 = [8,8,8,8] + [8,8,8]) */
    int k1max = r0 == 8 ? (n8 == 6 ? 3 : 2) : 3;
    /* the whole transform as ONE pass when it fits one workgroup (P <= 8192 points, <= 1024
     * threads of 8 points): one HBM round trip instead of two -- 4096 = [8,8,8,8] and
     * 8192 = [2,8,8,8,8] (HSFFT_WHOLE=0: the two-pass schedule) */
    {
        long long pall = r0;
        for (int i = 0; i < n8; i++) pall *= 8;
        if (n8 <= 4 && pall <= 8192 && env_int("HSFFT_WHOLE", 1) && r8_has_variant(r0, n8, 1, 1, 1)) k1max = n8;
    }
    /* number of later passes needed if the first takes k1 eights: ceil((n8-k1)/3) */
    int best_k1 = -1, best_np = 1 << 30, best_bal = 1 << 30;
    for (int k1 = r0 == 8 ? 0 : 1; k1 <= k1max && k1 <= n8; k1++) { /* every pass needs P >= 8 */
        const int rest = n8 - k1, np = 1 + (rest + 2) / 3;
        int bal = 0;
        if (rest) {
            const int per = (rest + (np - 1) - 1) / (np - 1);
            bal = per > k1 + 1 ? per - k1 - 1 : k1 + 1 - per;
        }
        const int forced = env_int("HSFFT_K1", -1);
        if (forced >= 0 && k1 != forced) continue;
        if (np < best_np || (np == best_np && bal < best_bal)) {
            best_np = np;
            best_bal = bal;
            best_k1 = k1;
        }
    }
    if (best_k1 < 0 || best_np > HS_MAX_PASSES) return -1;
    long long B = 1;
    int np = 0, s = 0;
    const int later = best_np - 1;
    int remaining = n8 - best_k1;
    for (int ip = 0; ip < best_np; ip++) {
        hsd_pass *p = &e->pass[np++];
        memset(p, 0, sizeof *p);
        int k = ip == 0 ? best_k1 : (remaining + (later - (ip - 1)) - 1) / (later - (ip - 1));
        if (ip > 0) remaining -= k;
        p->nst = ip == 0 ? 1 + k : k;
        p->P = 1;
        for (int i = 0; i < p->nst; i++) {
            p->radix[i] = e->stage_r[s++];
            p->gcs_off[i] = -1;
            p->P *= p->radix[i];
        }
        p->leaf = ip == 0;
        p->B = B;
        p->A = e->M / (B * p->P);
        p->variant = HS_KV_R8X3;
        if (ip == 0) {
            /* WM columns per workgroup: as many as the LDS (<=128 KiB) and the variant table allow */
            static const int gopts[] = {32, 16, 8, 4, 2, 1};
            int gmax = env_int("HSFFT_G1", 0);
            if (gmax <= 0) gmax = p->P >= 4096 ? 1 : p->P >= 2048 ? 2 : p->P >= 1024 ? 4 : p->P >= 512 ? 8 : p->P >= 64 ? 16 : 32;
            int G = 1;
            for (unsigned i = 0; i < sizeof gopts / sizeof gopts[0]; i++)
                if (gopts[i] <= gmax && gopts[i] <= p->A && r8_has_variant(p->radix[0], p->nst - 1, gopts[i], 1, 1)) {
                    G = gopts[i];
                    break;
                }
            p->Wm = G;
            p->Wq = 1;
            p->G = G;
        } else {
            static const int gopts[] = {32, 16, 8, 4};
            int gmax = env_int("HSFFT_G2", 0);
            if (gmax <= 0) gmax = p->P >= 512 ? 8 : 32;
            int G = 0;
            for (unsigned i = 0; i < sizeof gopts / sizeof gopts[0]; i++)
                if (gopts[i] <= gmax && gopts[i] <= B && r8_has_variant(8, p->nst - 1, gopts[i], gopts[i], 0)) {
                    G = gopts[i];
                    break;
                }
            if (!G) return -1;
            p->Wm = 1;
            p->Wq = G;
            p->G = G;
        }
        B *= p->P;
    }
    e->npass = np;
    return 0;
}

/* Groups stages into passes of at most Pmax points and chooses the tile so that global
 * loads/stores move >= 128 contiguous bytes (8 complex) per row where the shape allows. */
static int build_passes(hs_entry *e)
{
    if (build_passes_pow2(e) == 0) return 0;
    if (e->nst <= HS_MAX_PASS_STAGES && env_int("HSFFT_MR_ROW", 1) && !env_int("HSFFT_GENERIC", 0)) {
        /* a whole-row kernel for this radix list (hsfft_pass_mr.h k_row): one pass, one HBM
         * round trip per row */
        hsd_pass *p = &e->pass[0];
        memset(p, 0, sizeof *p);
        p->nst = e->nst;
        p->P = 1;
        for (int s = 0; s < e->nst; s++) {
            p->radix[s] = e->stage_r[s];
            p->gcs_off[s] = -1;
            p->P *= e->stage_r[s];
        }
        p->leaf = e->first_leaf;
        p->B = 1;
        p->A = 1;
        p->Wq = p->Wm = p->G = 1;
        p->variant = HS_KV_MR;
        if (p->P == e->M && mr_has_variant(p)) {
            e->npass = 1;
            return 0;
        }
    }
    /* a whole row that fits the generic kernel's LDS ping-pong (32 B per point <= 160 KiB):
     * one pass, one HBM round trip, instead of passes of <= Pmax points (HSFFT_WHOLE=0) */
    int odd = 0, nodd = 0; /* distinct odd radices >= 11 (the generic kernel specialises one) */
    for (int i = 0; i < e->nst; i++) {
        const int r = e->stage_r[i];
        if (r == 2 || r == 3 || r == 4 || r == 5 || r == 7 || r == 8 || r == odd) continue;
        odd = r;
        nodd++;
    }
    const int whole = env_int("HSFFT_WHOLE", 1) && e->M <= 5120 && e->nst <= HS_MAX_PASS_STAGES && nodd <= 1;
    const int pmax = whole ? e->M : pass_pmax();
    int s = 0, np = 0;
    long long B = 1;
    while (s < e->nst) {
        if (np >= HS_MAX_PASSES) return -1;
        hsd_pass *p = &e->pass[np];
        memset(p, 0, sizeof *p);
        p->P = 1;
        p->leaf = (s == 0) && e->first_leaf;
        while (s < e->nst && p->nst < HS_MAX_PASS_STAGES && (p->nst == 0 || (long long)p->P * e->stage_r[s] <= pmax)) {
            p->radix[p->nst] = e->stage_r[s];
            p->gcs_off[p->nst] = -1;
            p->P *= e->stage_r[s];
            p->nst++;
            s++;
        }
        p->B = B;
        p->A = e->M / (B * p->P);
        int gmax = 2048 / p->P;
        if (gmax < 1) gmax = 1;
        int wq = (int)(B < 8 ? B : 8);
        if (wq > gmax) wq = gmax;
        int wm = 8 / wq;
        if (wm * wq > gmax) wm = gmax / wq;
        if (wm < 1) wm = 1;
        if (wm > p->A) wm = (int)p->A;
        p->Wq = wq;
        p->Wm = wm;
        p->G = wq * wm;
        p->variant = HS_KV_GENERIC;
        if (!env_int("HSFFT_GENERIC", 0) && mr_has_variant(p)) p->variant = HS_KV_MR;
        B *= p->P;
        np++;
    }
    e->npass = np;
    return 0;
}

/* odd-radix constants: cos/sin(i*PI2/p) for i <= (p-1)/2, mirrored (ref :1527-1541) */
static int build_gcs(hs_entry *e)
{
    int total = 0;
    for (int i = 0; i < e->npass; i++)
        for (int s = 0; s < e->pass[i].nst; s++) {
            int r = e->pass[i].radix[s];
            if (r == 2 || r == 3 || r == 4 || r == 5 || r == 7 || r == 8) continue;
            if (r > 63) {
                hs_seterr("radix %d exceeds the odd-radix kernel limit (63)", r);
                return -1;
            }
            total += 2 * (r - 1);
        }
    e->ngcs = total;
    e->gcs = total ? malloc(sizeof(double) * (size_t)total) : NULL;
    int off = 0;
    for (int i = 0; i < e->npass; i++)
        for (int s = 0; s < e->pass[i].nst; s++) {
            int r = e->pass[i].radix[s];
            if (r == 2 || r == 3 || r == 4 || r == 5 || r == 7 || r == 8) continue;
            const int mid = (r - 1) / 2;
            double *cs = e->gcs + off, *sn = cs + (r - 1);
            for (int k = 1; k <= mid; k++) {
                double sv, cv;
                sincos(k * PI2 / r, &sv, &cv);
                cs[k - 1] = cv;
                sn[k - 1] = sv;
            }
            for (int k = 0; k < mid; k++) {
                sn[k + mid] = -sn[mid - 1 - k];
                cs[k + mid] = cs[mid - 1 - k];
            }
            e->pass[i].gcs_off[s] = off;
            off += 2 * (r - 1);
        }
    return 0;
}

static void free_devstate(hs_devstate *d)
{
    if (!d) return;
    hsd_free(d->d_tw);
    hsd_free(d->d_gcs);
    hsd_free(d->d_chirp);
    hsd_free(d->d_hk);
    free(d);
}

/* drop a device state that is being replaced: freed now, or by its last pinned user */
static void retire_devstate(hs_devstate *d)
{
    if (!d) return;
    if (d->refs > 0) d->retired = 1;
    else free_devstate(d);
}

/* (device lock held) release a pin taken by the concurrent small path */
static void devstate_put(hs_devstate *d)
{
    if (d && --d->refs == 0 && d->retired) free_devstate(d);
}

static void entry_free(hs_entry *e)
{
    int cur = hsd_get_device();
    for (int d = 0; d < HS_MAX_DEV; d++)
        if (e->ds[d]) {
            hsd_set_device(d);
            retire_devstate(e->ds[d]);
        }
    if (cur >= 0) hsd_set_device(cur);
    free(e->tw_private);
    free(e->gcs);
    free(e->chirp);
    free(e);
}

static int snapshot_matches(const hs_entry *e, const struct fft_set *o)
{
    if (e->N != o->N || e->sgn != o->sgn || e->lt != o->lt || e->lf != o->lf) return 0;
    for (int i = 0; i < o->lf && i < 64; i++)
        if (e->factors[i] != o->factors[i]) return 0;
    return 1;
}

static hs_entry *entry_build(const struct fft_set *o)
{
    if (o->lf < 0 || o->lf > 64) {
        hs_seterr("plan has %d factors", o->lf);
        return NULL;
    }
    hs_entry *e = calloc(1, sizeof *e);
    e->key = o;
    e->N = o->N;
    e->sgn = o->sgn;
    e->lt = o->lt;
    e->lf = o->lf;
    memcpy(e->factors, o->factors, sizeof e->factors);
    memcpy(e->rfac, o->factors, sizeof e->rfac);
    e->rlf = o->lf;
    e->tw_from_struct = 1;
    long long prod = 1;
    for (int i = 0; i < o->lf; i++) prod *= o->factors[i];
    if (o->lt == 0) {
        e->M = o->N;
    } else {
        /* bluestein_fft runs at the log2 length; fft_init sized the plan with log10.  Where
         * they disagree (N = 2^k+1, defect D5) the reference reads past its twiddles; here
         * the exec-side length gets its own factorisation and twiddle table. */
        e->M = hs_bluestein_M_exec(o->N);
        if (prod != e->M) {
            e->tw_from_struct = 0;
            e->rlf = factors(e->M, e->rfac);
            e->tw_private = calloc((size_t)e->M, sizeof(fft_data));
            hs_longvector(e->tw_private, e->M, e->rfac, e->rlf, hs_twiddle_mode() == 1);
            if (o->sgn == -1)
                for (int i = 0; i < e->M; i++) e->tw_private[i].im = -e->tw_private[i].im;
        }
    }
    if (e->M <= 0) {
        hs_seterr("invalid transform length %d", e->M);
        free(e);
        return NULL;
    }
    if (e->M > 1) {
        e->nst = effective_stages(e->M, e->rfac, e->rlf, e->stage_r, &e->first_leaf);
        if (e->nst < 0) {
            hs_seterr("factor list of the plan does not describe length %d", e->M);
            free(e->tw_private);
            free(e);
            return NULL;
        }
        if (build_passes(e) || build_gcs(e)) {
            free(e->tw_private);
            free(e->gcs);
            free(e);
            return NULL;
        }
        if (env_int("HSFFT_PLAN_DEBUG", 0)) { /* dev: the pass schedule */
            fprintf(stderr, "hsfft plan N=%d M=%d:", e->N, e->M);
            for (int i = 0; i < e->npass; i++) {
                const hsd_pass *p = &e->pass[i];
                fprintf(stderr, " [P=%d r=", p->P);
                for (int s = 0; s < p->nst; s++) fprintf(stderr, "%s%d", s ? "," : "", p->radix[s]);
                fprintf(stderr, " A=%lld B=%lld G=%d Wq=%d v=%d]", (long long)p->A, (long long)p->B, p->G, p->Wq, p->variant);
            }
            fprintf(stderr, "\n");
        }
        if (0) {
            free(e->tw_private);
            free(e->gcs);
            free(e);
            return NULL;
        }
    }
    if (o->lt == 1) { /* chirp h(n) = exp(i*pi*n^2/N), ref :1674-1690 */
        const double PI = 3.1415926535897932384626433832795;
        const int N = o->N;
        e->chirp = malloc(sizeof(fft_data) * (size_t)N);
        const double theta = PI / N;
        int l2 = 0;
        const int len2 = 2 * N;
        for (int n = 0; n < N; n++) {
            double sn, cs;
            sincos(theta * l2, &sn, &cs);
            e->chirp[n].re = cs;
            e->chirp[n].im = sn;
            l2 += 2 * n + 1;
            while (l2 > len2) l2 -= len2;
        }
    }
    return e;
}

/* unlink e (registry lock held); it is freed now, or by the last hs_entry_put */
static void entry_retire(hs_entry **pp)
{
    hs_entry *e = *pp;
    *pp = e->next;
    e->next = NULL;
    e->dead = 1;
    if (e->refs == 0) entry_free(e);
}

hs_entry *hs_entry_get(const struct fft_set *obj)
{
    pthread_mutex_lock(&g_lock);
    hs_entry **pp = &g_entries, *e = NULL;
    for (; *pp; pp = &(*pp)->next)
        if ((*pp)->key == obj) {
            e = *pp;
            break;
        }
    if (e && !snapshot_matches(e, obj)) { /* caller edited the public fields: rebuild */
        entry_retire(pp);
        e = NULL;
    }
    if (!e) {
        e = entry_build(obj);
        if (e) {
            e->next = g_entries;
            g_entries = e;
        }
    }
    if (e) e->refs++;
    pthread_mutex_unlock(&g_lock);
    return e;
}

void hs_entry_put(hs_entry *e)
{
    if (!e) return;
    pthread_mutex_lock(&g_lock);
    if (--e->refs == 0 && e->dead) entry_free(e);
    pthread_mutex_unlock(&g_lock);
}

void hs_entry_release(const struct fft_set *obj)
{
    pthread_mutex_lock(&g_lock);
    for (hs_entry **pp = &g_entries; *pp; pp = &(*pp)->next)
        if ((*pp)->key == obj) {
            entry_retire(pp);
            break;
        }
    pthread_mutex_unlock(&g_lock);
}

/* ------------------------------------------------------------------ scratch */
#define HS_NSCRATCH 11
static void *g_scr[HS_MAX_DEV][HS_NSCRATCH];
static size_t g_scr_sz[HS_MAX_DEV][HS_NSCRATCH];

/* (callers hold the device lock) */
void *hs_scratch(int cls, size_t bytes)
{
    int d = hsd_get_device();
    if (d < 0 || d >= HS_MAX_DEV || cls < 0 || cls >= HS_NSCRATCH) return NULL;
    if (g_scr_sz[d][cls] < bytes) {
        hsd_sync();
        hsd_free(g_scr[d][cls]);
        g_scr[d][cls] = hsd_malloc(bytes);
        g_scr_sz[d][cls] = g_scr[d][cls] ? bytes : 0;
    }
    return g_scr[d][cls];
}

int hsfft_release_scratch(void)
{
    const int d = hs_lock_device();
    int rc = 0;
    if (hs_require_gpu() == 0) {
        (void)hsd_pool_drain(); /* and the parked per-thread sets of exited threads */
        rc = hsd_sync() ? HSFFT_ERR_DEVICE : 0;
        for (int c = 0; c < HS_NSCRATCH; c++) {
            if (hsd_free(g_scr[d][c]) && !rc) rc = HSFFT_ERR_DEVICE;
            g_scr[d][c] = NULL;
            g_scr_sz[d][c] = 0;
        }
    }
    hs_unlock_device(d);
    return rc;
}

void hs_crash_trace_install(void);
static void *g_pin[HS_MAX_DEV][2];
static size_t g_pin_sz[HS_MAX_DEV];

/* Teardown (include/hsfft_gpu.h): every device object the library holds, on every device,
 * after waiting for that device's work -- the scratch pool, the page-locked staging slots, the
 * device state of every live plan (twiddles, odd-radix constants, Bluestein chirp / hk), the
 * real plans' device twiddles, the idle convolution plan pairs, the persistent-launch counters
 * and error words, the calling thread's own slots / words / streams, the timing and ordering
 * events and the library streams.  Everything is re-created on demand.  Callers must not run
 * other library calls concurrently. */
static void thread_pins_free_now(void);
int hsfft_finalize(void)
{
    g_errbuf[0] = 0;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int cur = hsd_get_device();
    hs_conv_cache_release(); /* frees plans: their device state on every device goes with them */
    thread_pins_free_now();  /* its streams, events and error words: hsd_finalize_device below */
    (void)hsd_pool_drain();  /* the parked per-thread sets of exited threads */
    const int ndev = hsd_device_count() < HS_MAX_DEV ? hsd_device_count() : HS_MAX_DEV;
    for (int d = 0; d < ndev; d++) {
        if (hsd_set_device(d)) {
            if (!rc) rc = HSFFT_ERR_DEVICE;
            continue;
        }
        const int dl = hs_lock_device();
        if (hsd_sync() && !rc) {
            hs_seterr("hsfft_finalize: %s", hsd_errstr());
            rc = HSFFT_ERR_DEVICE;
        }
        for (int c = 0; c < HS_NSCRATCH; c++) {
            hsd_free(g_scr[d][c]);
            g_scr[d][c] = NULL;
            g_scr_sz[d][c] = 0;
        }
        hsd_host_free(g_pin[d][0]);
        hsd_host_free(g_pin[d][1]);
        g_pin[d][0] = g_pin[d][1] = NULL;
        g_pin_sz[d] = 0;
        pthread_mutex_lock(&g_lock);
        for (hs_entry *e = g_entries; e; e = e->next)
            if (e->ds[d]) {
                retire_devstate(e->ds[d]);
                e->ds[d] = NULL;
            }
        pthread_mutex_unlock(&g_lock);
        hs_real_release_device(d);
        const int fr = hsd_finalize_device();
        if (fr && !rc) {
            hs_seterr("hsfft_finalize: %s", hsd_errstr());
            rc = HSFFT_ERR_DEVICE;
        }
        hs_unlock_device(dl);
    }
    if (cur >= 0) hsd_set_device(cur);
    return rc;
}

/* HSFFT_CRASH_TRACE=1 (diagnostics): on SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT the
 * library writes the signal, the faulting address and instruction pointer, the native
 * backtrace (library + offset per frame) and /proc/self/maps to stderr, then re-raises the
 * signal with its default action.  Installed when the library is loaded and again when a
 * device is selected (a tool that installs its own handler while the runtime initialises would
 * otherwise replace it). */
static void crash_puts(const char *s)
{
    size_t n = strlen(s);
    while (n > 0) {
        const ssize_t w = write(2, s, n);
        if (w <= 0) return;
        s += w;
        n -= (size_t)w;
    }
}

static void crash_hex(const char *label, unsigned long long v)
{
    char b[40];
    int i = 39;
    b[i] = 0;
    do {
        b[--i] = "0123456789abcdef"[v & 15];
        v >>= 4;
    } while (v && i > 2);
    b[--i] = 'x';
    b[--i] = '0';
    crash_puts(label);
    crash_puts(b + i);
}

static void crash_handler(int sig, siginfo_t *si, void *ucv)
{
    crash_hex("\n*** hsfft crash trace: signal ", (unsigned long long)sig);
    crash_hex(" fault address ", (unsigned long long)(uintptr_t)si->si_addr);
#if defined(__x86_64__)
    const ucontext_t *uc = (const ucontext_t *)ucv;
    crash_hex(" rip ", (unsigned long long)uc->uc_mcontext.gregs[REG_RIP]);
#else
    (void)ucv;
#endif
    crash_puts("\n*** backtrace:\n");
    void *fr[64];
    const int n = backtrace(fr, 64);
    backtrace_symbols_fd(fr, n, 2);
    crash_puts("*** /proc/self/maps:\n");
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        char buf[4096];
        ssize_t r;
        while ((r = read(fd, buf, sizeof buf)) > 0)
            if (write(2, buf, (size_t)r) != r) break;
        close(fd);
    }
    crash_puts("*** end of hsfft crash trace\n");
    signal(sig, SIG_DFL);
    raise(sig);
}

void hs_crash_trace_install(void)
{
    const char *e = getenv("HSFFT_CRASH_TRACE");
    if (!e || !atoi(e)) return;
    void *warm[2];
    (void)backtrace(warm, 2); /* loads the unwinder now, not inside the handler */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    const int sigs[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
    for (unsigned i = 0; i < sizeof sigs / sizeof sigs[0]; i++) sigaction(sigs[i], &sa, NULL);
}

__attribute__((constructor)) static void crash_trace_ctor(void) { hs_crash_trace_install(); }

/* Chunk sizes, one knob per path, all read per call: HSFFT_CHUNK_MB (c2c intermediates of
 * 3+-pass chains), HSFFT_BLUE_CHUNK_MB (Bluestein M-point intermediates), HSFFT_REAL_CHUNK_MB
 * (the real paths' inner intermediate, hsfft_real.c). */
size_t hs_env_mb(const char *name, double dflt_mb)
{
    const char *s = getenv(name);
    const double mb = s ? atof(s) : dflt_mb;
    const size_t v = (size_t)(mb * (double)(1u << 20));
    return v < (1u << 20) ? (1u << 20) : v;
}

static size_t chunk_bytes(void) { return hs_env_mb("HSFFT_CHUNK_MB", 256.0); }

/* Bluestein scratch per chunk (two M-point intermediates): large chunks keep the three
 * launches per chunk long enough to fill the chip (measured, 8192 x 99991: 64 rows 14.9,
 * 256 rows 16.0, 1024 rows 16.9 GSamples/s; 16 rows 12.7) */
static size_t blue_chunk_bytes(void) { return hs_env_mb("HSFFT_BLUE_CHUNK_MB", 4096.0); }

/* ------------------------------------------------------------------ device state */
static int run_chain(hs_entry *e, hs_devstate *ds, const void *I, long long idist, void *O, long long odist,
                     int batch, int sgn, int conj, int dir, int load_op, const void *laux, int store_op,
                     const void *saux, long long nsig);

static hs_devstate *devstate(hs_entry *e)
{
    const int d = hsd_get_device();
    if (d < 0 || d >= HS_MAX_DEV) {
        hs_seterr("invalid current device %d", d);
        return NULL;
    }
    /* bumped by hsfft_plan_refresh from any thread, read here under the device lock: atomic */
    const int ver = __atomic_load_n(&e->version, __ATOMIC_ACQUIRE);
    if (e->ds[d] && e->ds_version[d] == ver) return e->ds[d];
    retire_devstate(e->ds[d]); /* a concurrent small call may still hold it */
    e->ds[d] = NULL;
    hs_devstate *s = calloc(1, sizeof *s);
    /* the one schedule whose kernel reads it -- the whole-row [3,3,5,5,7,8] pass (12600, the
     * mr::k_row2 F45 kernel) -- also gets its last stage's twiddles transposed to [i-1][k] at
     * d_tw + M (one 16-B word per lane, lanes on consecutive k); the launch is told by
     * hsd_launch.tw_t, so no other kernel can read an unbuilt region */
    static const int row_r[6] = {3, 3, 5, 5, 7, 8};
    int trl = e->lt == 0 && e->npass == 1 && e->pass[0].variant == HS_KV_MR && e->pass[0].nst == 6;
    for (int i = 0; trl && i < 6; i++) trl = e->pass[0].radix[i] == row_r[i];
    const size_t twb = sizeof(fft_data) * (size_t)(e->M > 1 ? e->M : 1) * (trl ? 2 : 1);
    const fft_data *twsrc = e->tw_from_struct ? e->key->twiddle : e->tw_private;
    s->d_tw = hsd_malloc(twb);
    if (!s->d_tw || hsd_h2d(s->d_tw, twsrc, sizeof(fft_data) * (size_t)(e->M > 1 ? e->M - 1 : 0))) goto fail;
    if (trl) {
        const int r = e->stage_r[e->nst - 1], L = e->M / r;
        fft_data *t = malloc(sizeof(fft_data) * (size_t)(r - 1) * (size_t)L);
        if (!t) goto fail;
        for (int k = 0; k < L; k++)
            for (int i = 0; i < r - 1; i++) t[(size_t)i * L + k] = twsrc[L - 1 + (r - 1) * k + i];
        const int rc = hsd_h2d((fft_data *)s->d_tw + e->M, t, sizeof(fft_data) * (size_t)(r - 1) * (size_t)L);
        free(t);
        if (rc) goto fail;
    }
    if (e->ngcs) {
        s->d_gcs = hsd_malloc(sizeof(double) * (size_t)e->ngcs);
        if (!s->d_gcs || hsd_h2d(s->d_gcs, e->gcs, sizeof(double) * (size_t)e->ngcs)) goto fail;
    }
    if (e->lt == 1) {
        const int N = e->N, M = e->M;
        s->d_chirp = hsd_malloc(sizeof(fft_data) * (size_t)N);
        s->d_hk = hsd_malloc(sizeof(fft_data) * (size_t)M);
        if (!s->d_chirp || !s->d_hk || hsd_h2d(s->d_chirp, e->chirp, sizeof(fft_data) * (size_t)N)) goto fail;
        /* hk = FFT_M(hl / M): padded + mirrored chirp (ref :1692-1703), scaled (:1787-1792),
         * transformed with the plan's own sign and twiddles (:1797) -- once per plan */
        fft_data *hl = calloc((size_t)M, sizeof(fft_data));
        const double scale = 1.0 / M;
        for (int i = 0; i < M; i++) {
            fft_data v = {0.0, 0.0};
            if (i < N) v = e->chirp[i];
            else if (i >= M - N + 1) v = e->chirp[M - i];
            hl[i].im = v.im * scale;
            hl[i].re = v.re * scale;
        }
        void *d_hl = hsd_malloc(sizeof(fft_data) * (size_t)M);
        int rc = d_hl ? hsd_h2d(d_hl, hl, sizeof(fft_data) * (size_t)M) : -1;
        free(hl);
        e->ds[d] = s; /* run_chain needs the twiddles */
        if (!rc) rc = run_chain(e, s, d_hl, M, s->d_hk, M, 1, e->sgn, 0, e->sgn, HS_LOAD_PLAIN, NULL,
                                HS_STORE_PLAIN, NULL, M);
        if (!rc) rc = hsd_sync();
        hsd_free(d_hl);
        e->ds[d] = NULL;
        if (rc) goto fail;
    }
    s->tw_t = trl;
    e->ds[d] = s;
    e->ds_version[d] = ver;
    return s;
fail:
    if (!g_errbuf[0]) hs_seterr("device state: %s", hsd_errstr());
    free_devstate(s);
    return NULL;
}

/* ------------------------------------------------------------------ pass chains */
/* this thread's completion word for its next launch (small host-buffer path): set by the
 * caller, consumed by launch_pass; t_done_armed says whether the kernel took it */
static __thread unsigned *t_done;
static __thread unsigned t_done_val;
static __thread int t_done_armed;

static int launch_pass(hs_entry *e, hs_devstate *ds, int i, const void *in, long long idist, void *out,
                       long long odist, int batch, int sgn, int conj, int dir, int load_op, const void *laux,
                       int store_op, const void *saux, long long nsig)
{
    hsd_launch l;
    memset(&l, 0, sizeof l);
    if (t_done) {
        l.done = t_done;
        l.done_val = t_done_val;
        l.armed = &t_done_armed;
        t_done = NULL;
    }
    l.in = in;
    l.out = out;
    l.idist = idist;
    l.odist = odist;
    l.batch = batch;
    l.sgn = sgn;
    l.dir = dir;
    l.conj = conj;
    l.tw = ds->d_tw;
    l.tw_t = ds->tw_t;
    l.gcs = (const double *)ds->d_gcs;
    l.load_op = load_op;
    l.load_aux = laux;
    l.store_op = store_op;
    l.store_aux = saux;
    l.nsig = nsig;
#ifdef HSFFT_DEV_PROBES
    /* development build only: every row aliased to one buffer (on-die timing, results wrong) */
    if (env_int("HSFFT_DEV_ALIAS", 0) & 1) l.idist = l.odist = 0;
#endif
    int rc = hsd_run_pass(&e->pass[i], &l);
    if (rc) hs_seterr("pass %d: %s", i, hsd_errstr());
    return rc;
}

#ifdef HSFFT_DEV_PROBES
/* Development build only (round 6: measured slower, 52-67 vs 91 GSamples/s on c2 -- DESIGN.md
 * §5).  Two-pass chain over the batch in chunks of `chunk` rows, software-pipelined over two
 * streams: pass A of chunk k+1 (library stream) overlaps pass B of chunk k (second stream),
 * ordered by events; at most `lag` chunks run ahead so the in-flight intermediates stay in
 * the 256 MiB Infinity Cache.  The library stream waits for the last pass B at the end. */
static int run_pipelined(hs_entry *e, hs_devstate *ds, const void *I, long long idist, void *O, long long odist,
                         int batch, int chunk, int sgn, int conj, int dir, int load_op, const void *laux,
                         int store_op, const void *saux, long long nsig)
{
    const int lag = env_int("HSFFT_PIPE_LAG", 2);
    int rc = 0, k = 0;
    for (long long c0 = 0; c0 < batch && !rc; c0 += chunk, k++) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        fft_data *W = (fft_data *)O + c0 * odist;
        hsd_select_stream(0);
        if (k >= lag) rc = hsd_event_wait(2 * (k - lag) + 1); /* pass B of chunk k-lag done */
        if (!rc) rc = launch_pass(e, ds, 0, (const fft_data *)I + c0 * idist, idist, W, odist, cb, sgn, conj, dir,
                                  load_op, laux, HS_STORE_PLAIN, NULL, nsig);
        if (!rc) rc = hsd_event_record(2 * k);
        hsd_select_stream(1);
        if (!rc) rc = hsd_event_wait(2 * k);
        if (!rc) rc = launch_pass(e, ds, 1, W, odist, W, odist, cb, sgn, conj, dir, HS_LOAD_PLAIN, NULL, store_op,
                                  saux, nsig);
        if (!rc) rc = hsd_event_record(2 * k + 1);
    }
    hsd_select_stream(0);
    if (!rc && k > 0) rc = hsd_event_wait(2 * (k - 1) + 1);
    return rc;
}
#endif

/* One mixed-radix transform of length M per row, chained over the plan's passes.  Reads
 * I (never written), writes O.  Intermediate buffers come from the scratch pool; the last
 * pass (A == 1: it reads and writes the same element set per tile) may run in place on O
 * when O is a plain M-length row buffer. */
static int run_chain(hs_entry *e, hs_devstate *ds, const void *I, long long idist, void *O, long long odist,
                     int batch, int sgn, int conj, int dir, int load_op, const void *laux, int store_op,
                     const void *saux, long long nsig)
{
    const int n = e->npass;
    const long long M = e->M;
    if (M == 1 || n == 0) { /* N == 1: the reference copies (ref :332-342) */
        for (int b = 0; b < batch; b++)
            if (hsd_d2d_async((fft_data *)O + b * odist, (const fft_data *)I + b * idist, sizeof(fft_data))) return -2;
        return 0;
    }
    if (n == 1)
        return launch_pass(e, ds, 0, I, idist, O, odist, batch, sgn, conj, dir, load_op, laux, store_op, saux, nsig);
    const int last_inplace = store_op != HS_STORE_CHIRP && odist == M;
    /* passes 0..n-2 write scratch except that pass n-2 writes O when the last pass can run
     * in place; consecutive scratch writes alternate between two buffers */
    const int writes = (n - 1) - (last_inplace ? 1 : 0);
    const int need = writes < 2 ? writes : 2;
    long long chunk = batch;
    if (need) {
        long long per = (long long)(chunk_bytes() / (sizeof(fft_data) * (size_t)M));
        if (per < 1) per = 1;
        if (chunk > per) chunk = per;
    }
#ifdef HSFFT_DEV_PROBES
    else { /* development build only: all passes over a few rows at a time, the intermediate in
            * the 256 MiB Infinity Cache between passes (HSFFT_MALL_ROWS; measured slower) */
        const int rows = env_int("HSFFT_MALL_ROWS", 0);
        if (rows > 0 && chunk > rows) chunk = rows;
    }
#endif
    void *S[2] = {NULL, NULL};
    for (int k = 0; k < need; k++) {
        S[k] = hs_scratch(k, sizeof(fft_data) * (size_t)(chunk * M));
        if (!S[k]) {
            hs_seterr("scratch allocation of %lld bytes failed", (long long)(chunk * M * 16));
            return HSFFT_ERR_NOMEM;
        }
    }
#ifdef HSFFT_DEV_PROBES
    if (!need && n == 2 && chunk < batch && env_int("HSFFT_PIPE", 0))
        return run_pipelined(e, ds, I, idist, O, odist, batch, (int)chunk, sgn, conj, dir, load_op, laux, store_op,
                             saux, nsig);
    const int dev_np = env_int("HSFFT_DEV_NPASS", 0); /* development build only: stop after this many passes */
#else
    const int dev_np = 0;
#endif
    for (long long c0 = 0; c0 < batch; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        const void *R = (const fft_data *)I + c0 * idist;
        long long rdist = idist;
        int lop = load_op, j = 0;
        for (int i = 0; i < (dev_np > 0 && dev_np < n ? dev_np : n); i++) {
            void *W;
            long long wdist;
            if (i == n - 1 || (i == n - 2 && last_inplace)) {
                W = (fft_data *)O + c0 * odist;
                wdist = odist;
            } else {
                W = S[j++ & 1];
                wdist = M;
            }
            const int sop = i == n - 1 ? store_op : HS_STORE_PLAIN;
            int rc = launch_pass(e, ds, i, R, rdist, W, wdist, cb, sgn, conj, dir, lop, laux, sop, saux, nsig);
            if (rc) return rc;
            R = W;
            rdist = wdist;
            lop = HS_LOAD_PLAIN;
        }
    }
    return 0;
}

/* persistent Bluestein launches whose rows ran on the three-launch path instead (grid not
 * co-resident, or waits timed out in a synchronous call); hsfft_bluestein_fallbacks() */
static void thread_resources_used(int d);
static long long g_blue_fallbacks;

long long hsfft_thread_streams_created(void) { return hsd_thread_streams_created(); }
long long hsfft_bluestein_fallbacks(void) { return __atomic_load_n(&g_blue_fallbacks, __ATOMIC_RELAXED); }

/* Bluestein (ref :1735-1907) on rows of length N: pre-multiply fused into the first pass of
 * FFT #2, the spectrum product into its last pass, FFT #3 runs with conjugated twiddles and
 * sign -sgn, the post-multiply is fused into its last pass.  hk was computed once per plan. */
static int run_bluestein(hs_entry *e, hs_devstate *ds, const void *in, long long idist, void *out, long long odist,
                         int batch)
{
    const long long M = e->M, N = e->N;
    long long chunk = (long long)(blue_chunk_bytes() / (sizeof(fft_data) * (size_t)M));
    if (chunk < 1) chunk = 1;
    if (chunk > batch) chunk = batch;
    /* M = 512 x 512 as two [8,8,8] passes: the forward FFT's last pass, the spectrum product
     * and the inverse FFT's first pass run as one kernel (the columns coincide) */
    const hsd_pass *p0 = &e->pass[0], *p1 = &e->pass[1];
    const int fuse = e->npass == 2 && M == 512 * 512 && p0->P == 512 && p1->P == 512 && p0->nst == 3 &&
                     p1->nst == 3 && p0->variant == HS_KV_R8X3 && p1->variant == HS_KV_R8X3 &&
                     p0->radix[0] == 8 && !env_int("HSFFT_BLUE_NOFUSE", 0);
    /* one persistent launch per 65536 rows (hsfft_blue_xcd.h): groups of 64 workgroups carry
     * one row at a time through all three kernels, the intermediates stay on die
     * (HSFFT_BLUE_XCD=0: three launches per chunk).  A grid that cannot be co-resident is
     * refused on the host and its rows run on the three-launch path below at once.  Device-
     * buffer batched calls are asynchronous (a timed-out wait is reported by the caller's next
     * hsfft_synchronize()); synchronous entry points (t_sync_call) and HSFFT_BX_SYNC=1 wait,
     * and a launch whose waits timed out makes its rows run on the three-launch path as well.
     * Both count as fallbacks. */
    const int ng = env_int("HSFFT_BLUE_XCD", 8);
    const int sync = t_sync_call > 0 || env_int("HSFFT_BX_SYNC", 0) ? 1 : t_deferred_call > 0 ? 2 : 0;
    long long done = 0;
    if (fuse && ng > 0 && !t_no_xcd) {
        thread_resources_used(hsd_get_device()); /* this thread's error words are recycled when it exits */
        const size_t ib = (size_t)ng * 4 * sizeof(fft_data) * (size_t)M; /* 4 images per group */
        void *img = hs_scratch(3, ib);
        int rc = img ? 0 : 1;
        for (long long c0 = 0; c0 < batch && rc == 0; c0 += 65536) {
            const int cb = (int)(batch - c0 < 65536 ? batch - c0 : 65536);
            rc = hsd_blue_xcd((const fft_data *)in + c0 * idist, idist, (fft_data *)out + c0 * odist, odist, ds->d_tw,
                              ds->d_chirp, ds->d_hk, img, ib, N, cb, e->sgn, ng, sync);
            if (rc == 0) done = c0 + cb;
        }
        if (rc < 0) {
            hs_seterr("bluestein persistent launch: %s", hsd_errstr());
            return HSFFT_ERR_DEVICE;
        }
        if (rc == 2 || rc == 3) __atomic_fetch_add(&g_blue_fallbacks, 1, __ATOMIC_RELAXED);
        if (done == batch) return 0;
    }
    if (done) {
        in = (const fft_data *)in + done * idist;
        out = (fft_data *)out + done * odist;
        batch -= (int)done;
        if (chunk > batch) chunk = batch;
    }
    /* the two M-point intermediates; halved while the allocation fails (a fuller device runs
     * in smaller chunks) */
    void *mid = NULL, *mid2 = NULL;
    for (;;) {
        mid = hs_scratch(3, sizeof(fft_data) * (size_t)(chunk * M));
        mid2 = fuse && mid ? hs_scratch(8, sizeof(fft_data) * (size_t)(chunk * M)) : NULL;
        if ((mid && (mid2 || !fuse)) || chunk == 1) break;
        chunk = (chunk + 1) / 2;
    }
    if (!mid || (fuse && !mid2)) {
        hs_seterr("bluestein scratch allocation of %lld bytes failed", (long long)(chunk * M * 16));
        return HSFFT_ERR_NOMEM;
    }
#ifdef HSFFT_DEV_PROBES
    /* development build only (results WRONG): every row of a chunk uses the same M-point
     * intermediate, so the hand-offs between the three kernels stay on die */
    const long long md = (env_int("HSFFT_DEV_ALIAS", 0) & 2) ? 0 : M;
#else
    const long long md = M;
#endif
    for (long long c0 = 0; c0 < batch && fuse; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        int rc = hsd_blue_first((const fft_data *)in + c0 * idist, idist, mid, md, ds->d_tw, ds->d_chirp, N, cb, e->sgn);
        if (rc < 0) hs_seterr("bluestein first pass: %s", hsd_errstr());
        if (rc == 1)
            rc = launch_pass(e, ds, 0, (const fft_data *)in + c0 * idist, idist, mid, M, cb, e->sgn, 0, e->sgn,
                             HS_LOAD_CHIRP, ds->d_chirp, HS_STORE_PLAIN, NULL, N);
        if (!rc && hsd_blue_mid(mid, mid2, md, ds->d_tw, ds->d_hk, cb, e->sgn, 0, e->sgn, -1 * e->sgn, 1)) {
            hs_seterr("bluestein middle: %s", hsd_errstr());
            rc = HSFFT_ERR_DEVICE;
        }
        if (!rc) {
            rc = hsd_blue_last(mid2, md, (fft_data *)out + c0 * odist, odist, ds->d_tw, ds->d_chirp, N, cb, e->sgn);
            if (rc < 0) hs_seterr("bluestein last pass: %s", hsd_errstr());
            if (rc == 1)
                rc = launch_pass(e, ds, 1, mid2, M, (fft_data *)out + c0 * odist, odist, cb, -1 * e->sgn, 1, e->sgn,
                                 HS_LOAD_PLAIN, NULL, HS_STORE_CHIRP, ds->d_chirp, N);
        }
        if (rc) return rc;
    }
    for (long long c0 = 0; c0 < batch && !fuse; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        int rc = run_chain(e, ds, (const fft_data *)in + c0 * idist, idist, mid, M, cb, e->sgn, 0, e->sgn,
                           HS_LOAD_CHIRP, ds->d_chirp, HS_STORE_SPEC, ds->d_hk, N);
        if (!rc)
            rc = run_chain(e, ds, mid, M, (fft_data *)out + c0 * odist, odist, cb, -1 * e->sgn, 1, e->sgn,
                           HS_LOAD_PLAIN, NULL, HS_STORE_CHIRP, ds->d_chirp, N);
        if (rc) return rc;
    }
    return 0;
}

int hs_r2c_fused(hs_entry *e, const void *in, long long idist, void *Z, void *X, long long xdist, const void *tw2,
                 int batch, int compact)
{
    const hsd_pass *p0 = &e->pass[0], *p1 = &e->pass[1];
    if (e->lt != 0 || e->npass != 2 || p1->variant != HS_KV_R8X3 || p1->nst != 3 || p1->P != 512 || p1->A != 1 ||
        p1->B % 16 || p0->B != 1 || !env_int("HSFFT_R2C_FUSE", 1))
        return 1; /* HSFFT_R2C_FUSE=0: pass B + k_r2c_post2 (r2c 2^22: 85 vs 93 GSamples/s fused) */
    hs_devstate *ds = devstate(e);
    if (!ds) return HSFFT_ERR_DEVICE;
    /* HSFFT_R2C_OVL = S (measurement, development build; 27.97 / 24.75 / 23.87 vs 22.32 ms per
     * 512 rows for S = 32 / 64 / 128): the call in sub-chunks of S rows, pass A of every
     * sub-chunk on the library stream and the split walk of sub-chunk s on the pipeline stream
     * behind pass A(s) only, so the walks (latency-bound) overlap the later pass As
     * (bandwidth-bound); Z holds every row, so nothing is reused; the library stream then waits
     * for the last walk */
#ifdef HSFFT_DEV_PROBES
    const int ovl = env_int("HSFFT_R2C_OVL", 0); /* development build only: measured slower */
    if (ovl > 0 && batch > ovl && hsd_stream_index() == 0) {
        const int ns = (batch + ovl - 1) / ovl;
        int rc = 0;
        for (int s = 0; s < ns && !rc; s++) {
            const long long r0 = (long long)s * ovl;
            const int nb = (int)(batch - r0 < ovl ? batch - r0 : ovl);
            void *Zs = (char *)Z + r0 * e->M * (long long)sizeof(fft_data);
            hsd_select_stream(0);
            rc = launch_pass(e, ds, 0, (const char *)in + r0 * idist * (long long)sizeof(fft_data), idist, Zs, e->M,
                             nb, e->sgn, 0, e->sgn, HS_LOAD_PLAIN, NULL, HS_STORE_PLAIN, NULL, e->M);
            if (!rc) rc = hsd_event_record(2 * s) ? HSFFT_ERR_DEVICE : 0;
            hsd_select_stream(1);
            if (!rc) rc = hsd_event_wait(2 * s) ? HSFFT_ERR_DEVICE : 0;
            if (!rc && hsd_r2c_last(Zs, e->M, (char *)X + r0 * xdist * (long long)sizeof(fft_data), xdist, ds->d_tw,
                                    tw2, e->M, p1->B, nb, e->sgn, compact)) {
                hs_seterr("r2c last pass: %s", hsd_errstr());
                rc = HSFFT_ERR_DEVICE;
            }
            if (!rc) rc = hsd_event_record(2 * s + 1) ? HSFFT_ERR_DEVICE : 0;
        }
        hsd_select_stream(0);
        if (!rc) rc = hsd_event_wait(2 * (ns - 1) + 1) ? HSFFT_ERR_DEVICE : 0;
        return rc;
    }
#endif
    int rc = launch_pass(e, ds, 0, in, idist, Z, e->M, batch, e->sgn, 0, e->sgn, HS_LOAD_PLAIN, NULL, HS_STORE_PLAIN,
                         NULL, e->M);
    if (!rc && hsd_r2c_last(Z, e->M, X, xdist, ds->d_tw, tw2, e->M, p1->B, batch, e->sgn, compact)) {
        hs_seterr("r2c last pass: %s", hsd_errstr());
        rc = HSFFT_ERR_DEVICE;
    }
    return rc;
}

int hs_c2c_rows(hs_entry *e, const void *in, long long idist, void *out, long long odist, int batch)
{
    hs_devstate *ds = devstate(e);
    if (!ds) return HSFFT_ERR_DEVICE;
    if (e->lt == 1) return run_bluestein(e, ds, in, idist, out, odist, batch);
    return run_chain(e, ds, in, idist, out, odist, batch, e->sgn, 0, e->sgn, HS_LOAD_PLAIN, NULL, HS_STORE_PLAIN,
                     NULL, e->M);
}

/* ------------------------------------------------------------------ drop-in fft_exec */
/* Small host-pointer transforms (one pass, rows up to HSFFT_SMALL_KB, default 1 MiB): the
 * rows are copied into page-locked host slots and the kernel reads and writes them over the
 * host link directly -- no H2D / D2H copy launches, one kernel launch and one wait per call
 * (BASELINE config 1, N = 1024).  Per-device slots, used under the device lock. */
static int small_host_exec(hs_entry *e, const fft_data *inp, fft_data *oup, size_t bytes)
{
    const int d = hsd_get_device();
    if (d < 0 || d >= HS_MAX_DEV) return 1;
    if (g_pin_sz[d] < bytes) {
        hsd_host_free(g_pin[d][0]);
        hsd_host_free(g_pin[d][1]);
        g_pin[d][0] = hsd_host_alloc(bytes);
        g_pin[d][1] = hsd_host_alloc(bytes);
        g_pin_sz[d] = g_pin[d][0] && g_pin[d][1] ? bytes : 0;
        if (!g_pin_sz[d]) return 1; /* no pinned memory: the staged path */
    }
    memcpy(g_pin[d][0], inp, bytes);
    int rc = hs_c2c_rows(e, g_pin[d][0], e->N, g_pin[d][1], e->N, 1);
    if (!rc) rc = hsd_sync();
    if (!rc) memcpy(oup, g_pin[d][1], bytes);
    return rc;
}

static void fft_exec_locked(fft_object obj, fft_data *inp, fft_data *oup)
{
    if (obj == NULL || inp == NULL || oup == NULL) {
        fprintf(stderr, "Error: Invalid FFT object or data pointers\n");
        exit(EXIT_FAILURE);
    }
    if (obj->lt != 0 && obj->lt != 1) {
        fprintf(stderr, "Error: Invalid FFT object type (lt = %d)\n", obj->lt);
        exit(EXIT_FAILURE);
    }
    g_errbuf[0] = 0;
    if (hs_require_gpu()) fatal("fft_exec needs an MI355X");
    hs_entry *e = hs_entry_get(obj);
    if (!e) fatal("fft_exec: invalid plan");
    t_sync_call++;
    const int N = obj->N;
    const size_t bytes = sizeof(fft_data) * (size_t)N;
    const int din = hsd_is_device_ptr(inp), dout = hsd_is_device_ptr(oup);
    int rc;
    const size_t small = (size_t)env_int("HSFFT_SMALL_KB", 1024) * 1024;
    if (din && dout && inp != oup) {
        rc = hs_c2c_rows(e, inp, N, oup, N, 1);
    } else if (!din && !dout && e->lt == 0 && e->npass == 1 && bytes <= small &&
               (rc = small_host_exec(e, inp, oup, bytes)) <= 0) {
        /* done (rc 0) or failed (rc < 0) on the pinned path */
    } else {
        /* host (or aliased) buffers: staged through device memory, synchronous */
        fft_data *di = hs_scratch(5, bytes), *dq = hs_scratch(6, bytes);
        if (!di || !dq) fatal("fft_exec: device staging allocation failed");
        rc = din ? hsd_d2d_async(di, inp, bytes) : hsd_h2d(di, inp, bytes);
        if (!rc) rc = hs_c2c_rows(e, di, N, dq, N, 1);
        if (!rc) rc = dout ? hsd_d2d_async(oup, dq, bytes) : hsd_d2h(oup, dq, bytes);
    }
    if (!rc) rc = hsd_sync();
    t_sync_call--;
    hs_entry_put(e);
    if (rc) fatal("fft_exec failed");
}

/* Small host-buffer transforms without the device lock: one-pass mixed-radix plans on host
 * buffers run on this thread's own stream with this thread's own page-locked slots, so
 * threads calling fft_exec at once overlap their launches, transfers and waits instead of
 * taking turns on the device lock (the reference's fft_exec is reentrant on a shared plan,
 * highSpeedFFT.c:1920-1942).  The device lock is held only while the plan's device state is
 * built.  Returns 1 when the call does not qualify (then the locked path runs). */
static __thread void *t_pin[HS_MAX_DEV][2];
static __thread size_t t_pin_sz[HS_MAX_DEV];
/* this thread's completion word per device (page-locked) and its sequence */
static __thread unsigned *t_flag[HS_MAX_DEV];
/* the value this thread's next completion word on device d must reach: it travels WITH the word
 * when a set is parked and adopted (a new owner restarting at 1 would take the previous owner's
 * last value, if it was 1, for its own first completion -- round 6, caught by
 * test_thread_generations_recycle_resources) */
static __thread unsigned t_seq[HS_MAX_DEV];

/* Per-thread resources (page-locked slots, completion words, the thread's own streams and
 * persistent-launch error words) are recycled, not destroyed, when the thread exits: a pthread
 * key whose destructor runs in the exiting thread parks them in the device layer's pool
 * (hsd_thread_park, no HIP call -- round 5: under rocprofv3 a HIP call there aborted the
 * process), and a thread's first use of a device adopts a parked set (hsd_thread_adopt).  So a
 * caller that recycles or spawns threads neither leaks pinned memory or streams nor pays for
 * creating and destroying them; hsfft_release_scratch / hsfft_finalize destroy the pool. */
static pthread_key_t g_tkey;
static pthread_once_t g_tkey_once = PTHREAD_ONCE_INIT;
static __thread unsigned t_adopted; /* bit d: this thread has taken its set of device d */

static void thread_resources_free(void *unused)
{
    (void)unused;
    for (int d = 0; d < HS_MAX_DEV; d++) {
        const hsd_tset h = {{t_pin[d][0], t_pin[d][1]}, t_pin_sz[d], t_flag[d], t_seq[d]};
        hsd_thread_park(d, &h);
        t_pin[d][0] = t_pin[d][1] = NULL;
        t_pin_sz[d] = 0;
        t_flag[d] = NULL;
    }
    t_adopted = 0;
}

/* hsfft_finalize: the calling (live) thread's page-locked slots and words, at once */
static void thread_pins_free_now(void)
{
    for (int d = 0; d < HS_MAX_DEV; d++) {
        hsd_host_free(t_pin[d][0]);
        hsd_host_free(t_pin[d][1]);
        hsd_host_free(t_flag[d]);
        t_pin[d][0] = t_pin[d][1] = NULL;
        t_pin_sz[d] = 0;
        t_flag[d] = NULL;
    }
    t_adopted = 0; /* a later first use may adopt a parked set again */
}

static void tkey_init(void) { pthread_key_create(&g_tkey, thread_resources_free); }

/* this thread is about to use its own resources on device d: arm the exit destructor, and on
 * the thread's first use of d take a set an exited thread parked (if any) */
static void thread_resources_used(int d)
{
    pthread_once(&g_tkey_once, tkey_init);
    if (!pthread_getspecific(g_tkey)) pthread_setspecific(g_tkey, (void *)1);
    if (d < 0 || d >= HS_MAX_DEV || (t_adopted >> d & 1u)) return;
    t_adopted |= 1u << d;
    hsd_tset h;
    if (!t_pin[d][0] && !t_pin[d][1] && !t_flag[d] && hsd_thread_adopt(d, &h)) {
        t_pin[d][0] = h.pin[0];
        t_pin[d][1] = h.pin[1];
        t_pin_sz[d] = h.pin_sz;
        t_flag[d] = h.flag;
        t_seq[d] = h.seq; /* the word holds the previous owner's last value: continue after it */
    }
}

static int small_host_exec_concurrent(fft_object obj, fft_data *inp, fft_data *oup)
{
    if (obj == NULL || inp == NULL || oup == NULL || (obj->lt != 0 && obj->lt != 1)) return 1; /* locked path reports */
    if (obj->lt != 0 || !env_int("HSFFT_SMALL_CONCURRENT", 1)) return 1;
    g_errbuf[0] = 0;
    if (hs_require_gpu()) return 1;
    const size_t bytes = sizeof(fft_data) * (size_t)obj->N;
    if (bytes > (size_t)env_int("HSFFT_SMALL_KB", 1024) * 1024) return 1;
    const int d = hsd_get_device();
    if (d < 0 || d >= HS_MAX_DEV || hsd_is_device_ptr(inp) || hsd_is_device_ptr(oup)) return 1;
    hs_entry *e = hs_entry_get(obj);
    if (!e) return 1;
    if (e->lt != 0 || e->npass != 1) {
        hs_entry_put(e);
        return 1;
    }
    hs_lock_device(); /* the plan's device state is built once, under the lock */
    hs_devstate *ds = devstate(e);
    if (ds) ds->refs++; /* pinned until this call has completed (a refresh retires, never frees it) */
    hs_unlock_device(d);
    if (!ds) {
        hs_entry_put(e);
        return 1;
    }
    thread_resources_used(d);
    if (t_pin_sz[d] < bytes) {
        hsd_host_free(t_pin[d][0]);
        hsd_host_free(t_pin[d][1]);
        t_pin[d][0] = hsd_host_alloc(bytes);
        t_pin[d][1] = hsd_host_alloc(bytes);
        t_pin_sz[d] = t_pin[d][0] && t_pin[d][1] ? bytes : 0;
        if (!t_pin_sz[d]) {
            hs_lock_device();
            devstate_put(ds);
            hs_unlock_device(d);
            hs_entry_put(e);
            return 1;
        }
    }
    const int fmode = env_int("HSFFT_SMALL_FLAG", 2);
    if (!t_flag[d] && fmode) {
        t_flag[d] = (unsigned *)hsd_host_alloc(64);
        if (t_flag[d]) memset(t_flag[d], 0, 64); /* no stale value can match the next sequence */
        t_seq[d] = 0;
    }
    const int use_flag = fmode >= 1 && t_flag[d] != NULL; /* the mode of THIS call, not of the first */
    memcpy(t_pin[d][0], inp, bytes);
    hsd_select_stream(3);
    t_done_armed = 0;
    if (use_flag) {
        if (++t_seq[d] == 0) t_seq[d] = 1;
        if (fmode >= 2) { /* a one-workgroup kernel stores the word itself */
            t_done = t_flag[d];
            t_done_val = t_seq[d];
        }
    }
    int rc = run_chain(e, ds, t_pin[d][0], obj->N, t_pin[d][1], obj->N, 1, e->sgn, 0, e->sgn, HS_LOAD_PLAIN, NULL,
                       HS_STORE_PLAIN, NULL, e->M);
    t_done = NULL;
    if (!rc) {
        /* completion seen through a host word instead of the stream wait: stored by the
         * kernel (HSFFT_SMALL_FLAG=2, one-workgroup launches), else by the command processor
         * after the kernel (1); 0: the stream wait */
        if (use_flag && t_done_armed) rc = hsd_host_word_wait(t_flag[d], t_seq[d]);
        else if (use_flag) rc = hsd_stream_signal_wait(t_flag[d], t_seq[d]);
        else rc = hsd_stream_sync();
    }
    if (rc) hsd_stream_sync(); /* nothing of this call may still run when the pin is dropped */
    hsd_select_stream(0);
    hs_lock_device();
    devstate_put(ds);
    hs_unlock_device(d);
    hs_entry_put(e);
    if (rc) fatal("fft_exec failed");
    memcpy(oup, t_pin[d][1], bytes);
    return 0;
}

void fft_exec(fft_object obj, fft_data *inp, fft_data *oup)
{
    hs_env_begin(); /* this call's knob lookups: one snapshot (see hs_getenv) */
    const int small = small_host_exec_concurrent(obj, inp, oup);
    hs_env_end();
    if (small == 0) return;
    const int d = hs_lock_device();
    fft_exec_locked(obj, inp, oup);
    hs_unlock_device(d);
}

/* ------------------------------------------------------------------ extension API */
int hsfft_device_count(void) { return hsd_device_count(); }
int hsfft_set_device(int dev)
{
    const int rc = hsd_set_device(dev) ? HSFFT_ERR_DEVICE : 0;
    hs_crash_trace_install(); /* after the runtime (and any tool) initialised: ours wins */
    return rc;
}
int hsfft_get_device(void) { return hsd_get_device(); }
void *hsfft_malloc(size_t bytes) { return hs_require_gpu() ? NULL : hsd_malloc(bytes); }
int hsfft_free(void *p) { return hsd_free(p) ? HSFFT_ERR_DEVICE : 0; }
int hsfft_memcpy_h2d(void *d, const void *h, size_t n) { return hsd_h2d(d, h, n) ? HSFFT_ERR_DEVICE : 0; }
int hsfft_memcpy_d2h(void *h, const void *d, size_t n) { return hsd_d2h(h, d, n) ? HSFFT_ERR_DEVICE : 0; }
int hsfft_memset(void *d, int v, size_t n) { return hsd_memset_async(d, v, n) ? HSFFT_ERR_DEVICE : 0; }
int hsfft_synchronize(void)
{
    g_errbuf[0] = 0;
    if (hsd_sync_report()) {
        hs_seterr("hsfft_synchronize: %s", hsd_errstr());
        return HSFFT_ERR_DEVICE;
    }
    return 0;
}
void *hsfft_get_stream(void) { return hsd_stream(); }

int hsfft_plan_refresh(fft_object obj)
{
    if (!obj) return HSFFT_ERR_ARG;
    hs_entry *e = hs_entry_get(obj);
    if (!e) return HSFFT_ERR_ARG;
    __atomic_fetch_add(&e->version, 1, __ATOMIC_ACQ_REL);
    hs_entry_put(e);
    return 0;
}

int hsfft_plan_num_passes(fft_object obj)
{
    if (!obj) return HSFFT_ERR_ARG;
    hs_entry *e = hs_entry_get(obj);
    const int n = e ? e->npass : HSFFT_ERR_ARG;
    hs_entry_put(e);
    return n;
}

static int drmap(const struct fft_set *o, int *map, int oo, int io, int stride, int n, int fi)
{
    if (n == 1 || is_leaf_len(n)) { /* leaf gather: out slot oo+i <- in index io+i*stride */
        for (int i = 0; i < n; i++) map[oo + i] = io + i * stride;
        return 0;
    }
    if (fi >= o->lf || o->factors[fi] <= 1 || n % o->factors[fi]) return HSFFT_ERR_ARG;
    const int r = o->factors[fi], L = n / r;
    for (int i = 0; i < r; i++)
        if (drmap(o, map, oo + i * L, io + i * stride, stride * r, L, fi + 1)) return HSFFT_ERR_ARG;
    return 0;
}

int hsfft_digit_reverse_map(fft_object obj, int *map)
{
    if (!obj || !map || obj->lt != 0 || obj->N < 1) return HSFFT_ERR_ARG;
    return drmap(obj, map, 0, 0, 1, obj->N, 0);
}

int hsfft_exec_batched(fft_object obj, const fft_data *d_in, fft_data *d_out, int batch)
{
    g_errbuf[0] = 0;
    if (!obj || !d_in || !d_out || batch < 0 || d_in == d_out) {
        hs_seterr("hsfft_exec_batched: invalid arguments");
        return HSFFT_ERR_ARG;
    }
    if (batch == 0) return 0;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    hs_entry *e = hs_entry_get(obj);
    rc = e ? hs_c2c_rows(e, d_in, obj->N, d_out, obj->N, batch) : HSFFT_ERR_ARG;
    hs_entry_put(e);
    hs_unlock_device(d);
    return rc;
}

/* Host-resident batch: rows are streamed through two HBM staging
 * slots in chunks, H2D on stream 1, the transform on the library stream, D2H on stream 2,
 * ordered by events so that chunk k+1's upload and chunk k-1's download overlap chunk k's
 * transform (PCIe-bound).  Caller buffers are page-locked for the call when possible. */
static size_t host_chunk_bytes(void)
{
    const char *s = getenv("HSFFT_HOST_CHUNK_MB");
    size_t v = (size_t)(s ? atof(s) : 256.0) * (1u << 20);
    return v < (1u << 20) ? (1u << 20) : v;
}

static int exec_host_locked(fft_object obj, hs_entry *e, const fft_data *h_in, fft_data *h_out, int batch);

int hsfft_exec_batched_host(fft_object obj, const fft_data *h_in, fft_data *h_out, int batch)
{
    g_errbuf[0] = 0;
    if (!obj || !h_in || !h_out || batch < 0 || h_in == h_out) {
        hs_seterr("hsfft_exec_batched_host: invalid arguments");
        return HSFFT_ERR_ARG;
    }
    if (batch == 0) return 0;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    hs_entry *e = hs_entry_get(obj);
    (void)hsd_blue_deferred_take(); /* a word an earlier, failed pipeline left set (the stream is idle) */
    t_deferred_call++;
    rc = e ? exec_host_locked(obj, e, h_in, h_out, batch) : HSFFT_ERR_ARG;
    t_deferred_call--;
    if (rc == 0 && e && hsd_blue_deferred_take()) {
        /* a persistent Bluestein launch of the pipeline timed out (its waits, or its census): the
         * whole batch again, every Bluestein row on the three-launch path */
        __atomic_fetch_add(&g_blue_fallbacks, 1, __ATOMIC_RELAXED);
        t_no_xcd++;
        t_sync_call++;
        rc = exec_host_locked(obj, e, h_in, h_out, batch);
        t_sync_call--;
        t_no_xcd--;
    }
    hs_entry_put(e);
    hs_unlock_device(d);
    return rc;
}

static int exec_host_locked(fft_object obj, hs_entry *e, const fft_data *h_in, fft_data *h_out, int batch)
{
    int rc = 0;
    const long long N = obj->N;
    const size_t row = sizeof(fft_data) * (size_t)N, total = row * (size_t)batch;
    long long chunk = (long long)(host_chunk_bytes() / row);
    if (chunk < 1) chunk = 1;
    if (chunk > batch) chunk = batch;
    fft_data *din = hs_scratch(7, 2 * row * (size_t)chunk), *dout = hs_scratch(9, 2 * row * (size_t)chunk);
    if (!din || !dout) return HSFFT_ERR_NOMEM;
    const int reg_in = hsd_host_register((void *)h_in, total), reg_out = hsd_host_register(h_out, total);
    enum { EV_H = 40, EV_X = 42, EV_D = 44 };
    int k = 0;
    for (long long c0 = 0; c0 < batch && !rc; c0 += chunk, k++) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk), sl = k & 1;
        fft_data *di = din + (size_t)sl * chunk * N, *dq = dout + (size_t)sl * chunk * N;
        hsd_select_stream(1);
        if (k >= 2) rc = hsd_event_wait(EV_X + sl); /* slot's previous transform has read di */
        if (!rc) rc = hsd_h2d_async(di, h_in + c0 * N, row * (size_t)cb);
        if (!rc) rc = hsd_event_record(EV_H + sl);
        hsd_select_stream(0);
        if (!rc) rc = hsd_event_wait(EV_H + sl);
        if (!rc && k >= 2) rc = hsd_event_wait(EV_D + sl); /* slot's previous output is home */
        if (!rc) rc = hs_c2c_rows(e, di, N, dq, N, cb);
        if (!rc) rc = hsd_event_record(EV_X + sl);
        hsd_select_stream(2);
        if (!rc) rc = hsd_event_wait(EV_X + sl);
        if (!rc) rc = hsd_d2h_async(h_out + c0 * N, dq, row * (size_t)cb);
        if (!rc) rc = hsd_event_record(EV_D + sl);
    }
    for (int st = 2; st >= 0; st--) {
        hsd_select_stream(st);
        if (hsd_stream_sync() && !rc) rc = HSFFT_ERR_DEVICE;
    }
    hsd_select_stream(0);
    if (!rc && hsd_sync()) rc = HSFFT_ERR_DEVICE;
    if (reg_in) hsd_host_unregister((void *)h_in);
    if (reg_out) hsd_host_unregister(h_out);
    if (rc && !g_errbuf[0]) hs_seterr("hsfft_exec_batched_host: %s", hsd_errstr());
    return rc < 0 ? rc : (rc ? HSFFT_ERR_DEVICE : 0);
}

int hsfft_fill_complex(fft_data *d_x, int64_t count, uint64_t seed, uint64_t offset)
{
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    rc = hsd_fill_complex(d_x, count, seed, offset) ? HSFFT_ERR_DEVICE : 0;
    hs_unlock_device(d);
    return rc;
}

int hsfft_fill_real(fft_type *d_x, int64_t count, uint64_t seed, uint64_t offset)
{
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    rc = hsd_fill_real(d_x, count, seed, offset) ? HSFFT_ERR_DEVICE : 0;
    hs_unlock_device(d);
    return rc;
}

static int time_locked(fft_object obj, hs_entry *e, const fft_data *d_in, fft_data *d_out, int batch, int iters,
                       float *ms, float *pass_ms, int max_pass);

/* ------------------------------------------------------------------ drop-in latency in C
 * BASELINE config 1 (one N = 1024 fft_exec on host buffers) timed the way the reference is
 * timed -- a C loop of fft_exec calls, no interpreter between calls (bench.py used to time it
 * through ctypes, ~1 us per call of binding overhead; round 6).  Warm-up threads run first and
 * exit (their per-thread sets are parked), then `nthreads` fresh threads (which adopt them)
 * start together on a barrier and each make `iters` calls on the shared plan with their own
 * copy of the input. */
/* the timed threads' common start: go 0 wait, 1 run, 2 abandon (a thread could not be created) */
typedef struct {
    pthread_mutex_t mtx;
    pthread_cond_t cv;
    int go;
} hs_tx_start;

typedef struct {
    fft_object obj;
    const fft_data *in;
    fft_data *out;
    int iters, dev;
    double *lat; /* thread 0: per-call microseconds */
    hs_tx_start *start;
} hs_tx_arg;

static double hs_now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void *hs_tx_worker(void *p)
{
    hs_tx_arg *a = (hs_tx_arg *)p;
    const size_t bytes = sizeof(fft_data) * (size_t)a->obj->N;
    fft_data *x = (fft_data *)malloc(bytes), *y = (fft_data *)malloc(bytes);
    if (x) memcpy(x, a->in, bytes);
    int go = 1;
    if (a->start) {
        pthread_mutex_lock(&a->start->mtx);
        while (a->start->go == 0) pthread_cond_wait(&a->start->cv, &a->start->mtx);
        go = a->start->go;
        pthread_mutex_unlock(&a->start->mtx);
    }
    if (x && y && go == 1) {
        (void)hsd_set_device(a->dev);
        for (int i = 0; i < a->iters; i++) {
            const double t0 = a->lat ? hs_now_us() : 0.0;
            fft_exec(a->obj, x, y);
            if (a->lat) a->lat[i] = hs_now_us() - t0;
        }
        if (a->out) memcpy(a->out, y, bytes);
    }
    free(x);
    free(y);
    return NULL;
}

static int hs_cmp_double(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int hsfft_time_exec_host(fft_object obj, const fft_data *in, fft_data *out, int nthreads, int iters, int warmup,
                         double *us)
{
    g_errbuf[0] = 0;
    if (!obj || !in || !out || !us || nthreads < 1 || nthreads > 64 || iters < 1 || warmup < 0) {
        hs_seterr("hsfft_time_exec_host: invalid arguments");
        return HSFFT_ERR_ARG;
    }
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int dev = hsd_get_device();
    pthread_t th[64];
    hs_tx_arg args[64];
    if (warmup > 0) { /* warm-up threads: plan state built, per-thread sets created, then parked */
        int nw = 0;
        for (int t = 0; t < nthreads; t++, nw++) {
            args[t] = (hs_tx_arg){obj, in, NULL, warmup, dev, NULL, NULL};
            if (pthread_create(&th[t], NULL, hs_tx_worker, &args[t])) break;
        }
        for (int t = 0; t < nw; t++) pthread_join(th[t], NULL); /* (they use args: joined before any return) */
        if (nw < nthreads) {
            hs_seterr("hsfft_time_exec_host: thread creation failed");
            return HSFFT_ERR_NOMEM;
        }
    }
    double *lat = (double *)malloc(sizeof(double) * (size_t)iters);
    if (!lat) return HSFFT_ERR_NOMEM;
    hs_tx_start st = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0};
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        args[t] = (hs_tx_arg){obj, in, t == 0 ? out : NULL, iters, dev, t == 0 ? lat : NULL, &st};
        if (pthread_create(&th[t], NULL, hs_tx_worker, &args[t])) break;
        started++;
    }
    /* every thread is created (and has copied nothing yet): start them together, or abandon */
    pthread_mutex_lock(&st.mtx);
    st.go = started == nthreads ? 1 : 2;
    pthread_cond_broadcast(&st.cv);
    pthread_mutex_unlock(&st.mtx);
    const double t0 = hs_now_us();
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    const double wall = hs_now_us() - t0;
    pthread_cond_destroy(&st.cv);
    pthread_mutex_destroy(&st.mtx);
    if (started < nthreads) {
        free(lat);
        hs_seterr("hsfft_time_exec_host: thread creation failed");
        return HSFFT_ERR_NOMEM;
    }
    qsort(lat, (size_t)iters, sizeof(double), hs_cmp_double);
    us[0] = lat[iters / 2];
    us[1] = lat[iters / 10];
    us[2] = lat[(size_t)iters * 9 / 10];
    us[3] = wall / ((double)nthreads * iters);
    free(lat);
    return 0;
}

int hsfft_time_batched(fft_object obj, const fft_data *d_in, fft_data *d_out, int batch, int iters, float *ms,
                       float *pass_ms, int max_pass)
{
    if (!obj || iters < 1 || !ms) return HSFFT_ERR_ARG;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    hs_entry *e = hs_entry_get(obj);
    rc = e ? time_locked(obj, e, d_in, d_out, batch, iters, ms, pass_ms, max_pass) : HSFFT_ERR_ARG;
    hs_entry_put(e);
    hs_unlock_device(d);
    return rc;
}

static int time_locked(fft_object obj, hs_entry *e, const fft_data *d_in, fft_data *d_out, int batch, int iters,
                       float *ms, float *pass_ms, int max_pass)
{
    int rc;
    if (hsd_timer_start()) return HSFFT_ERR_DEVICE;
    for (int it = 0; it < iters; it++) {
        rc = hs_c2c_rows(e, d_in, obj->N, d_out, obj->N, batch);
        if (rc) return rc;
    }
    if (hsd_timer_stop(ms)) return HSFFT_ERR_DEVICE;
    if (pass_ms && max_pass > 0 && e->lt == 0 && e->npass > 0) {
        /* one instrumented iteration: events around every pass launch of a 2-pass in-place
         * chain (the chain's own launch order), so per-kernel averages can be reported */
        hs_devstate *ds = devstate(e);
        const int n = e->npass < max_pass ? e->npass : max_pass;
        if (e->npass <= 2 && ds) {
            for (int i = 0; i < e->npass; i++) {
                const void *R = i == 0 ? (const void *)d_in : (const void *)d_out;
                if (i < n) hsd_pass_timer_begin(i);
                rc = launch_pass(e, ds, i, R, obj->N, d_out, obj->N, batch, e->sgn, 0, e->sgn, HS_LOAD_PLAIN, NULL,
                                 HS_STORE_PLAIN, NULL, e->M);
                if (i < n) hsd_pass_timer_end(i);
                if (rc) return rc;
            }
            hsd_pass_timer_read(n, pass_ms);
        } else {
            for (int i = 0; i < n; i++) pass_ms[i] = -1.0f;
        }
    }
    return 0;
}

int hsfft_bench_copy(const void *d_src, void *d_dst, size_t bytes, int iters, float *ms)
{
    if (!d_src || !d_dst || !ms || iters < 1 || bytes % 16) return HSFFT_ERR_ARG;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    rc = hsd_copy_bench(d_src, d_dst, (long long)(bytes / 16), iters, ms) ? HSFFT_ERR_DEVICE : 0;
    hs_unlock_device(d);
    return rc;
}

int hsfft_count_diff_words(const void *d_a, const void *d_b, size_t bytes, uint64_t *count)
{
    if (!d_a || !d_b || !count || bytes % 8) return HSFFT_ERR_ARG;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    unsigned long long c = 0;
    rc = hsd_count_diff(d_a, d_b, (long long)(bytes / 8), &c) ? HSFFT_ERR_DEVICE : 0;
    hs_unlock_device(d);
    *count = c;
    return rc;
}

/* one host thread per device: each selects its device, enqueues its contiguous shard and
 * waits for it; no data crosses devices.  Per-device state (twiddles, Bluestein hk) is built
 * by that device's thread, so first use builds all devices' state concurrently. */
typedef struct {
    fft_object obj;
    const fft_data *in;
    fft_data *out;
    int dev, rows, rc;
    char err[512];
} hs_shard;

static void *shard_main(void *arg)
{
    hs_shard *s = arg;
    s->rc = hsd_set_device(s->dev) ? HSFFT_ERR_DEVICE : 0;
    t_sync_call++; /* the shard waits anyway: Bluestein rows of a timed-out launch are re-run */
    if (!s->rc && s->rows > 0) s->rc = hsfft_exec_batched(s->obj, s->in, s->out, s->rows);
    if (!s->rc && hsd_sync_report()) s->rc = HSFFT_ERR_DEVICE;
    t_sync_call--;
    if (s->rc) snprintf(s->err, sizeof s->err, "device %d: %.400s", s->dev, g_errbuf[0] ? g_errbuf : hsd_errstr());
    return NULL;
}

int hsfft_exec_multi(fft_object obj, const fft_data *const *d_in, fft_data *const *d_out, int batch, int ndev)
{
    g_errbuf[0] = 0;
    if (!obj || !d_in || !d_out || ndev < 1 || batch < 0 || ndev > HS_MAX_DEV) return HSFFT_ERR_ARG;
    int rc = hs_require_gpu();
    if (rc) return rc;
    if (ndev > hsd_device_count()) return HSFFT_ERR_ARG;
    const int cur = hsd_get_device();
    hs_shard sh[HS_MAX_DEV];
    pthread_t th[HS_MAX_DEV];
    int started[HS_MAX_DEV] = {0};
    for (int g = 0; g < ndev; g++) {
        const int b0 = (int)((long long)batch * g / ndev), b1 = (int)((long long)batch * (g + 1) / ndev);
        memset(&sh[g], 0, sizeof sh[g]);
        sh[g].obj = obj;
        sh[g].in = d_in[g];
        sh[g].out = d_out[g];
        sh[g].dev = g;
        sh[g].rows = b1 - b0;
        started[g] = pthread_create(&th[g], NULL, shard_main, &sh[g]) == 0;
        if (!started[g]) shard_main(&sh[g]); /* no thread: run the shard here */
    }
    for (int g = 0; g < ndev; g++) {
        if (started[g]) pthread_join(th[g], NULL);
        if (sh[g].rc && !rc) {
            rc = sh[g].rc;
            hs_seterr("hsfft_exec_multi: %s", sh[g].err);
        }
    }
    if (cur >= 0) hsd_set_device(cur);
    return rc;
}
