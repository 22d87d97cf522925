/*
 * hsfft_host.h -- host-side internals shared by the C translation units of libhsfft.so.
 */
#ifndef HSFFT_HOST_H_
#define HSFFT_HOST_H_

#include "highspeedFFT.h"
#include "hsfft_internal.h"
#include "real.h"

#ifdef __cplusplus
extern "C" {
#endif

/* per-device state of one plan: device copies of what the plan needs */
typedef struct hs_devstate {
    void *d_tw;   /* M-1 (+1) complex twiddles, copied from the public struct; only the
                   * [3,3,5,5,7,8] whole-row schedule (N = 12600) also holds the last stage's block
                   * transposed at d_tw + M, and readers are told so by tw_t below */
    void *d_gcs;  /* odd-radix cos/sin constants */
    void *d_chirp;/* Bluestein chirp h(n), N complex */
    void *d_hk;   /* Bluestein spectrum of the scaled, mirrored chirp, M complex */
    int tw_t;     /* 1: d_tw + M holds the last stage's block transposed (the 12600 row kernel) */
    /* users outside the device lock (the concurrent small fft_exec path) pin the state for
     * their whole call: a rebuild (hsfft_plan_refresh) then retires it instead of freeing it,
     * and the last hs_devstate_put frees it.  Both fields change under the device lock. */
    int refs;
    int retired;
} hs_devstate;

/* schedule derived from the public plan fields (snapshot) */
typedef struct hs_entry {
    const struct fft_set *key;
    int N, sgn, lt, lf, M; /* M = length of the mixed-radix transform actually run */
    int factors[64];       /* snapshot of the public fields (edits trigger a rebuild) */
    int rlf, rfac[64];     /* factor list actually executed (differs only for D5) */
    int tw_from_struct;    /* 1: twiddles copied from the struct; 0: private table (D5) */
    fft_data *tw_private;  /* Bluestein plan/exec length mismatch (D5): own M_exec table */
    int nst;
    int stage_r[HS_MAX_STAGES];  /* innermost first */
    int first_leaf;
    int npass;
    hsd_pass pass[HS_MAX_PASSES];
    double *gcs;           /* host odd-radix constants */
    int ngcs;
    fft_data *chirp;       /* Bluestein chirp (host) */
    hs_devstate *ds[HS_MAX_DEV];
    int version;           /* bumped by hsfft_plan_refresh: device copies re-uploaded */
    int ds_version[HS_MAX_DEV];
    int refs;              /* users holding the entry (hs_entry_get .. hs_entry_put) */
    int dead;              /* unlinked (free_fft or a rebuild): freed by the last put */
    struct hs_entry *next;
} hs_entry;

/* planner (hsfft_plan.c) */
int hs_twiddle_mode(void);
void hs_longvector(fft_data *tw, int M, const int *fac, int lf, int exact);
int hs_bluestein_M_init(int N); /* fft_init sizing (log10), ref :242-252 */
int hs_bluestein_M_exec(int N); /* bluestein_fft sizing (log2), ref :1750-1751 */

/* registry / scheduling / execution (hsfft_exec.c).  hs_entry_get returns the entry with a
 * reference held; every successful get is paired with hs_entry_put. */
hs_entry *hs_entry_get(const struct fft_set *obj);
void hs_entry_put(hs_entry *e);
void hs_entry_release(const struct fft_set *obj);
/* Reentrancy: every public entry point that enqueues work or touches per-device state
 * (scratch pool, staging slots, streams, events, lazily built device state) runs under the
 * recursive lock of the calling thread's current device.  Host threads on different devices
 * run concurrently; threads sharing a device take turns per call. */
int hs_lock_device(void);
void hs_unlock_device(int dev);
int hs_require_gpu(void);
void hs_seterr(const char *fmt, ...);
int hs_c2c_rows(hs_entry *e, const void *in, long long idist, void *out, long long odist, int batch);
/* r2c with the split fused into the last c2c pass: returns 1 when the plan's schedule does
 * not allow it (caller falls back to c2c + split), 0 on success, < 0 on error */
int hs_r2c_fused(hs_entry *e, const void *in, long long idist, void *Z, void *X, long long xdist, const void *tw2,
                 int batch, int compact);
/* scratch buffers per device: class 0..2 chain pool, 3 Bluestein mid, 4 real staging, 5-7 misc,
 * 8 Bluestein second mid, 9 host pipeline, 10 convolution spectra */
int hs_c2r_rows(fft_real_object r, const fft_data *d_in, long long xdist, fft_type *d_out, int batch);
/* c2r of the product d_a .* d_b (compact or reference-layout rows xdist apart) */
int hs_c2r_product_rows(fft_real_object r, const fft_data *d_a, const fft_data *d_b, long long xdist, fft_type *d_out,
                        int batch);
void *hs_scratch(int cls, size_t bytes);
/* brackets a synchronous entry point on this thread (1 enter, 0 leave): persistent Bluestein
 * launches inside it wait and re-run timed-out rows instead of reporting them later */
void hs_sync_call(int enter);
/* release this layer's device objects (hsfft_finalize): idle convolution plan pairs, real
 * plans' device twiddles on the current device */
void hs_conv_cache_release(void);
void hs_real_release_device(int dev);
/* bytes from an environment knob given in MiB (default dflt_mb; at least 1 MiB) */
size_t hs_env_mb(const char *name, double dflt_mb);

#ifdef __cplusplus
}
#endif

#endif
