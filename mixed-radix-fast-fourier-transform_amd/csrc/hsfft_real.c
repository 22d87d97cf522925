/*
 * hsfft_real.c -- real-signal transforms of libhsfft.so (host C; compute on the GPU).
 *   fft_real_init  ref src/real.c:26-64    (inner N/2 complex plan + twiddle2)
 *   fft_r2c_exec   ref src/real.c:78-136   (pack = reinterpretation, c2c, split, mirror)
 *   fft_c2r_exec   ref src/real.c:150-193  (pre-twiddle, c2c, unpack = reinterpretation)
 *   free_real_fft  ref src/real.c:259-267  (also releases device state of both objects)
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsfft_gpu.h"
#include "hsfft_host.h"

typedef struct hs_real_entry {
    const struct fft_real_set *key;
    void *d_tw2[HS_MAX_DEV];
    struct hs_real_entry *next;
} hs_real_entry;

static pthread_mutex_t g_rlock = PTHREAD_MUTEX_INITIALIZER;
static hs_real_entry *g_real;

fft_real_object fft_real_init(int N, int sgn)
{
    if (N <= 0 || N % 2 != 0) {
        fprintf(stderr, "Error: Signal length (%d) must be positive and even\n", N);
        exit(EXIT_FAILURE);
    }
    const int h = N / 2;
    fft_real_object r = (fft_real_object)malloc(sizeof(struct fft_real_set) + sizeof(fft_data) * (size_t)h);
    if (r == NULL) {
        fprintf(stderr, "Error: Memory allocation failed for real FFT object\n");
        exit(EXIT_FAILURE);
    }
    r->cobj = fft_init(h, sgn);
    if (r->cobj == NULL) {
        free(r);
        fprintf(stderr, "Error: Failed to initialize complex FFT object\n");
        exit(EXIT_FAILURE);
    }
    for (int k = 0; k < h; k++) {
        double sn, cs;
        sincos(PI2 * k / N, &sn, &cs);
        r->twiddle2[k].re = cs;
        r->twiddle2[k].im = sn;
    }
    return r;
}

static void *tw2_device(fft_real_object r)
{
    const int d = hsd_get_device();
    if (d < 0 || d >= HS_MAX_DEV) return NULL;
    pthread_mutex_lock(&g_rlock);
    hs_real_entry *e = g_real;
    while (e && e->key != r) e = e->next;
    if (!e) {
        e = calloc(1, sizeof *e);
        e->key = r;
        e->next = g_real;
        g_real = e;
    }
    if (!e->d_tw2[d]) {
        const size_t b = sizeof(fft_data) * (size_t)r->cobj->N;
        e->d_tw2[d] = hsd_malloc(b);
        if (e->d_tw2[d] && hsd_h2d(e->d_tw2[d], r->twiddle2, b)) {
            hsd_free(e->d_tw2[d]);
            e->d_tw2[d] = NULL;
        }
    }
    void *p = e->d_tw2[d];
    pthread_mutex_unlock(&g_rlock);
    return p;
}

void free_real_fft(fft_real_object r)
{
    if (r == NULL) return;
    pthread_mutex_lock(&g_rlock);
    for (hs_real_entry **pp = &g_real; *pp; pp = &(*pp)->next)
        if ((*pp)->key == r) {
            hs_real_entry *e = *pp;
            *pp = e->next;
            const int cur = hsd_get_device();
            for (int d = 0; d < HS_MAX_DEV; d++)
                if (e->d_tw2[d]) {
                    hsd_set_device(d);
                    hsd_free(e->d_tw2[d]);
                }
            if (cur >= 0) hsd_set_device(cur);
            free(e);
            break;
        }
    pthread_mutex_unlock(&g_rlock);
    free_fft(r->cobj);
    free(r);
}

/* (hsfft_finalize) drop every real plan's device twiddles on device `dev` (rebuilt on demand) */
void hs_real_release_device(int dev)
{
    pthread_mutex_lock(&g_rlock);
    for (hs_real_entry *e = g_real; e; e = e->next)
        if (e->d_tw2[dev]) {
            hsd_free(e->d_tw2[dev]);
            e->d_tw2[dev] = NULL;
        }
    pthread_mutex_unlock(&g_rlock);
}

/* row chunk for the inner c2c's intermediate Z (scratch class 4): HSFFT_CHUNK_MB of Z per
 * chunk, default 16 GiB (measured, 4096 x 2^22 r2c, fused split: 2 GiB 91.7, 4 GiB 94.1,
 * 8 GiB 98.3, 16 GiB 99.9 GSamples/s -- longer launches fill the chip better); halved while
 * the allocation fails, so a device with less free HBM still runs, in smaller chunks */
static fft_data *real_chunk(int h, int batch, long long *chunk)
{
    const size_t bytes = hs_env_mb("HSFFT_REAL_CHUNK_MB", 16384.0);
    long long rows = (long long)(bytes / (sizeof(fft_data) * (size_t)h));
    if (rows < 1) rows = 1;
    if (rows > batch) rows = batch;
    for (;;) {
        fft_data *Z = hs_scratch(4, sizeof(fft_data) * (size_t)(rows * h));
        if (Z || rows == 1) {
            *chunk = rows;
            if (!Z) hs_seterr("scratch allocation of %lld bytes failed", (long long)(rows * h * 16));
            return Z;
        }
        rows = (rows + 1) / 2;
    }
}

static int r2c_locked(fft_real_object r, hs_entry *e, const fft_type *d_in, fft_data *d_out, int batch);

int hsfft_r2c_batched(fft_real_object r, const fft_type *d_in, fft_data *d_out, int batch)
{
    if (!r || !r->cobj || !d_in || !d_out || batch < 0) {
        hs_seterr("hsfft_r2c_batched: invalid arguments");
        return HSFFT_ERR_ARG;
    }
    if (batch == 0) return 0;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    hs_entry *e = hs_entry_get(r->cobj);
    rc = e ? r2c_locked(r, e, d_in, d_out, batch) : HSFFT_ERR_DEVICE;
    hs_entry_put(e);
    hs_unlock_device(d);
    return rc;
}

static int r2c_locked(fft_real_object r, hs_entry *e, const fft_type *d_in, fft_data *d_out, int batch)
{
    int rc = 0;
    void *tw2 = tw2_device(r);
    if (!tw2) return HSFFT_ERR_DEVICE;
    const int h = r->cobj->N, N = 2 * h;
    long long chunk;
    fft_data *Z = real_chunk(h, batch, &chunk);
    if (!Z) return HSFFT_ERR_NOMEM;
    for (long long c0 = 0; c0 < batch; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        /* x[2k], x[2k+1] packed as complex = the same bytes (ref real.c:99-103) */
        rc = hs_r2c_fused(e, d_in + c0 * N, h, Z, d_out + c0 * N, N, tw2, cb, 0);
        if (rc == 1) {
            rc = hs_c2c_rows(e, d_in + c0 * N, h, Z, h, cb);
            if (!rc) rc = hsd_r2c_post(Z, tw2, d_out + c0 * N, h, cb, h, N) ? HSFFT_ERR_DEVICE : 0;
        }
        if (rc) return rc;
    }
    return 0;
}

/* compact r2c: bins 0..N/2 per row (rows of N/2+1 complex), the
 * non-redundant half of the reference's mirrored output -- 16 B written per real sample
 * instead of 24 for the same values (bit-identical to bins 0..N/2 of hsfft_r2c_batched) */
static int r2c_compact_locked(fft_real_object r, hs_entry *e, const fft_type *d_in, fft_data *d_out, int batch);

int hsfft_r2c_batched_compact(fft_real_object r, const fft_type *d_in, fft_data *d_out, int batch)
{
    if (!r || !r->cobj || !d_in || !d_out || batch < 0) {
        hs_seterr("hsfft_r2c_batched_compact: invalid arguments");
        return HSFFT_ERR_ARG;
    }
    if (batch == 0) return 0;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    hs_entry *e = hs_entry_get(r->cobj);
    rc = e ? r2c_compact_locked(r, e, d_in, d_out, batch) : HSFFT_ERR_DEVICE;
    hs_entry_put(e);
    hs_unlock_device(d);
    return rc;
}

static int r2c_compact_locked(fft_real_object r, hs_entry *e, const fft_type *d_in, fft_data *d_out, int batch)
{
    int rc = 0;
    void *tw2 = tw2_device(r);
    if (!tw2) return HSFFT_ERR_DEVICE;
    const int h = r->cobj->N, N = 2 * h;
    long long chunk;
    fft_data *Z = real_chunk(h, batch, &chunk);
    if (!Z) return HSFFT_ERR_NOMEM;
    for (long long c0 = 0; c0 < batch && !rc; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        rc = hs_r2c_fused(e, d_in + c0 * N, h, Z, d_out + c0 * (h + 1), h + 1, tw2, cb, 1);
        if (rc == 1) {
            rc = hs_c2c_rows(e, d_in + c0 * N, h, Z, h, cb);
            if (!rc)
                rc = hsd_r2c_post_compact(Z, tw2, d_out + c0 * (h + 1), h, cb, h, h + 1) ? HSFFT_ERR_DEVICE : 0;
        }
    }
    return rc;
}

int hsfft_c2r_batched(fft_real_object r, const fft_data *d_in, fft_type *d_out, int batch)
{
    if (!r || !r->cobj || !d_in || !d_out || batch < 0) {
        hs_seterr("hsfft_c2r_batched: invalid arguments");
        return HSFFT_ERR_ARG;
    }
    if (batch == 0) return 0;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    rc = hs_c2r_rows(r, d_in, 2LL * r->cobj->N, d_out, batch);
    hs_unlock_device(d);
    return rc;
}

/* (callers hold the device lock) */
int hs_c2r_product_rows(fft_real_object r, const fft_data *d_a, const fft_data *d_b, long long xdist, fft_type *d_out,
                        int batch)
{
    int rc = 0;
    hs_entry *e = hs_entry_get(r->cobj);
    void *tw2 = e ? tw2_device(r) : NULL;
    const int h = r->cobj->N, N = 2 * h;
    long long chunk = 1;
    fft_data *Zi = tw2 ? real_chunk(h, batch, &chunk) : NULL;
    if (!tw2) rc = HSFFT_ERR_DEVICE;
    else if (!Zi) rc = HSFFT_ERR_NOMEM;
    for (long long c0 = 0; c0 < batch && !rc; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        rc = hsd_c2r_pre_mul(d_a + c0 * xdist, d_b + c0 * xdist, tw2, Zi, h, cb, xdist, h) ? HSFFT_ERR_DEVICE : 0;
        if (!rc) rc = hs_c2c_rows(e, Zi, h, d_out + c0 * N, h, cb);
    }
    hs_entry_put(e);
    return rc;
}

/* c2r of rows xdist complex apart (the reference layout: N; compact spectra: N/2+1 -- the
 * pre-twiddle reads bins 0..N/2 only, ref real.c:169-179) */
int hs_c2r_rows(fft_real_object r, const fft_data *d_in, long long xdist, fft_type *d_out, int batch)
{
    int rc = 0;
    hs_entry *e = hs_entry_get(r->cobj);
    void *tw2 = e ? tw2_device(r) : NULL;
    const int h = r->cobj->N, N = 2 * h;
    long long chunk = 1;
    fft_data *Zi = tw2 ? real_chunk(h, batch, &chunk) : NULL;
    if (!tw2) rc = HSFFT_ERR_DEVICE;
    else if (!Zi) rc = HSFFT_ERR_NOMEM;
    for (long long c0 = 0; c0 < batch && !rc; c0 += chunk) {
        const int cb = (int)(batch - c0 < chunk ? batch - c0 : chunk);
        rc = hsd_c2r_pre(d_in + c0 * xdist, tw2, Zi, h, cb, xdist, h) ? HSFFT_ERR_DEVICE : 0;
        /* unpacking complex_output into interleaved reals is again a reinterpretation */
        if (!rc) rc = hs_c2c_rows(e, Zi, h, d_out + c0 * N, h, cb);
    }
    hs_entry_put(e);
    return rc;
}

int hsfft_time_r2c_batched(fft_real_object r, const fft_type *d_in, fft_data *d_out, int batch, int iters, float *ms)
{
    if (!r || iters < 1 || !ms) return HSFFT_ERR_ARG;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    rc = hsfft_r2c_batched(r, d_in, d_out, batch); /* device state outside the timing */
    if (!rc && hsd_timer_start()) rc = HSFFT_ERR_DEVICE;
    for (int i = 0; i < iters && !rc; i++) rc = hsfft_r2c_batched(r, d_in, d_out, batch);
    if (!rc && hsd_timer_stop(ms)) rc = HSFFT_ERR_DEVICE;
    hs_unlock_device(d);
    return rc;
}

static void real_fail(const char *what)
{
    fprintf(stderr, "Error: %s (%s)\n", what, hsfft_last_error());
    exit(EXIT_FAILURE);
}

static void r2c_exec_locked(fft_real_object r, fft_type *inp, fft_data *oup)
{
    if (r == NULL || inp == NULL || oup == NULL) {
        fprintf(stderr, "Error: Invalid real FFT object or data pointers\n");
        exit(EXIT_FAILURE);
    }
    if (hs_require_gpu()) real_fail("fft_r2c_exec needs an MI355X");
    const int N = 2 * r->cobj->N;
    const int din = hsd_is_device_ptr(inp), dout = hsd_is_device_ptr(oup);
    int rc;
    if (din && dout) {
        rc = hsfft_r2c_batched(r, inp, oup, 1);
    } else {
        double *di = hs_scratch(5, sizeof(double) * (size_t)N);
        fft_data *dq = hs_scratch(6, sizeof(fft_data) * (size_t)N);
        if (!di || !dq) real_fail("fft_r2c_exec: staging allocation failed");
        rc = din ? hsd_d2d_async(di, inp, sizeof(double) * (size_t)N) : hsd_h2d(di, inp, sizeof(double) * (size_t)N);
        if (!rc) rc = hsfft_r2c_batched(r, di, dq, 1);
        if (!rc) rc = dout ? hsd_d2d_async(oup, dq, sizeof(fft_data) * (size_t)N) : hsd_d2h(oup, dq, sizeof(fft_data) * (size_t)N);
    }
    if (!rc) rc = hsd_sync();
    if (rc) real_fail("fft_r2c_exec failed");
}

void fft_r2c_exec(fft_real_object r, fft_type *inp, fft_data *oup)
{
    const int d = hs_lock_device();
    hs_sync_call(1); /* synchronous: a Bluestein inner plan re-runs timed-out rows itself */
    r2c_exec_locked(r, inp, oup);
    hs_sync_call(0);
    hs_unlock_device(d);
}

static void c2r_exec_locked(fft_real_object r, fft_data *inp, fft_type *oup)
{
    if (r == NULL || inp == NULL || oup == NULL) {
        fprintf(stderr, "Error: Invalid real FFT object or data pointers\n");
        exit(EXIT_FAILURE);
    }
    if (hs_require_gpu()) real_fail("fft_c2r_exec needs an MI355X");
    const int h = r->cobj->N, N = 2 * h;
    const int din = hsd_is_device_ptr(inp), dout = hsd_is_device_ptr(oup);
    int rc;
    if (din && dout) {
        rc = hsfft_c2r_batched(r, inp, oup, 1);
    } else {
        /* only bins 0..N/2 are read (real.c:169-179); the staging row is N long */
        fft_data *di = hs_scratch(5, sizeof(fft_data) * (size_t)N);
        double *dq = hs_scratch(6, sizeof(double) * (size_t)N);
        if (!di || !dq) real_fail("fft_c2r_exec: staging allocation failed");
        rc = din ? hsd_d2d_async(di, inp, sizeof(fft_data) * (size_t)(h + 1))
                 : hsd_h2d(di, inp, sizeof(fft_data) * (size_t)(h + 1));
        if (!rc) rc = hsfft_c2r_batched(r, di, dq, 1);
        if (!rc) rc = dout ? hsd_d2d_async(oup, dq, sizeof(double) * (size_t)N) : hsd_d2h(oup, dq, sizeof(double) * (size_t)N);
    }
    if (!rc) rc = hsd_sync();
    if (rc) real_fail("fft_c2r_exec failed");
}

void fft_c2r_exec(fft_real_object r, fft_data *inp, fft_type *oup)
{
    const int d = hs_lock_device();
    hs_sync_call(1); /* synchronous: a Bluestein inner plan re-runs timed-out rows itself */
    c2r_exec_locked(r, inp, oup);
    hs_sync_call(0);
    hs_unlock_device(d);
}
