/*
 * hsfft_convolve.c -- FFT convolution entry points of libhsfft.so (host C; compute on GPU).
 *   next_power_of_two        ref src/convolve.c:20-25
 *   find_optimal_fft_length  ref src/convolve.c:39-56
 *   fft_convolve             ref src/convolve.c:74-214 (r2c x2, spectral product, c2r,
 *                            scale by 1/P, slice by output type)
 * The reference builds two real plans per call; here plans are cached per padded length
 * (their contents are identical for the same length and sign).
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsfft_gpu.h"
#include "hsfft_host.h"

int next_power_of_two(int n)
{
    if (n <= 0) return 1;
    return (int)pow(2, ceil(log2(n)));
}

int find_optimal_fft_length(int min_length, const char *conv_type, int length1, int length2)
{
    if (conv_type && strcmp(conv_type, "linear") == 0) return next_power_of_two(min_length);
    if (conv_type && strcmp(conv_type, "circular") == 0)
        return next_power_of_two(length1 > length2 ? length1 : length2);
    fprintf(stderr, "Error: Invalid convolution type\n");
    exit(EXIT_FAILURE);
}

/* Plan cache: entries are reference counted -- a slot in use by any thread is never
 * evicted; when every slot is busy the call builds a private pair and frees it afterwards.
 * A slot being built carries its P and mode with `building` set: a concurrent request for the
 * same length waits for that build instead of evicting another slot for a duplicate pair. */
#define HS_CONV_CACHE 8
static pthread_mutex_t g_clock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_cbuilt = PTHREAD_COND_INITIALIZER;
static struct {
    int P, mode, refs, building;
    unsigned long long used; /* LRU stamp */
    fft_real_object f, i;
} g_cache[HS_CONV_CACHE];
static unsigned long long g_cache_clock;

typedef struct {
    fft_real_object f, i;
    int slot; /* cache slot held, or -1 for a private pair */
} conv_pair;

static conv_pair conv_plans(int P)
{
    const int mode = hsfft_get_twiddle_mode();
    conv_pair cp = {NULL, NULL, -1};
    pthread_mutex_lock(&g_clock);
    for (;;) {
        int victim = -1, pending = 0;
        for (int k = 0; k < HS_CONV_CACHE; k++) {
            const int same = g_cache[k].P == P && g_cache[k].mode == mode;
            if (same && g_cache[k].building) {
                pending = 1;
                break;
            }
            if (same && g_cache[k].f) {
                g_cache[k].refs++;
                g_cache[k].used = ++g_cache_clock;
                cp.f = g_cache[k].f;
                cp.i = g_cache[k].i;
                cp.slot = k;
                pthread_mutex_unlock(&g_clock);
                return cp;
            }
            if (g_cache[k].refs == 0 && !g_cache[k].building &&
                (victim < 0 || !g_cache[k].f || (g_cache[victim].f && g_cache[k].used < g_cache[victim].used)))
                victim = k;
        }
        if (pending) { /* another thread is building this length: wait, then look again */
            pthread_cond_wait(&g_cbuilt, &g_clock);
            continue;
        }
        if (victim < 0) break;
        /* reserve the least recently used idle slot; build and free outside the lock (plans
         * of other lengths / devices are not held up) */
        fft_real_object of = g_cache[victim].f, oi = g_cache[victim].i;
        g_cache[victim].P = P;
        g_cache[victim].mode = mode;
        g_cache[victim].refs = 1;
        g_cache[victim].building = 1;
        g_cache[victim].used = ++g_cache_clock;
        g_cache[victim].f = g_cache[victim].i = NULL;
        pthread_mutex_unlock(&g_clock);
        if (of) {
            free_real_fft(of);
            free_real_fft(oi);
        }
        cp.f = fft_real_init(P, 1);
        cp.i = fft_real_init(P, -1);
        cp.slot = victim;
        pthread_mutex_lock(&g_clock);
        g_cache[victim].building = 0;
        if (cp.f && cp.i) {
            g_cache[victim].f = cp.f;
            g_cache[victim].i = cp.i;
        } else { /* failed build: the slot goes back empty, the caller keeps what it got */
            g_cache[victim].P = 0;
            g_cache[victim].refs = 0;
            cp.slot = -1;
        }
        pthread_cond_broadcast(&g_cbuilt);
        pthread_mutex_unlock(&g_clock);
        return cp;
    }
    pthread_mutex_unlock(&g_clock);
    cp.f = fft_real_init(P, 1);
    cp.i = fft_real_init(P, -1);
    return cp;
}

static void conv_plans_done(conv_pair cp)
{
    if (cp.slot < 0) {
        free_real_fft(cp.f);
        free_real_fft(cp.i);
        return;
    }
    pthread_mutex_lock(&g_clock);
    g_cache[cp.slot].refs--;
    pthread_mutex_unlock(&g_clock);
}

/* (hsfft_finalize) free every idle cached plan pair; slots in use or being built are kept */
void hs_conv_cache_release(void)
{
    fft_real_object fr[2 * HS_CONV_CACHE];
    int n = 0;
    pthread_mutex_lock(&g_clock);
    for (int k = 0; k < HS_CONV_CACHE; k++)
        if (g_cache[k].refs == 0 && !g_cache[k].building && g_cache[k].f) {
            fr[n++] = g_cache[k].f;
            fr[n++] = g_cache[k].i;
            g_cache[k].f = g_cache[k].i = NULL;
            g_cache[k].P = 0;
        }
    pthread_mutex_unlock(&g_clock);
    for (int k = 0; k < n; k++) free_real_fft(fr[k]);
}

/* output window of the reference (convolve.c:163-201); returns length or -1 */
static int conv_window(const char *type, int linear, int clen, int P, int n, int m, int *start)
{
    *start = 0;
    if (!linear) return P;
    if (type == NULL || strcmp(type, "full") == 0) return clen; /* NULL: the reference crashes (D9) */
    if (strcmp(type, "same") == 0) {
        const int big = n > m ? n : m;
        *start = (clen - big) / 2;
        return big;
    }
    if (strcmp(type, "valid") == 0) {
        const int sm = n < m ? n : m, big = n > m ? n : m;
        *start = sm - 1;
        return big - sm + 1;
    }
    fprintf(stderr, "Error: Invalid output type. Use 'full', 'same', or 'valid'.\n");
    return -1;
}

static int conv_setup(const char *conv_type, int n, int m, int *linear, int *clen, int *P)
{
    if (conv_type == NULL) return -1;
    if (strcmp(conv_type, "linear") == 0) {
        *linear = 1;
        *clen = n + m - 1;
    } else if (strcmp(conv_type, "circular") == 0) {
        *linear = 0;
        *clen = n > m ? n : m;
    } else {
        fprintf(stderr, "Error: Invalid convolution type. Use 'linear' or 'circular'.\n");
        return -1;
    }
    *P = find_optimal_fft_length(*clen, conv_type, n, m);
    return 0;
}

/* device core: a (rows of n), b (rows of m) -> res (rows of P; divided by P if scale) */
static int conv_device(int P, const double *d_a, int n, const double *d_b, int m, double *d_res, int batch, int scale)
{
    const conv_pair cp = conv_plans(P);
    fft_real_object f = cp.f, iv = cp.i;
    /* the reference multiplies all P mirrored bins (convolve.c:147-151), but its c2r reads
     * bins 0..P/2 only (real.c:169-179): compact spectra of P/2+1 bins give the same bits
     * with a third less traffic */
    const long long cd = P / 2 + 1;
    double *pa = hs_scratch(7, sizeof(double) * (size_t)P * 2 * (size_t)batch);
    fft_data *spec = hs_scratch(10, sizeof(fft_data) * (size_t)cd * 2 * (size_t)batch);
    if (!pa || !spec) {
        conv_plans_done(cp);
        hs_seterr("convolution scratch allocation failed (%d rows of P = %d)", batch, P);
        return HSFFT_ERR_NOMEM;
    }
    double *pb = pa + (size_t)P * batch;
    fft_data *A = spec, *B = spec + (size_t)cd * batch;
    int rc = hsd_copy_rows(d_a, n, 0, n, pa, P, P, batch) || hsd_copy_rows(d_b, m, 0, m, pb, P, P, batch)
                 ? HSFFT_ERR_DEVICE : 0;
    if (!rc) rc = hsfft_r2c_batched_compact(f, pa, A, batch);
    if (!rc) rc = hsfft_r2c_batched_compact(f, pb, B, batch);
    if (!rc) rc = hs_c2r_product_rows(iv, A, B, cd, d_res, batch); /* product fused into the pre-twiddle */
    if (!rc && scale) rc = hsd_scale_real(d_res, P, batch, P, (double)P) ? HSFFT_ERR_DEVICE : 0;
    if (!rc) rc = hsd_sync() ? HSFFT_ERR_DEVICE : 0;
    conv_plans_done(cp);
    return rc;
}

static int convolve_locked(const char *type, const char *conv_type, fft_type *input1, int length1,
                           fft_type *input2, int length2, fft_type *output)
{
    if (input1 == NULL || input2 == NULL || output == NULL || length1 <= 0 || length2 <= 0) {
        fprintf(stderr, "Error: Invalid inputs for fft_convolve\n");
        return -1;
    }
    int linear, clen, P, start;
    if (conv_setup(conv_type, length1, length2, &linear, &clen, &P)) return -1;
    if (hs_require_gpu()) {
        fprintf(stderr, "Error: fft_convolve needs an MI355X (%s)\n", hsfft_last_error());
        exit(EXIT_FAILURE);
    }
    const int len = conv_window(type, linear, clen, P, length1, length2, &start);
    double *d_a = hs_scratch(5, sizeof(double) * (size_t)(length1 + length2));
    double *d_res = hsfft_malloc(sizeof(double) * (size_t)P);
    if (!d_a || !d_res) {
        hsfft_free(d_res);
        return -1;
    }
    double *d_b = d_a + length1;
    int rc = hsd_h2d(d_a, input1, sizeof(double) * (size_t)length1) || hsd_h2d(d_b, input2, sizeof(double) * (size_t)length2);
    if (!rc) rc = conv_device(P, d_a, length1, d_b, length2, d_res, 1, 1);
    if (!rc && len > 0) rc = hsd_d2h(output, d_res + start, sizeof(double) * (size_t)len);
    hsfft_free(d_res);
    if (rc) {
        fprintf(stderr, "Error: fft_convolve failed (%s)\n", hsfft_last_error());
        return -1;
    }
    return len;
}

int fft_convolve(const char *type, const char *conv_type, fft_type *input1, int length1, fft_type *input2,
                 int length2, fft_type *output)
{
    const int d = hs_lock_device();
    const int rc = convolve_locked(type, conv_type, input1, length1, input2, length2, output);
    hs_unlock_device(d);
    return rc;
}

int hsfft_convolve_batched(const char *type, const char *conv_type, const fft_type *d_a, int length1,
                           const fft_type *d_b, int length2, fft_type *d_out, int batch)
{
    if (!d_a || !d_b || !d_out || length1 <= 0 || length2 <= 0 || batch < 0) return HSFFT_ERR_ARG;
    int linear, clen, P, start;
    if (conv_setup(conv_type, length1, length2, &linear, &clen, &P)) return HSFFT_ERR_ARG;
    if (P < 2) { /* both lengths 1: the reference's real plan of length 1 exits (real.c:26-31) */
        hs_seterr("convolution of two length-1 signals: transform length %d is not even", P);
        return HSFFT_ERR_ARG;
    }
    const int len = conv_window(type, linear, clen, P, length1, length2, &start);
    if (len < 0) return HSFFT_ERR_ARG;
    if (batch == 0) return len;
    int rc = hs_require_gpu();
    if (rc) return rc;
    const int d = hs_lock_device();
    double *d_res = hsfft_malloc(sizeof(double) * (size_t)P * (size_t)batch);
    if (!d_res) {
        hs_unlock_device(d);
        return HSFFT_ERR_NOMEM;
    }
    rc = conv_device(P, d_a, length1, d_b, length2, d_res, batch, 0);
    /* the 1/P scale (convolve.c:157-160) fused into the window copy: same division per element */
    if (!rc && len > 0)
        rc = hsd_copy_rows_div(d_res, P, start, d_out, len, len, batch, (double)P) ? HSFFT_ERR_DEVICE : 0;
    if (!rc) rc = hsd_sync() ? HSFFT_ERR_DEVICE : 0;
    hsfft_free(d_res);
    hs_unlock_device(d);
    return rc ? rc : len;
}
