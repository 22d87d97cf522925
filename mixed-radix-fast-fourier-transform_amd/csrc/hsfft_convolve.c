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

#define HS_CONV_CACHE 8
static pthread_mutex_t g_clock = PTHREAD_MUTEX_INITIALIZER;
static struct {
    int P, mode;
    fft_real_object f, i;
} g_cache[HS_CONV_CACHE];
static int g_cache_next;

static void conv_plans(int P, fft_real_object *f, fft_real_object *i)
{
    const int mode = hsfft_get_twiddle_mode();
    pthread_mutex_lock(&g_clock);
    for (int k = 0; k < HS_CONV_CACHE; k++)
        if (g_cache[k].f && g_cache[k].P == P && g_cache[k].mode == mode) {
            *f = g_cache[k].f;
            *i = g_cache[k].i;
            pthread_mutex_unlock(&g_clock);
            return;
        }
    const int slot = g_cache_next++ % HS_CONV_CACHE;
    if (g_cache[slot].f) {
        free_real_fft(g_cache[slot].f);
        free_real_fft(g_cache[slot].i);
    }
    g_cache[slot].P = P;
    g_cache[slot].mode = mode;
    g_cache[slot].f = fft_real_init(P, 1);
    g_cache[slot].i = fft_real_init(P, -1);
    *f = g_cache[slot].f;
    *i = g_cache[slot].i;
    pthread_mutex_unlock(&g_clock);
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
    fft_real_object f, iv;
    conv_plans(P, &f, &iv);
    /* the reference multiplies all P mirrored bins (convolve.c:147-151), but its c2r reads
     * bins 0..P/2 only (real.c:169-179): compact spectra of P/2+1 bins give the same bits
     * with a third less traffic */
    const long long cd = P / 2 + 1;
    double *pa = hs_scratch(7, sizeof(double) * (size_t)P * 2 * (size_t)batch);
    fft_data *spec = hs_scratch(10, sizeof(fft_data) * (size_t)cd * 2 * (size_t)batch);
    if (!pa || !spec) return HSFFT_ERR_NOMEM;
    double *pb = pa + (size_t)P * batch;
    fft_data *A = spec, *B = spec + (size_t)cd * batch;
    int rc = hsd_copy_rows(d_a, n, 0, n, pa, P, P, batch) || hsd_copy_rows(d_b, m, 0, m, pb, P, P, batch)
                 ? HSFFT_ERR_DEVICE : 0;
    if (!rc) rc = hsfft_r2c_batched_compact(f, pa, A, batch);
    if (!rc) rc = hsfft_r2c_batched_compact(f, pb, B, batch);
    if (!rc) rc = hs_c2r_product_rows(iv, A, B, cd, d_res, batch); /* product fused into the pre-twiddle */
    if (!rc && scale) rc = hsd_scale_real(d_res, P, batch, P, (double)P) ? HSFFT_ERR_DEVICE : 0;
    if (!rc) rc = hsd_sync() ? HSFFT_ERR_DEVICE : 0;
    return rc;
}

int fft_convolve(const char *type, const char *conv_type, fft_type *input1, int length1, fft_type *input2,
                 int length2, fft_type *output)
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

int hsfft_convolve_batched(const char *type, const char *conv_type, const fft_type *d_a, int length1,
                           const fft_type *d_b, int length2, fft_type *d_out, int batch)
{
    if (!d_a || !d_b || !d_out || length1 <= 0 || length2 <= 0 || batch < 0) return HSFFT_ERR_ARG;
    int linear, clen, P, start;
    if (conv_setup(conv_type, length1, length2, &linear, &clen, &P)) return HSFFT_ERR_ARG;
    const int len = conv_window(type, linear, clen, P, length1, length2, &start);
    if (len < 0) return HSFFT_ERR_ARG;
    if (batch == 0) return len;
    int rc = hs_require_gpu();
    if (rc) return rc;
    double *d_res = hsfft_malloc(sizeof(double) * (size_t)P * (size_t)batch);
    if (!d_res) return HSFFT_ERR_NOMEM;
    rc = conv_device(P, d_a, length1, d_b, length2, d_res, batch, 0);
    /* the 1/P scale (convolve.c:157-160) fused into the window copy: same division per element */
    if (!rc && len > 0)
        rc = hsd_copy_rows_div(d_res, P, start, d_out, len, len, batch, (double)P) ? HSFFT_ERR_DEVICE : 0;
    if (!rc) rc = hsd_sync() ? HSFFT_ERR_DEVICE : 0;
    hsfft_free(d_res);
    return rc ? rc : len;
}
