/*
 * dropin_caller.c -- an unmodified-caller test of libhsfft.so (tests/test_gpu_c_caller.py).
 *
 * Written the way a user of the reference writes it: only the reference's own headers
 * (highspeedFFT.h, real.h) are included, buffers are plain malloc'd host memory, and the
 * calls follow the reference's usage -- fft_init / fft_exec / free_fft (highSpeedFFT.c:206,
 * :1920, :2315), fft_real_init / fft_r2c_exec / fft_c2r_exec / free_real_fft (real.c:26,
 * :78, :150, :259; as called by convolve.c:104-154) and fft_convolve (convolve.c:74).  The
 * program is compiled against include/ and linked to lib/libhsfft.so, i.e. "recompile and
 * relink unchanged".
 *
 * Input: a case file, one case per line
 *   c2c  <n> <sgn> <seed>                 splitmix64 complex input (tests/hsfft_testlib.py)
 *   r2c  <n> <sgn> <seed>                 splitmix64 real input
 *   c2r  <n> <sgn> <spectrum file>        n complex doubles read from the file
 *   conv <type> <conv_type> <n> <m> <seed_a> <seed_b>
 * Output: for every case, an int64 count of doubles followed by the doubles.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "highspeedFFT.h"
#include "real.h"

int fft_convolve(const char *type, const char *conv_type, fft_type *input1, int length1, fft_type *input2,
                 int length2, fft_type *output); /* convolve.c:74 has no header in the reference */

static double uniform(uint64_t seed, uint64_t i)
{
    uint64_t z = (seed ^ i) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 4503599627370496.0) - 1.0;
}

static void emit(FILE *o, const double *v, int64_t n)
{
    fwrite(&n, sizeof n, 1, o);
    fwrite(v, sizeof(double), (size_t)n, o);
}

int main(int argc, char **argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s <cases> <out>\n", argv[0]);
        return 2;
    }
    FILE *in = fopen(argv[1], "r"), *out = fopen(argv[2], "wb");
    if (!in || !out) return 2;
    char kind[16];
    while (fscanf(in, "%15s", kind) == 1) {
        if (!strcmp(kind, "c2c")) {
            int n, sgn;
            unsigned long long seed;
            if (fscanf(in, "%d %d %llu", &n, &sgn, &seed) != 3) return 3;
            fft_data *x = malloc(sizeof(fft_data) * (size_t)n), *y = calloc((size_t)n, sizeof(fft_data));
            for (int i = 0; i < n; i++) {
                x[i].re = uniform(seed, 2ull * i);
                x[i].im = uniform(seed, 2ull * i + 1);
            }
            fft_object obj = fft_init(n, sgn);
            fft_exec(obj, x, y);
            free_fft(obj);
            emit(out, (const double *)y, 2LL * n);
            free(x);
            free(y);
        } else if (!strcmp(kind, "r2c")) {
            int n, sgn;
            unsigned long long seed;
            if (fscanf(in, "%d %d %llu", &n, &sgn, &seed) != 3) return 3;
            fft_type *x = malloc(sizeof(fft_type) * (size_t)n);
            fft_data *y = calloc((size_t)n, sizeof(fft_data)); /* the reference writes all N bins */
            for (int i = 0; i < n; i++) x[i] = uniform(seed, (uint64_t)i);
            fft_real_object r = fft_real_init(n, sgn);
            fft_r2c_exec(r, x, y);
            free_real_fft(r);
            emit(out, (const double *)y, 2LL * n);
            free(x);
            free(y);
        } else if (!strcmp(kind, "c2r")) {
            int n, sgn;
            char path[4096];
            if (fscanf(in, "%d %d %4095s", &n, &sgn, path) != 3) return 3;
            fft_data *X = malloc(sizeof(fft_data) * (size_t)n);
            fft_type *y = calloc((size_t)n, sizeof(fft_type));
            FILE *f = fopen(path, "rb");
            if (!f || fread(X, sizeof(fft_data), (size_t)n, f) != (size_t)n) return 4;
            fclose(f);
            fft_real_object r = fft_real_init(n, sgn);
            fft_c2r_exec(r, X, y);
            free_real_fft(r);
            emit(out, y, n);
            free(X);
            free(y);
        } else if (!strcmp(kind, "conv")) {
            char type[16], ctype[16];
            int n, m;
            unsigned long long sa, sb;
            if (fscanf(in, "%15s %15s %d %d %llu %llu", type, ctype, &n, &m, &sa, &sb) != 6) return 3;
            fft_type *a = malloc(sizeof(fft_type) * (size_t)n), *b = malloc(sizeof(fft_type) * (size_t)m);
            for (int i = 0; i < n; i++) a[i] = uniform(sa, (uint64_t)i);
            for (int i = 0; i < m; i++) b[i] = uniform(sb, (uint64_t)i);
            const int cap = 2 * (n + m) + 8;
            fft_type *o = calloc((size_t)cap, sizeof(fft_type));
            const int len = fft_convolve(type, ctype, a, n, b, m, o);
            emit(out, o, len < 0 ? 0 : len);
            free(a);
            free(b);
            free(o);
        } else {
            fprintf(stderr, "unknown case %s\n", kind);
            return 3;
        }
    }
    fclose(in);
    fclose(out);
    return 0;
}
