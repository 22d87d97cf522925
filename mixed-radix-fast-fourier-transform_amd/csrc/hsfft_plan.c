/*
 * hsfft_plan.c -- drop-in planner of libhsfft.so (host C).
 *
 * Clean-room implementation of the reference planner semantics:
 *   dividebyN    ref src/highSpeedFFT.c:13-55 (lookup) and :1979-2025 (division chain)
 *   divideby     ref :1954-1968
 *   factors      ref :2038-2163 (greedy 53..2, then the 6k+-1 sweep)
 *   twiddle      ref :2186-2224 (unused by the library; kept for ABI)
 *   longvectorN  ref :2238-2313 (stage-major twiddles; table quirk D2 in reference mode)
 *   fft_init     ref :206-286
 *   free_fft     ref :2315-2318
 * The plan bytes (struct fft_set + twiddles) equal the reference's for the same N and sgn
 * in the default "reference" twiddle mode (tests/test_product_planner.py).  Trig values
 * come from glibc sincos, which is what GCC -O2 fuses the reference's cos/sin pairs into.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsfft_gpu.h"
#include "hsfft_host.h"

/* ------------------------------------------------------------------ twiddle mode */
static int g_mode = -1;
static __thread int t_mode = -1;

int hs_twiddle_mode(void)
{
    if (t_mode >= 0) return t_mode;
    if (g_mode < 0) {
        const char *s = getenv("HSFFT_TWIDDLE");
        g_mode = (s && strcmp(s, "exact") == 0) ? 1 : 0;
    }
    return g_mode;
}

int hsfft_set_twiddle_mode(int mode)
{
    if (mode != 0 && mode != 1) return HSFFT_ERR_ARG;
    t_mode = mode;
    return 0;
}

int hsfft_get_twiddle_mode(void) { return hs_twiddle_mode(); }

/* ------------------------------------------------------------------ factorisation */
static const int k_accept[] = {53, 47, 43, 41, 37, 31, 29, 23, 17, 13, 11, 8, 7, 5, 4, 3, 2};
static const int k_greedy[] = {53, 47, 43, 41, 37, 31, 29, 23, 19, 17, 13, 11, 8, 7, 5, 4, 3, 2};

int divideby(int M, int d)
{
    if (M <= 0 || d <= 0) {
        fprintf(stderr, "Error: Invalid inputs for divideby - number: %d, divisor: %d\n", M, d);
        exit(EXIT_FAILURE);
    }
    if (d == 1) return M == 1;
    while (M % d == 0) M /= d;
    return M == 1;
}

int dividebyN(int N)
{
    /* The reference's lookup (N < 1024) and division chain accept exactly the numbers whose
     * prime factors lie in {2,3,5,7,11,13,17,23,...,53}; 19 is not in the set (D10). */
    if (N <= 0) return 0;
    for (unsigned i = 0; i < sizeof k_accept / sizeof k_accept[0]; i++)
        while (N % k_accept[i] == 0) N /= k_accept[i];
    return N == 1;
}

int factors(int M, int *arr)
{
    if (arr == NULL) {
        fprintf(stderr, "Error: Invalid inputs for factors - number: %d, factors_array: %p\n", M, (void *)arr);
        exit(EXIT_FAILURE);
    }
    if (M <= 0) return 0;
    int n = 0;
    for (unsigned i = 0; i < sizeof k_greedy / sizeof k_greedy[0]; i++)
        while (M % k_greedy[i] == 0) {
            arr[n++] = k_greedy[i];
            M /= k_greedy[i];
        }
    if (M > 31)
        for (int k = 2; M > 1; k++) {
            const int lo = 6 * k - 1, hi = 6 * k + 1;
            while (M % lo == 0) { arr[n++] = lo; M /= lo; }
            while (M % hi == 0) { arr[n++] = hi; M /= hi; }
        }
    return n;
}

/* ------------------------------------------------------------------ twiddles */
/* The reference's static tables hold 11-significant-digit roots of unity; twiddle_tables[]
 * is indexed by radix but shifted one slot (ref :102-116), so slot r holds the table of
 * radix r+1.  g_slot[r] reproduces that indexing for r <= 12. */
static const fft_data T2[] = {{1.0, 0.0}, {0.0, -1.0}};
static const fft_data T3[] = {{1.0, 0.0}, {-0.5, -0.86602540378}, {-0.5, 0.86602540378}};
static const fft_data T4[] = {{1.0, 0.0}, {0.0, -1.0}, {-1.0, 0.0}, {0.0, 1.0}};
static const fft_data T5[] = {{1.0, 0.0}, {0.30901699437, -0.95105651629}, {-0.80901699437, -0.58778525229},
                              {-0.80901699437, 0.58778525229}, {0.30901699437, 0.95105651629}};
static const fft_data T7[] = {{1.0, 0.0}, {0.62348980185, -0.78183148246}, {-0.22252093395, -0.97492791218},
                              {-0.9009688679, -0.43388373911}, {-0.9009688679, 0.43388373911},
                              {-0.22252093395, 0.97492791218}, {0.62348980185, 0.78183148246}};
static const fft_data T8[] = {{1.0, 0.0}, {0.70710678118, -0.70710678118}, {0.0, -1.0},
                              {-0.70710678118, -0.70710678118}, {-1.0, 0.0}, {-0.70710678118, 0.70710678118},
                              {0.0, 1.0}, {0.70710678118, 0.70710678118}};

static const fft_data *slot_table(int r)
{
    /* slots 10 and 12 (radix-11/13 tables) are never selected by a factor list: 10 and 12
     * are not factors, 11 maps to an empty slot, and slot 13 lies past the array (D3),
     * which this implementation treats as "no table" */
    switch (r) {
    case 1: return T2;
    case 2: return T3;
    case 3: return T4;
    case 4: return T5;
    case 6: return T7;
    case 7: return T8;
    default: return NULL;
    }
}

void hs_longvector(fft_data *tw, int M, const int *fac, int lf, int exact)
{
    int Ls = 1, c = 0;
    for (int s = 0; s < lf; s++) {
        const int r = fac[lf - 1 - s];
        const int L = Ls * r;
        const fft_data *tab = (!exact && r <= 12) ? slot_table(r) : NULL;
        const double theta = -PI2 / L;
        for (int j = 0; j < Ls; j++)
            for (int k = 0; k < r - 1; k++) {
                if (c >= M - 1) continue;
                if (tab) {
                    tw[c] = tab[k];
                } else {
                    double sn, cs;
                    sincos((k + 1) * j * theta, &sn, &cs);
                    tw[c].re = cs;
                    tw[c].im = sn;
                }
                c++;
            }
        Ls = L;
    }
    if (c != M - 1)
        fprintf(stderr, "Warning: Twiddle factor count (%d) does not match expected (%d) for N=%d\n", c, M - 1, M);
}

void longvectorN(fft_data *sig, int N, int *array, int M)
{
    if (N <= 0 || array == NULL || M <= 0) {
        fprintf(stderr, "Error: Invalid inputs for longvectorN - signal_length: %d, prime_factors: %p, num_factors: %d\n",
                N, (void *)array, M);
        exit(EXIT_FAILURE);
    }
    hs_longvector(sig, N, array, M, hs_twiddle_mode() == 1);
}

void twiddle(fft_data *sig, int N, int radix)
{
    if (N <= 0 || radix <= 0) {
        fprintf(stderr, "Error: Invalid inputs for twiddle - signal_length: %d, radix: %d\n", N, radix);
        exit(EXIT_FAILURE);
    }
    const int n = N / radix;
    const fft_data *tab = radix <= 8 ? slot_table(radix) : NULL;
    int start = 0;
    if (tab) {
        const int wrap = radix - 1 > 0 ? radix - 1 : 1;
        for (int i = 0; i < n && i < radix; i++) sig[i] = tab[i % wrap];
        start = radix - 1;
    }
    for (int i = start; i < n; i++) {
        double sn, cs;
        sincos(PI2 * i / N, &sn, &cs);
        sig[i].re = cs;
        sig[i].im = -sn;
    }
}

/* ------------------------------------------------------------------ Bluestein sizing */
int hs_bluestein_M_init(int N)
{
    const int p2 = (int)pow(2.0, ceil(log10(N) / log10(2.0)));
    return p2 < 2 * N - 2 ? 2 * p2 : p2;
}

int hs_bluestein_M_exec(int N) { return (int)pow(2.0, ceil(log2((double)(2 * N - 1)))); }

/* ------------------------------------------------------------------ fft_init / free_fft */
fft_object fft_init(int N, int sgn)
{
    if (N <= 0) { /* the reference hangs in factors(0) or indexes its table negatively */
        fprintf(stderr, "Error: Signal length (%d) must be positive\n", N);
        return NULL;
    }
    const int mixed = dividebyN(N);
    const int count = mixed ? N : hs_bluestein_M_init(N);
    fft_object obj = (fft_object)malloc(sizeof(struct fft_set) + sizeof(fft_data) * (size_t)(count - 1));
    if (obj == NULL) return NULL;
    memset(obj->factors, 0, sizeof obj->factors);
    obj->lf = factors(count, obj->factors);
    if (obj->lf > 0) hs_longvector(obj->twiddle, count, obj->factors, obj->lf, hs_twiddle_mode() == 1);
    /* the reference leaves the last slot uninitialised (it only holds count-1 twiddles) */
    obj->twiddle[count - 1].re = 0.0;
    obj->twiddle[count - 1].im = 0.0;
    obj->lt = mixed ? 0 : 1;
    obj->N = N;
    obj->sgn = sgn;
    if (sgn == -1)
        for (int i = 0; i < count; i++) obj->twiddle[i].im = -obj->twiddle[i].im;
    return obj;
}

void free_fft(fft_object object)
{
    if (object) hs_entry_release(object);
    free(object);
}
