/* Which environment lookups does ONE drop-in fft_exec (N = 1024, host buffers) make?  The
 * executable defines getenv itself (exported with -rdynamic), so every getenv of libhsfft.so and
 * of the HIP runtime resolves here: each call is counted by name, then forwarded to libc's.
 *   gcc -O2 -rdynamic -o tools/experiments/c1_getenv tools/experiments/c1_getenv.c -Iinclude \
 *       -Lmixed-radix-fast-fourier-transform_amd/lib -lhsfft -ldl \
 *       -Wl,-rpath,$PWD/mixed-radix-fast-fourier-transform_amd/lib
 * Measurement aid only (round 6: 500 extra environment variables cost c1 5.5 us per call). */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "highspeedFFT.h"
#include "hsfft_gpu.h"

static char *(*real_getenv)(const char *);
static int counting;
static struct {
    char name[64];
    long n;
} tab[256];
static int ntab;
static long total;

char *getenv(const char *name)
{
    if (!real_getenv) real_getenv = (char *(*)(const char *))dlsym(RTLD_NEXT, "getenv");
    if (counting) {
        __atomic_fetch_add(&total, 1, __ATOMIC_RELAXED);
        int i = 0;
        for (; i < ntab; i++)
            if (!strncmp(tab[i].name, name, 63)) break;
        if (i == ntab && ntab < 256) {
            strncpy(tab[ntab].name, name, 63);
            ntab++;
        }
        if (i < 256) tab[i].n++;
    }
    return real_getenv(name);
}

static double now_us(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

int main(void)
{
    if (hsfft_set_device(0)) return 1;
    fft_object o = fft_init(1024, 1);
    fft_data *x = calloc(1024, sizeof *x), *y = calloc(1024, sizeof *y);
    for (int i = 0; i < 1024; i++) x[i].re = (double)(i % 7);
    for (int i = 0; i < 200; i++) fft_exec(o, x, y);
    const int calls = 2000;
    counting = 1;
    const double t0 = now_us();
    for (int i = 0; i < calls; i++) fft_exec(o, x, y);
    const double t1 = now_us();
    counting = 0;
    printf("%.2f getenv calls per fft_exec, %.2f us per call (mean, counting on)\n", (double)total / calls,
           (t1 - t0) / calls);
    for (int i = 0; i < ntab; i++) printf("  %-40s %.2f per call\n", tab[i].name, (double)tab[i].n / calls);
    free_fft(o);
    hsfft_finalize();
    return 0;
}
