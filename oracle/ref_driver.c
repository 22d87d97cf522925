/*
 * ref_driver.c -- TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Linked together with the UNMODIFIED reference sources (compiled from /root/reference/src
 * by oracle/Makefile into oracle/_ref/libhsref.so).  Provides a threaded timing loop for
 * bench.py's cpu_baseline leg: the reference has no batch API, and bluestein_fft mutates its
 * plan (highSpeedFFT.c:1759-1760), so every thread builds its own plan with fft_init.
 * Only the reference's public prototypes (highspeedFFT.h:34-59, real.h:46-84) are declared.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { double re, im; } rd_cplx;
typedef void *rd_obj;
extern rd_obj fft_init(int N, int sgn);
extern void fft_exec(rd_obj obj, rd_cplx *in, rd_cplx *out);
extern void free_fft(rd_obj obj);
extern rd_obj fft_real_init(int N, int sgn);
extern void fft_r2c_exec(rd_obj obj, double *in, rd_cplx *out);
extern void free_real_fft(rd_obj obj);

static double rd_uniform(uint64_t seed, uint64_t i)
{
    uint64_t z = (seed ^ i) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 4503599627370496.0) - 1.0;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

typedef struct {
    int N, sgn, real, b0, b1, reps;
    uint64_t seed;
    pthread_barrier_t *bar;
    double elapsed;
} rd_job;

static void *rd_worker(void *arg)
{
    rd_job *j = arg;
    int N = j->N;
    rd_obj obj = j->real ? fft_real_init(N, j->sgn) : fft_init(N, j->sgn);
    size_t nin = j->real ? (size_t)N : 2 * (size_t)N, rows = (size_t)(j->b1 - j->b0);
    double *in = malloc(sizeof(double) * nin * (rows ? rows : 1));
    rd_cplx *out = calloc((size_t)N * (rows ? rows : 1), sizeof(rd_cplx));
    /* the same splitmix64 stream the GPU path uses, generated before the timed region */
    for (size_t r = 0; r < rows; r++) {
        uint64_t base = (uint64_t)(j->b0 + (int)r) * (uint64_t)nin;
        for (size_t i = 0; i < nin; i++) in[r * nin + i] = rd_uniform(j->seed, base + i);
    }
    pthread_barrier_wait(j->bar);
    double t0 = now_s();
    for (int rep = 0; rep < j->reps; rep++)
    for (size_t r = 0; r < rows; r++) {
        if (j->real) fft_r2c_exec(obj, in + r * nin, out + r * (size_t)N);
        else fft_exec(obj, (rd_cplx *)(in + r * nin), out + r * (size_t)N);
    }
    j->elapsed = now_s() - t0;
    free(in);
    free(out);
    if (j->real) free_real_fft(obj);
    else free_fft(obj);
    return NULL;
}

/* Times `reps` sweeps over `batch` distinct transforms split over `nthreads` threads
 * (batch * reps transforms in all); returns wall seconds of the slowest thread (plan
 * creation and input generation excluded). */
double hsref_time_batch_reps(int N, int sgn, int real, int batch, int nthreads, uint64_t seed, int reps)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > batch) nthreads = batch;
    if (nthreads > 512) nthreads = 512;
    if (reps < 1) reps = 1;
    pthread_t th[512];
    rd_job jobs[512];
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (rd_job){N, sgn, real, (int)((long)batch * t / nthreads),
                           (int)((long)batch * (t + 1) / nthreads), reps, seed, &bar, 0.0};
        pthread_create(&th[t], NULL, rd_worker, &jobs[t]);
    }
    double worst = 0.0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].elapsed > worst) worst = jobs[t].elapsed;
    }
    pthread_barrier_destroy(&bar);
    return worst;
}

double hsref_time_batch(int N, int sgn, int real, int batch, int nthreads, uint64_t seed)
{
    return hsref_time_batch_reps(N, sgn, real, batch, nthreads, seed, 1);
}
