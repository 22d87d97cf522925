/*
 * highspeedFFT.h -- drop-in replacement for the reference header
 * (Tugbars/Mixed-Radix-Fast-Fourier-Transform, src/highspeedFFT.h:1-68).
 *
 * Same types, same struct layout (N@0, sgn@4, factors@8, lf@264, lt@268, twiddle@272,
 * sizeof 288) and the same prototypes, so existing C callers recompile/relink unchanged
 * against libhsfft.so.  The transforms themselves run on an AMD Instinct MI355X (gfx950);
 * see hsfft_gpu.h for the batched / device-pointer extension API.
 */
#ifndef HSFFT_H_
#define HSFFT_H_

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PI2 6.28318530717958647692528676655900577 /* ref highspeedFFT.h:13 */

#ifndef fft_type
#define fft_type double /* ref highspeedFFT.h:15-17; the GPU path supports double only */
#endif

/* complex sample, interleaved {re, im} (ref highspeedFFT.h:20-23) */
typedef struct fft_t {
    fft_type re;
    fft_type im;
} fft_data;

typedef struct fft_set *fft_object;

/* plan (ref highspeedFFT.h:36-43); twiddle[] holds N-1 (mixed radix) or M-1 (Bluestein)
 * stage-major twiddles, imaginary parts negated for sgn == -1 */
struct fft_set {
    int N;
    int sgn;
    int factors[64];
    int lf;
    int lt; /* 0 mixed radix, 1 Bluestein */
    fft_data twiddle[1];
};

/* replaces ref highSpeedFFT.c:206 (fft_init) */
fft_object fft_init(int N, int sgn);
/* replaces ref highSpeedFFT.c:1920 (fft_exec): out-of-place, N samples; host or device
 * pointers (device pointers run in place on the GPU, host pointers are staged) */
void fft_exec(fft_object obj, fft_data *inp, fft_data *oup);
/* replaces ref highSpeedFFT.c:1954 */
int divideby(int M, int d);
/* replaces ref highSpeedFFT.c:1979 */
int dividebyN(int N);
/* replaces ref highSpeedFFT.c:2038 */
int factors(int M, int *arr);
/* replaces ref highSpeedFFT.c:2186 (unused by the library, kept for ABI) */
void twiddle(fft_data *sig, int N, int radix);
/* replaces ref highSpeedFFT.c:2238 */
void longvectorN(fft_data *sig, int N, int *array, int M);
/* replaces ref highSpeedFFT.c:2315; also releases the plan's device state */
void free_fft(fft_object object);

#ifdef __cplusplus
}
#endif

#endif /* HSFFT_H_ */
