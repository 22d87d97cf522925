/*
 * real.h -- drop-in replacement for the reference real-signal header
 * (Tugbars/Mixed-Radix-Fast-Fourier-Transform, src/real.h:1-89), plus the convolution entry
 * point the reference defines in src/convolve.c without a header.
 */
#ifndef REAL_H_
#define REAL_H_

#include "highspeedFFT.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fft_real_set *fft_real_object;

/* ref real.h:23-32: layout cobj@0, twiddle2@8 (N/2 entries of (cos, sin)(2*pi*k/N)) */
struct fft_real_set {
    fft_object cobj;
    fft_data twiddle2[1];
};

/* replaces ref real.c:26 (fft_real_init); N must be positive and even */
fft_real_object fft_real_init(int N, int sgn);
/* replaces ref real.c:78 (fft_r2c_exec): N reals in, N complex out (Hermitian-mirrored,
 * as the reference writes, real.c:128-132) */
void fft_r2c_exec(fft_real_object obj, fft_type *inp, fft_data *oup);
/* replaces ref real.c:150 (fft_c2r_exec): reads N/2+1 bins, writes N reals (unnormalised) */
void fft_c2r_exec(fft_real_object obj, fft_data *inp, fft_type *oup);
/* replaces ref real.c:259 */
void free_real_fft(fft_real_object obj);

/* replaces ref convolve.c:74 (fft_convolve), :20 and :39 */
int fft_convolve(const char *type, const char *conv_type, fft_type *input1, int length1,
                 fft_type *input2, int length2, fft_type *output);
int next_power_of_two(int n);
int find_optimal_fft_length(int min_length, const char *conv_type, int length1, int length2);

#ifdef __cplusplus
}
#endif

#endif /* REAL_H_ */
