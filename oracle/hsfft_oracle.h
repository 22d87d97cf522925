/*
 * hsfft_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference highSpeedFFT arithmetic (Tugbars/Mixed-Radix-Fast-
 * Fourier-Transform, src/highSpeedFFT.c, src/real.c, src/convolve.c).  It is the checker
 * the GPU path is compared against; it is never linked into, loaded by, or called from the
 * product library (libhsfft.so).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it.
 *
 * Pinning: tests/test_oracle_pin.py compares it bit-for-bit with the reference compiled
 * unmodified from /root/reference/src (oracle/_ref/libhsref.so, built by oracle/Makefile)
 * and tests/test_oracle_golden.py against committed fixtures generated from that build
 * (tests/golden/make_golden.py).
 */
#ifndef HSFFT_ORACLE_H_
#define HSFFT_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double re, im; } orc_cplx;

/* flags */
#define ORC_TWIDDLE_EXACT 1  /* compute every stage twiddle with sincos (reference: USE_TWIDDLE_TABLES off) */
#define ORC_LEAF2_ASIS    2  /* radix-2 leaf reads the caller's output slot (defect D1) instead of x0 */

typedef struct orc_plan orc_plan;

orc_plan *orc_plan_create(int N, int sgn, int flags);
void      orc_plan_destroy(orc_plan *p);
int       orc_plan_lt(const orc_plan *p);          /* 0 mixed radix, 1 Bluestein */
int       orc_plan_M(const orc_plan *p);           /* transform length the twiddles belong to */
int       orc_plan_factors(const orc_plan *p, int *out64);
const orc_cplx *orc_plan_twiddles(const orc_plan *p); /* M-1 entries, sign already applied */

/* one transform, out-of-place; `out` is read first only in ORC_LEAF2_ASIS mode */
void orc_exec(const orc_plan *p, const orc_cplx *in, orc_cplx *out);
/* contiguous rows; nthreads<=0 -> 1 */
void orc_exec_batch(const orc_plan *p, const orc_cplx *in, orc_cplx *out, int batch, int nthreads);

/* planner pieces (reference highSpeedFFT.c:1979-2163) */
int orc_dividebyN(int N);
int orc_factors(int M, int *arr);
/* digit-reversal map of the recursion: out position q <- input index map[q] */
void orc_digit_reverse_map(const orc_plan *p, int *map);

/* real transforms (reference real.c:26-193) */
typedef struct orc_real_plan orc_real_plan;
orc_real_plan *orc_real_create(int N, int sgn, int flags);
void orc_real_destroy(orc_real_plan *rp);
void orc_r2c(const orc_real_plan *rp, const double *in, orc_cplx *out);   /* writes N outputs */
void orc_c2r(const orc_real_plan *rp, const orc_cplx *in, double *out);   /* reads N/2+1 inputs */
void orc_r2c_batch(const orc_real_plan *rp, const double *in, orc_cplx *out, int batch, int nthreads);

/* convolution (reference convolve.c:74-214); returns output length or -1 */
int orc_convolve(const char *type, const char *conv_type, const double *a, int n,
                 const double *b, int m, double *out, int flags);

/* synthetic inputs: u(i) = splitmix64(seed ^ i) mapped to [-1, 1) */
double orc_uniform(uint64_t seed, uint64_t i);
void   orc_fill_complex(orc_cplx *x, int64_t count, uint64_t seed, uint64_t offset);
void   orc_fill_real(double *x, int64_t count, uint64_t seed, uint64_t offset);

#ifdef __cplusplus
}
#endif
#endif
