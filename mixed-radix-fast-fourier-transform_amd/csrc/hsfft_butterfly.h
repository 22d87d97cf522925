/*
 * hsfft_butterfly.h -- radix-2/3/4/5/7/8 and odd-radix butterflies for gfx950.
 *
 * Arithmetic restated from the reference (src/highSpeedFFT.c): leaves :344-713, combine
 * stages :714-1474, odd radix :1475-1628.  Every expression keeps the reference's operand
 * order and association; compiled with -ffp-contract=off so no FMA is formed, which makes
 * the results bit-identical to the CPU reference.  Two leaf/combine differences matter:
 * radix-5/7 sum their DC output as x0+(t0+t1[+t2]) in the leaf (:515, :608) and as
 * ((x0+t0)+t1)[+t2] in the combine stage (:950, :1132).
 */
#ifndef HSFFT_BUTTERFLY_H_
#define HSFFT_BUTTERFLY_H_

#include <hip/hip_runtime.h>

namespace hsb {

constexpr double K3 = 0.86602540378;
constexpr double K5C1 = 0.30901699437, K5C2 = -0.80901699437;
constexpr double K5S1 = 0.95105651629, K5S2 = 0.58778525229;
constexpr double K7C1 = 0.62348980185, K7C2 = -0.22252093395, K7C3 = -0.9009688679;
constexpr double K7S1 = 0.78183148246, K7S2 = 0.97492791218, K7S3 = 0.43388373911;
constexpr double K8 = 0.70710678118654752440084436210485;

template <int R>
__device__ __forceinline__ void bfly(double *xr, double *xi, int sgn, bool leaf);

template <>
__device__ __forceinline__ void bfly<2>(double *xr, double *xi, int, bool)
{
    double ar = xr[0], ai = xi[0], br = xr[1], bi = xi[1];
    xr[0] = ar + br; xi[0] = ai + bi;
    xr[1] = ar - br; xi[1] = ai - bi;
}

template <>
__device__ __forceinline__ void bfly<3>(double *xr, double *xi, int sgn, bool)
{
    const double sc = sgn * K3;
    double t0r = xr[1] + xr[2], t0i = xi[1] + xi[2];
    double t1r = sc * (xr[1] - xr[2]), t1i = sc * (xi[1] - xi[2]);
    double t2r = xr[0] - t0r * 0.5, t2i = xi[0] - t0i * 0.5;
    xr[0] = xr[0] + t0r; xi[0] = xi[0] + t0i;
    xr[1] = t2r + t1i; xi[1] = t2i - t1r;
    xr[2] = t2r - t1i; xi[2] = t2i + t1r;
}

template <>
__device__ __forceinline__ void bfly<4>(double *xr, double *xi, int sgn, bool)
{
    double t0r = xr[0] + xr[2], t0i = xi[0] + xi[2];
    double t1r = xr[0] - xr[2], t1i = xi[0] - xi[2];
    double t2r = xr[1] + xr[3], t2i = xi[1] + xi[3];
    double t3r = sgn * (xr[1] - xr[3]), t3i = sgn * (xi[1] - xi[3]);
    xr[0] = t0r + t2r; xi[0] = t0i + t2i;
    xr[1] = t1r + t3i; xi[1] = t1i - t3r;
    xr[2] = t0r - t2r; xi[2] = t0i - t2i;
    xr[3] = t1r - t3i; xi[3] = t1i + t3r;
}

template <>
__device__ __forceinline__ void bfly<5>(double *xr, double *xi, int sgn, bool leaf)
{
    const double ar = xr[0], ai = xi[0];
    double t0r = xr[1] + xr[4], t0i = xi[1] + xi[4];
    double t1r = xr[2] + xr[3], t1i = xi[2] + xi[3];
    double t2r = xr[1] - xr[4], t2i = xi[1] - xi[4];
    double t3r = xr[2] - xr[3], t3i = xi[2] - xi[3];
    double y0r, y0i;
    if (leaf) { y0r = ar + (t0r + t1r); y0i = ai + (t0i + t1i); }
    else      { y0r = ar + t0r + t1r;   y0i = ai + t0i + t1i; }
    double t4r = K5C1 * t0r + K5C2 * t1r, t4i = K5C1 * t0i + K5C2 * t1i, t5r, t5i;
    if (sgn == 1) { t5r = K5S1 * t2r + K5S2 * t3r; t5i = K5S1 * t2i + K5S2 * t3i; }
    else          { t5r = -K5S1 * t2r - K5S2 * t3r; t5i = -K5S1 * t2i - K5S2 * t3i; }
    double t6r = ar + t4r, t6i = ai + t4i;
    double y1r = t6r + t5i, y1i = t6i - t5r, y4r = t6r - t5i, y4i = t6i + t5r;
    t4r = K5C2 * t0r + K5C1 * t1r; t4i = K5C2 * t0i + K5C1 * t1i;
    if (sgn == 1) { t5r = K5S2 * t2r - K5S1 * t3r; t5i = K5S2 * t2i - K5S1 * t3i; }
    else          { t5r = -K5S2 * t2r + K5S1 * t3r; t5i = -K5S2 * t2i + K5S1 * t3i; }
    t6r = ar + t4r; t6i = ai + t4i;
    xr[0] = y0r; xi[0] = y0i;
    xr[1] = y1r; xi[1] = y1i;
    xr[4] = y4r; xi[4] = y4i;
    xr[2] = t6r + t5i; xi[2] = t6i - t5r;
    xr[3] = t6r - t5i; xi[3] = t6i + t5r;
}

template <>
__device__ __forceinline__ void bfly<7>(double *xr, double *xi, int sgn, bool leaf)
{
    const double ar = xr[0], ai = xi[0];
    double t0r = xr[1] + xr[6], t3r = xr[1] - xr[6], t0i = xi[1] + xi[6], t3i = xi[1] - xi[6];
    double t1r = xr[2] + xr[5], t4r = xr[2] - xr[5], t1i = xi[2] + xi[5], t4i = xi[2] - xi[5];
    double t2r = xr[3] + xr[4], t5r = xr[3] - xr[4], t2i = xi[3] + xi[4], t5i = xi[3] - xi[4];
    double y0r, y0i;
    if (leaf) { y0r = ar + (t0r + t1r + t2r); y0i = ai + (t0i + t1i + t2i); }
    else      { y0r = ar + t0r + t1r + t2r;   y0i = ai + t0i + t1i + t2i; }
    double t6r, t6i, t7r, t7i;
    /* outputs 1 / 6 */
    t6r = ar + K7C1 * t0r + K7C2 * t1r + K7C3 * t2r;
    t6i = ai + K7C1 * t0i + K7C2 * t1i + K7C3 * t2i;
    if (sgn == 1) { t7r = -K7S1 * t3r - K7S2 * t4r - K7S3 * t5r; t7i = -K7S1 * t3i - K7S2 * t4i - K7S3 * t5i; }
    else          { t7r = K7S1 * t3r + K7S2 * t4r + K7S3 * t5r;  t7i = K7S1 * t3i + K7S2 * t4i + K7S3 * t5i; }
    double y1r = t6r - t7i, y1i = t6i + t7r, y6r = t6r + t7i, y6i = t6i - t7r;
    /* outputs 2 / 5 */
    t6r = ar + K7C2 * t0r + K7C3 * t1r + K7C1 * t2r;
    t6i = ai + K7C2 * t0i + K7C3 * t1i + K7C1 * t2i;
    if (sgn == 1) { t7r = -K7S2 * t3r + K7S3 * t4r + K7S1 * t5r; t7i = -K7S2 * t3i + K7S3 * t4i + K7S1 * t5i; }
    else          { t7r = K7S2 * t3r - K7S3 * t4r - K7S1 * t5r;  t7i = K7S2 * t3i - K7S3 * t4i - K7S1 * t5i; }
    double y2r = t6r - t7i, y2i = t6i + t7r, y5r = t6r + t7i, y5i = t6i - t7r;
    /* outputs 3 / 4 */
    t6r = ar + K7C3 * t0r + K7C1 * t1r + K7C2 * t2r;
    t6i = ai + K7C3 * t0i + K7C1 * t1i + K7C2 * t2i;
    if (sgn == 1) { t7r = -K7S3 * t3r + K7S1 * t4r - K7S2 * t5r; t7i = -K7S3 * t3i + K7S1 * t4i - K7S2 * t5i; }
    else          { t7r = K7S3 * t3r - K7S1 * t4r + K7S2 * t5r;  t7i = K7S3 * t3i - K7S1 * t4i + K7S2 * t5i; }
    xr[0] = y0r; xi[0] = y0i;
    xr[1] = y1r; xi[1] = y1i; xr[6] = y6r; xi[6] = y6i;
    xr[2] = y2r; xi[2] = y2i; xr[5] = y5r; xi[5] = y5i;
    xr[3] = t6r - t7i; xi[3] = t6i + t7r;
    xr[4] = t6r + t7i; xi[4] = t6i - t7r;
}

template <>
__device__ __forceinline__ void bfly<8>(double *xr, double *xi, int sgn, bool)
{
    double t0r = xr[0] + xr[4], t4r = xr[0] - xr[4], t0i = xi[0] + xi[4], t4i = xi[0] - xi[4];
    double t1r = xr[1] + xr[7], t5r = xr[1] - xr[7], t1i = xi[1] + xi[7], t5i = xi[1] - xi[7];
    double t2r = xr[3] + xr[5], t6r = xr[3] - xr[5], t2i = xi[3] + xi[5], t6i = xi[3] - xi[5];
    double t3r = xr[2] + xr[6], t7r = xr[2] - xr[6], t3i = xi[2] + xi[6], t7i = xi[2] - xi[6];
    double y0r = t0r + t1r + t2r + t3r, y0i = t0i + t1i + t2i + t3i;
    double y4r = t0r - t1r - t2r + t3r, y4i = t0i - t1i - t2i + t3i;
    double d1r = t1r - t2r, d1i = t1i - t2i, d2r = t5r + t6r, d2i = t5i + t6i;
    double t8r, t8i, t9r, t9i;
    t8r = t4r + K8 * d1r; t8i = t4i + K8 * d1i;
    if (sgn == 1) { t9r = -K8 * d2r - t7r; t9i = -K8 * d2i - t7i; }
    else          { t9r = K8 * d2r + t7r;  t9i = K8 * d2i + t7i; }
    double y1r = t8r - t9i, y1i = t8i + t9r, y7r = t8r + t9i, y7i = t8i - t9r;
    t8r = t0r - t3r; t8i = t0i - t3i;
    if (sgn == 1) { t9r = -t5r + t6r; t9i = -t5i + t6i; }
    else          { t9r = t5r - t6r;  t9i = t5i - t6i; }
    double y2r = t8r - t9i, y2i = t8i + t9r, y6r = t8r + t9i, y6i = t8i - t9r;
    t8r = t4r - K8 * d1r; t8i = t4i - K8 * d1i;
    if (sgn == 1) { t9r = -K8 * d2r + t7r; t9i = -K8 * d2i + t7i; }
    else          { t9r = K8 * d2r - t7r;  t9i = K8 * d2i - t7i; }
    xr[0] = y0r; xi[0] = y0i; xr[4] = y4r; xi[4] = y4i;
    xr[1] = y1r; xi[1] = y1i; xr[7] = y7r; xi[7] = y7i;
    xr[2] = y2r; xi[2] = y2i; xr[6] = y6r; xi[6] = y6i;
    xr[3] = t8r - t9i; xi[3] = t8i + t9r;
    xr[5] = t8r + t9i; xi[5] = t8i - t9r;
}

/* odd radix p (>= 9, <= 63) from host-precomputed cos/sin (sincos(i*PI2/p), mirrored as
 * at :1536-1541): cs[0..p-2], sn[0..p-2]. */
__device__ inline void bfly_odd(double *xr, double *xi, int p, int sgn, const double *cs, const double *sn)
{
    const int mid = (p - 1) / 2;
    double tr[64], ti[64], yr[64], yi[64];
    for (int i = 0; i < mid; i++) {
        tr[i] = xr[i + 1] + xr[p - 1 - i];
        ti[i + mid] = xi[i + 1] - xi[p - 1 - i];
        ti[i] = xi[i + 1] + xi[p - 1 - i];
        tr[i + mid] = xr[i + 1] - xr[p - 1 - i];
    }
    double ar = xr[0], ai = xi[0];
    for (int i = 0; i < mid; i++) { ar += tr[i]; ai += ti[i]; }
    yr[0] = ar; yi[0] = ai;
    for (int u = 0; u < mid; u++) {
        double ur = xr[0], ui = xi[0], vr = 0.0, vi = 0.0;
        for (int v = 0; v < mid; v++) {
            int t = ((u + 1) * (v + 1)) % p - 1;
            ur += cs[t] * tr[v];
            ui += cs[t] * ti[v];
            vr -= sn[t] * tr[v + mid];
            vi -= sn[t] * ti[v + mid];
        }
        vr = sgn * vr;
        vi = sgn * vi;
        yr[u + 1] = ur - vi; yi[u + 1] = ui + vr;
        yr[p - u - 1] = ur + vi; yi[p - u - 1] = ui - vr;
    }
    for (int i = 0; i < p; i++) { xr[i] = yr[i]; xi[i] = yi[i]; }
}

/* twiddle application of the combine stages: b = x * w, written as at :740-741 */
__device__ __forceinline__ void twmul(double &xr, double &xi, double wr, double wi)
{
    double br = xr * wr - xi * wi;
    double bi = xi * wr + xr * wi;
    xr = br;
    xi = bi;
}

}  // namespace hsb

#endif
