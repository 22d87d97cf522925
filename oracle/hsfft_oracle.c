/*
 * hsfft_oracle.c -- TEST INFRASTRUCTURE ONLY (see hsfft_oracle.h).
 *
 * A compact, data-driven CPU restatement of the reference highSpeedFFT algorithm.  The
 * reference unrolls one hand-written block per radix; here the recursion, twiddle
 * application and butterflies are table/loop driven, but every floating-point expression
 * keeps the reference's operand order so results are bit-identical.  Each block cites the
 * reference lines it restates (paths relative to the reference root).
 *
 * Build: oracle/Makefile (gcc -O2 -std=gnu11 -ffp-contract=off, no -march).
 */
#define _GNU_SOURCE
#include "hsfft_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const double ORC_PI2 = 6.28318530717958647692528676655900577; /* highspeedFFT.h:13 */
static const double ORC_PI = 3.1415926535897932384626433832795;      /* highSpeedFFT.c:1682 */

struct orc_plan {
    int N, sgn, lt, M, lf, flags;
    int fac[64];
    orc_cplx *tw;        /* M-1 stage-major twiddles, imaginary parts negated when sgn == -1 */
    orc_cplx *hlt;       /* Bluestein chirp (N entries), lt == 1 only */
    struct orc_plan *mp; /* Bluestein: inner mixed-radix view of length M (shares tw) */
};

/* ------------------------------------------------------------------------------------ */
/* planner: highSpeedFFT.c:13-55 (lookup), 1979-2025 (dividebyN), 2038-2163 (factors)    */
/* ------------------------------------------------------------------------------------ */

int orc_dividebyN(int N)
{
    /* lookup table and division chain accept the same prime set; 19 is absent (defect D10) */
    static const int ok[] = {53, 47, 43, 41, 37, 31, 29, 23, 17, 13, 11, 8, 7, 5, 4, 3, 2};
    if (N <= 0) return 0;
    int r = N;
    for (unsigned i = 0; i < sizeof ok / sizeof ok[0]; i++)
        while (r % ok[i] == 0) r /= ok[i];
    return r == 1;
}

int orc_factors(int M, int *arr)
{
    static const int greedy[] = {53, 47, 43, 41, 37, 31, 29, 23, 19, 17, 13, 11, 8, 7, 5, 4, 3, 2};
    int n = 0, r = M;
    if (M <= 0) return 0;
    for (unsigned i = 0; i < sizeof greedy / sizeof greedy[0]; i++)
        while (r % greedy[i] == 0) { arr[n++] = greedy[i]; r /= greedy[i]; }
    if (r > 31) { /* 6k +- 1 sweep, highSpeedFFT.c:2139-2160 */
        for (int k = 2; r > 1; k++) {
            int f1 = 6 * k - 1, f2 = 6 * k + 1;
            while (r % f1 == 0) { arr[n++] = f1; r /= f1; }
            while (r % f2 == 0) { arr[n++] = f2; r /= f2; }
        }
    }
    return n;
}

/* The reference indexes twiddle_tables[] by radix but the table is shifted by one slot
 * (highSpeedFFT.c:102-116, used at :2257): radix 2,3,4,7 copy the first r-1 entries of the
 * radix 3,4,5,8 tables for every column j (defect D2).  Radix 13 reads past the array (D3);
 * the oracle computes it instead. */
static const orc_cplx *quirk_table(int r)
{
    static const orc_cplx t3[] = {{1.0, 0.0}, {-0.5, -0.86602540378}, {-0.5, 0.86602540378}};
    static const orc_cplx t4[] = {{1.0, 0.0}, {0.0, -1.0}, {-1.0, 0.0}, {0.0, 1.0}};
    static const orc_cplx t5[] = {{1.0, 0.0}, {0.30901699437, -0.95105651629},
                                  {-0.80901699437, -0.58778525229}, {-0.80901699437, 0.58778525229},
                                  {0.30901699437, 0.95105651629}};
    static const orc_cplx t8[] = {{1.0, 0.0}, {0.70710678118, -0.70710678118}, {0.0, -1.0},
                                  {-0.70710678118, -0.70710678118}, {-1.0, 0.0},
                                  {-0.70710678118, 0.70710678118}, {0.0, 1.0},
                                  {0.70710678118, 0.70710678118}};
    switch (r) {
    case 2: return t3;
    case 3: return t4;
    case 4: return t5;
    case 7: return t8;
    default: return NULL;
    }
}

/* longvectorN, highSpeedFFT.c:2238-2313: stage-major, innermost factor first */
static void orc_twiddles(orc_cplx *tw, int M, const int *fac, int lf, int exact)
{
    int Ls = 1, c = 0;
    for (int s = 0; s < lf; s++) {
        int r = fac[lf - 1 - s];
        int L = Ls * r;
        const orc_cplx *tab = exact ? NULL : quirk_table(r);
        double theta = -ORC_PI2 / L;
        for (int j = 0; j < Ls; j++)
            for (int k = 0; k < r - 1; k++) {
                if (c >= M - 1) continue;
                if (tab) {
                    tw[c] = tab[k];
                } else {
                    double a = (k + 1) * j * theta, sn, cs;
                    sincos(a, &sn, &cs);
                    tw[c].re = cs;
                    tw[c].im = sn;
                }
                c++;
            }
        Ls = L;
    }
}

static orc_plan *plan_mixed(int M, int sgn, int flags)
{
    orc_plan *p = calloc(1, sizeof *p);
    p->N = p->M = M;
    p->sgn = sgn;
    p->flags = flags;
    p->lf = orc_factors(M, p->fac);
    p->tw = calloc((size_t)(M > 1 ? M : 1), sizeof(orc_cplx));
    orc_twiddles(p->tw, M, p->fac, p->lf, flags & ORC_TWIDDLE_EXACT);
    if (sgn == -1) /* fft_init, highSpeedFFT.c:273-283 */
        for (int i = 0; i < M - 1; i++) p->tw[i].im = -p->tw[i].im;
    return p;
}

orc_plan *orc_plan_create(int N, int sgn, int flags)
{
    if (N <= 0) return NULL;
    if (orc_dividebyN(N)) return plan_mixed(N, sgn, flags);

    /* Bluestein.  fft_init sizes M with log10 (highSpeedFFT.c:242-252) but bluestein_fft
     * re-derives it with log2 (:1750-1751); they disagree for N = 2^k+1 (defect D5).  The
     * exec-side length is the one the arithmetic needs, so the oracle plans with it. */
    int M = (int)pow(2.0, ceil(log2((double)(2 * N - 1))));
    orc_plan *p = calloc(1, sizeof *p);
    p->N = N;
    p->sgn = sgn;
    p->lt = 1;
    p->flags = flags;
    p->M = M;
    p->mp = plan_mixed(M, sgn, flags);
    p->lf = p->mp->lf;
    memcpy(p->fac, p->mp->fac, sizeof p->fac);
    p->tw = p->mp->tw;
    /* chirp h(n) = exp(i*pi*n^2/N), n^2 tracked incrementally mod 2N with '>' (:1680-1690) */
    p->hlt = malloc(sizeof(orc_cplx) * (size_t)N);
    double theta = ORC_PI / N;
    int l2 = 0, len2 = 2 * N;
    for (int n = 0; n < N; n++) {
        double a = theta * l2, sn, cs;
        sincos(a, &sn, &cs);
        p->hlt[n].re = cs;
        p->hlt[n].im = sn;
        l2 += 2 * n + 1;
        while (l2 > len2) l2 -= len2;
    }
    return p;
}

void orc_plan_destroy(orc_plan *p)
{
    if (!p) return;
    if (p->mp) {
        free(p->mp->tw);
        free(p->mp);
    } else {
        free(p->tw);
    }
    free(p->hlt);
    free(p);
}

int orc_plan_lt(const orc_plan *p) { return p->lt; }
int orc_plan_M(const orc_plan *p) { return p->M; }
const orc_cplx *orc_plan_twiddles(const orc_plan *p) { return p->tw; }
int orc_plan_factors(const orc_plan *p, int *out64)
{
    memcpy(out64, p->fac, sizeof p->fac);
    return p->lf;
}

/* ------------------------------------------------------------------------------------ */
/* butterflies: highSpeedFFT.c:344-713 (leaves), :714-1474 (combine), :1475-1628 (odd p)  */
/* Every expression keeps the reference's left-to-right association.                    */
/* ------------------------------------------------------------------------------------ */

static const double K3 = 0.86602540378;                                        /* :378, :763 */
static const double K5C1 = 0.30901699437, K5C2 = -0.80901699437;               /* :453, :916 */
static const double K5S1 = 0.95105651629, K5S2 = 0.58778525229;
static const double K7C1 = 0.62348980185, K7C2 = -0.22252093395, K7C3 = -0.9009688679; /* :530 */
static const double K7S1 = 0.78183148246, K7S2 = 0.97492791218, K7S3 = 0.43388373911;
static const double K8 = 0.70710678118654752440084436210485;                   /* :623 */

typedef struct { double r, i; } cx;

static void bfly2(cx *x, const cx *prev0)
{
    cx a = prev0 ? *prev0 : x[0]; /* D1: the reference leaf uses its stale output slot */
    cx b = x[1];
    x[0].r = a.r + b.r; x[0].i = a.i + b.i;
    x[1].r = a.r - b.r; x[1].i = a.i - b.i;
}

static void bfly3(cx *x, int sgn)
{
    double sc = sgn * K3;
    cx t0 = {x[1].r + x[2].r, x[1].i + x[2].i};
    cx t1 = {sc * (x[1].r - x[2].r), sc * (x[1].i - x[2].i)};
    cx t2 = {x[0].r - t0.r * 0.5, x[0].i - t0.i * 0.5};
    x[0].r = x[0].r + t0.r; x[0].i = x[0].i + t0.i;
    x[1].r = t2.r + t1.i; x[1].i = t2.i - t1.r;
    x[2].r = t2.r - t1.i; x[2].i = t2.i + t1.r;
}

static void bfly4(cx *x, int sgn)
{
    cx t0 = {x[0].r + x[2].r, x[0].i + x[2].i};
    cx t1 = {x[0].r - x[2].r, x[0].i - x[2].i};
    cx t2 = {x[1].r + x[3].r, x[1].i + x[3].i};
    cx t3 = {sgn * (x[1].r - x[3].r), sgn * (x[1].i - x[3].i)};
    x[0].r = t0.r + t2.r; x[0].i = t0.i + t2.i;
    x[1].r = t1.r + t3.i; x[1].i = t1.i - t3.r;
    x[2].r = t0.r - t2.r; x[2].i = t0.i - t2.i;
    x[3].r = t1.r - t3.i; x[3].i = t1.i + t3.r;
}

static void bfly5(cx *x, int sgn, int leaf)
{
    cx a = x[0];
    cx t0 = {x[1].r + x[4].r, x[1].i + x[4].i};
    cx t1 = {x[2].r + x[3].r, x[2].i + x[3].i};
    cx t2 = {x[1].r - x[4].r, x[1].i - x[4].i};
    cx t3 = {x[2].r - x[3].r, x[2].i - x[3].i};
    cx y[5];
    if (leaf) { /* :515-516 */
        y[0].r = a.r + (t0.r + t1.r); y[0].i = a.i + (t0.i + t1.i);
    } else {    /* :950-951 */
        y[0].r = a.r + t0.r + t1.r; y[0].i = a.i + t0.i + t1.i;
    }
    for (int h = 0; h < 2; h++) {
        double ca = h ? K5C2 : K5C1, cb = h ? K5C1 : K5C2;
        cx t4 = {ca * t0.r + cb * t1.r, ca * t0.i + cb * t1.i}, t5;
        if (h == 0) {
            if (sgn == 1) { t5.r = K5S1 * t2.r + K5S2 * t3.r; t5.i = K5S1 * t2.i + K5S2 * t3.i; }
            else { t5.r = -K5S1 * t2.r - K5S2 * t3.r; t5.i = -K5S1 * t2.i - K5S2 * t3.i; }
        } else {
            if (sgn == 1) { t5.r = K5S2 * t2.r - K5S1 * t3.r; t5.i = K5S2 * t2.i - K5S1 * t3.i; }
            else { t5.r = -K5S2 * t2.r + K5S1 * t3.r; t5.i = -K5S2 * t2.i + K5S1 * t3.i; }
        }
        cx t6 = {a.r + t4.r, a.i + t4.i};
        int lo = 1 + h, hi = 4 - h;
        y[lo].r = t6.r + t5.i; y[lo].i = t6.i - t5.r;
        y[hi].r = t6.r - t5.i; y[hi].i = t6.i + t5.r;
    }
    memcpy(x, y, sizeof y);
}

static void bfly7(cx *x, int sgn, int leaf)
{
    static const double C[3][3] = {{K7C1, K7C2, K7C3}, {K7C2, K7C3, K7C1}, {K7C3, K7C1, K7C2}};
    cx a = x[0];
    cx t0 = {x[1].r + x[6].r, x[1].i + x[6].i}, t3 = {x[1].r - x[6].r, x[1].i - x[6].i};
    cx t1 = {x[2].r + x[5].r, x[2].i + x[5].i}, t4 = {x[2].r - x[5].r, x[2].i - x[5].i};
    cx t2 = {x[3].r + x[4].r, x[3].i + x[4].i}, t5 = {x[3].r - x[4].r, x[3].i - x[4].i};
    cx y[7];
    if (leaf) { /* :608-609 */
        y[0].r = a.r + (t0.r + t1.r + t2.r); y[0].i = a.i + (t0.i + t1.i + t2.i);
    } else {    /* :1132-1133 */
        y[0].r = a.r + t0.r + t1.r + t2.r; y[0].i = a.i + t0.i + t1.i + t2.i;
    }
    for (int h = 0; h < 3; h++) {
        cx t6 = {a.r + C[h][0] * t0.r + C[h][1] * t1.r + C[h][2] * t2.r,
                 a.i + C[h][0] * t0.i + C[h][1] * t1.i + C[h][2] * t2.i};
        cx t7;
        if (h == 0) {
            if (sgn == 1) { t7.r = -K7S1 * t3.r - K7S2 * t4.r - K7S3 * t5.r; t7.i = -K7S1 * t3.i - K7S2 * t4.i - K7S3 * t5.i; }
            else { t7.r = K7S1 * t3.r + K7S2 * t4.r + K7S3 * t5.r; t7.i = K7S1 * t3.i + K7S2 * t4.i + K7S3 * t5.i; }
        } else if (h == 1) {
            if (sgn == 1) { t7.r = -K7S2 * t3.r + K7S3 * t4.r + K7S1 * t5.r; t7.i = -K7S2 * t3.i + K7S3 * t4.i + K7S1 * t5.i; }
            else { t7.r = K7S2 * t3.r - K7S3 * t4.r - K7S1 * t5.r; t7.i = K7S2 * t3.i - K7S3 * t4.i - K7S1 * t5.i; }
        } else {
            if (sgn == 1) { t7.r = -K7S3 * t3.r + K7S1 * t4.r - K7S2 * t5.r; t7.i = -K7S3 * t3.i + K7S1 * t4.i - K7S2 * t5.i; }
            else { t7.r = K7S3 * t3.r - K7S1 * t4.r + K7S2 * t5.r; t7.i = K7S3 * t3.i - K7S1 * t4.i + K7S2 * t5.i; }
        }
        int lo = 1 + h, hi = 6 - h;
        y[lo].r = t6.r - t7.i; y[lo].i = t6.i + t7.r;
        y[hi].r = t6.r + t7.i; y[hi].i = t6.i - t7.r;
    }
    memcpy(x, y, sizeof y);
}

static void bfly8(cx *x, int sgn)
{
    cx t0 = {x[0].r + x[4].r, x[0].i + x[4].i}, t4 = {x[0].r - x[4].r, x[0].i - x[4].i};
    cx t1 = {x[1].r + x[7].r, x[1].i + x[7].i}, t5 = {x[1].r - x[7].r, x[1].i - x[7].i};
    cx t2 = {x[3].r + x[5].r, x[3].i + x[5].i}, t6 = {x[3].r - x[5].r, x[3].i - x[5].i};
    cx t3 = {x[2].r + x[6].r, x[2].i + x[6].i}, t7 = {x[2].r - x[6].r, x[2].i - x[6].i};
    cx y[8], t8, t9;
    y[0].r = t0.r + t1.r + t2.r + t3.r; y[0].i = t0.i + t1.i + t2.i + t3.i;
    y[4].r = t0.r - t1.r - t2.r + t3.r; y[4].i = t0.i - t1.i - t2.i + t3.i;
    cx d1 = {t1.r - t2.r, t1.i - t2.i}, d2 = {t5.r + t6.r, t5.i + t6.i};
    /* outputs 1 / 7 */
    t8.r = t4.r + K8 * d1.r; t8.i = t4.i + K8 * d1.i;
    if (sgn == 1) { t9.r = -K8 * d2.r - t7.r; t9.i = -K8 * d2.i - t7.i; }
    else { t9.r = K8 * d2.r + t7.r; t9.i = K8 * d2.i + t7.i; }
    y[1].r = t8.r - t9.i; y[1].i = t8.i + t9.r; y[7].r = t8.r + t9.i; y[7].i = t8.i - t9.r;
    /* outputs 2 / 6 */
    t8.r = t0.r - t3.r; t8.i = t0.i - t3.i;
    if (sgn == 1) { t9.r = -t5.r + t6.r; t9.i = -t5.i + t6.i; }
    else { t9.r = t5.r - t6.r; t9.i = t5.i - t6.i; }
    y[2].r = t8.r - t9.i; y[2].i = t8.i + t9.r; y[6].r = t8.r + t9.i; y[6].i = t8.i - t9.r;
    /* outputs 3 / 5 */
    t8.r = t4.r - K8 * d1.r; t8.i = t4.i - K8 * d1.i;
    if (sgn == 1) { t9.r = -K8 * d2.r + t7.r; t9.i = -K8 * d2.i + t7.i; }
    else { t9.r = K8 * d2.r - t7.r; t9.i = K8 * d2.i - t7.i; }
    y[3].r = t8.r - t9.i; y[3].i = t8.i + t9.r; y[5].r = t8.r + t9.i; y[5].i = t8.i - t9.r;
    memcpy(x, y, sizeof y);
}

/* odd radix p >= 11 (and any radix without a dedicated kernel), :1475-1628 */
static void bfly_odd(cx *x, int p, int sgn)
{
    int mid = (p - 1) / 2;
    double cs[64], sn[64], tr[64], ti[64];
    for (int i = 1; i <= mid; i++) {
        double s, c;
        sincos(i * ORC_PI2 / p, &s, &c);
        cs[i - 1] = c;
        sn[i - 1] = s;
    }
    for (int i = 0; i < mid; i++) {
        sn[i + mid] = -sn[mid - 1 - i];
        cs[i + mid] = cs[mid - 1 - i];
    }
    for (int i = 0; i < mid; i++) {
        tr[i] = x[i + 1].r + x[p - 1 - i].r;
        ti[i + mid] = x[i + 1].i - x[p - 1 - i].i;
        ti[i] = x[i + 1].i + x[p - 1 - i].i;
        tr[i + mid] = x[i + 1].r - x[p - 1 - i].r;
    }
    cx y[128];
    double ar = x[0].r, ai = x[0].i;
    for (int i = 0; i < mid; i++) { ar += tr[i]; ai += ti[i]; }
    y[0].r = ar; y[0].i = ai;
    for (int u = 0; u < mid; u++) {
        double ur = x[0].r, ui = x[0].i, vr = 0.0, vi = 0.0;
        for (int v = 0; v < mid; v++) {
            int t = ((u + 1) * (v + 1)) % p - 1;
            ur += cs[t] * tr[v];
            ui += cs[t] * ti[v];
            vr -= sn[t] * tr[v + mid];
            vi -= sn[t] * ti[v + mid];
        }
        vr = sgn * vr;
        vi = sgn * vi;
        y[u + 1].r = ur - vi; y[u + 1].i = ui + vr;
        y[p - u - 1].r = ur + vi; y[p - u - 1].i = ui - vr;
    }
    memcpy(x, y, sizeof(cx) * (size_t)p);
}

static int is_leaf(int n) { return n == 2 || n == 3 || n == 4 || n == 5 || n == 7 || n == 8; }

static void leaf_or_combine(cx *x, int r, int sgn, int leaf, const cx *prev0)
{
    switch (r) {
    case 2: bfly2(x, prev0); break;
    case 3: bfly3(x, sgn); break;
    case 4: bfly4(x, sgn); break;
    case 5: bfly5(x, sgn, leaf); break;
    case 7: bfly7(x, sgn, leaf); break;
    case 8: bfly8(x, sgn); break;
    default: bfly_odd(x, r, sgn); break;
    }
}

/* mixed_radix_dit_rec restated, :318-1629.  `conj` mirrors the in-place twiddle negation
 * bluestein_fft applies before its third transform (:1861-1865). */
static void dit(const orc_plan *p, orc_cplx *out, const orc_cplx *in, int sgn, int n, int stride,
                int fi, int conj)
{
    cx x[128];
    if (n == 1) {
        out[0] = in[0];
        return;
    }
    if (is_leaf(n)) {
        cx prev;
        for (int i = 0; i < n; i++) { x[i].r = in[(size_t)i * stride].re; x[i].i = in[(size_t)i * stride].im; }
        const cx *pp = NULL;
        if (n == 2 && (p->flags & ORC_LEAF2_ASIS)) { prev.r = out[0].re; prev.i = out[0].im; pp = &prev; }
        leaf_or_combine(x, n, sgn, 1, pp);
        for (int i = 0; i < n; i++) { out[i].re = x[i].r; out[i].im = x[i].i; }
        return;
    }
    int r = p->fac[fi], L = n / r;
    for (int i = 0; i < r; i++) dit(p, out + (size_t)i * L, in + (size_t)i * stride, sgn, L, stride * r, fi + 1, conj);
    /* radix 4/5/7 skip the twiddles at k == 0 (:826-855, :925-988, :1096-1186) */
    int skip0 = (r == 4 || r == 5 || r == 7);
    const orc_cplx *tw = p->tw + (L - 1);
    for (int k = 0; k < L; k++) {
        x[0].r = out[k].re; x[0].i = out[k].im;
        for (int i = 1; i < r; i++) {
            const orc_cplx *o = &out[k + (size_t)i * L];
            if (skip0 && k == 0) {
                x[i].r = o->re; x[i].i = o->im;
            } else {
                orc_cplx w = tw[(size_t)(r - 1) * k + (i - 1)];
                if (conj) w.im = -w.im;
                x[i].r = o->re * w.re - o->im * w.im;
                x[i].i = o->im * w.re + o->re * w.im;
            }
        }
        leaf_or_combine(x, r, sgn, 0, NULL);
        for (int i = 0; i < r; i++) { out[k + (size_t)i * L].re = x[i].r; out[k + (size_t)i * L].im = x[i].i; }
    }
}

static void exec_mixed(const orc_plan *p, const orc_cplx *in, orc_cplx *out, int sgn, int conj)
{
    dit(p, out, in, sgn, p->M, 1, 0, conj);
}

/* bluestein_fft, :1735-1907 */
static void exec_bluestein(const orc_plan *p, const orc_cplx *in, orc_cplx *out)
{
    int N = p->N, M = p->M, sgn = p->sgn;
    const orc_plan *mp = p->mp;
    const orc_cplx *h = p->hlt;
    orc_cplx *a = calloc((size_t)M, sizeof *a), *hk = calloc((size_t)M, sizeof *hk);
    orc_cplx *yn = calloc((size_t)M, sizeof *yn), *yno = calloc((size_t)M, sizeof *yno);
    /* padded chirp hl (:1692-1703), scaled by 1/M (:1787-1792) */
    double scale = 1.0 / M;
    for (int i = 0; i < M; i++) {
        orc_cplx v = {0.0, 0.0};
        if (i < N) v = h[i];
        else if (i >= M - N + 1) v = h[M - i];
        a[i].im = v.im * scale;
        a[i].re = v.re * scale;
    }
    exec_mixed(mp, a, hk, sgn, 0);
    for (int i = 0; i < M; i++) {
        if (i >= N) { a[i].re = 0.0; a[i].im = 0.0; continue; }
        double xr = in[i].re, xi = in[i].im, hr = h[i].re, hi = h[i].im;
        if (sgn == 1) { a[i].re = xr * hr + xi * hi; a[i].im = -xr * hi + xi * hr; }
        else { a[i].re = xr * hr - xi * hi; a[i].im = xr * hi + xi * hr; }
    }
    exec_mixed(mp, a, yn, sgn, 0);
    for (int i = 0; i < M; i++) {
        double yr = yn[i].re, yi = yn[i].im, kr = hk[i].re, ki = hk[i].im, t;
        if (sgn == 1) { t = yr * kr - yi * ki; yn[i].im = yr * ki + yi * kr; }
        else { t = yr * kr + yi * ki; yn[i].im = -yr * ki + yi * kr; }
        yn[i].re = t;
    }
    exec_mixed(mp, yn, yno, -1 * sgn, 1);
    for (int i = 0; i < N; i++) {
        double yr = yno[i].re, yi = yno[i].im, hr = h[i].re, hi = h[i].im;
        if (sgn == 1) { out[i].re = yr * hr + yi * hi; out[i].im = -yr * hi + yi * hr; }
        else { out[i].re = yr * hr - yi * hi; out[i].im = yr * hi + yi * hr; }
    }
    free(a); free(hk); free(yn); free(yno);
}

void orc_exec(const orc_plan *p, const orc_cplx *in, orc_cplx *out)
{
    if (p->lt) exec_bluestein(p, in, out);
    else exec_mixed(p, in, out, p->sgn, 0);
}

/* ------------------------------------------------------------------------------------ */
/* threaded batch driver (test / baseline convenience; the reference has no batch API)  */
/* ------------------------------------------------------------------------------------ */

struct orc_real_plan {
    orc_plan *c;
    orc_cplx *w2;  /* twiddle2[k] = (cos, sin)(2*pi*k/N), k < N/2 */
    int N;
};

typedef struct {
    const void *plan;
    const void *in;
    void *out;
    int b0, b1, kind;
} orc_job;

static void *orc_worker(void *arg)
{
    orc_job *j = arg;
    if (j->kind == 0) {
        const orc_plan *p = j->plan;
        const orc_cplx *in = j->in;
        orc_cplx *out = j->out;
        for (int b = j->b0; b < j->b1; b++) orc_exec(p, in + (size_t)b * p->N, out + (size_t)b * p->N);
    } else {
        const orc_real_plan *rp = j->plan;
        int N = rp->N;
        const double *in = j->in;
        orc_cplx *out = j->out;
        for (int b = j->b0; b < j->b1; b++) orc_r2c(rp, in + (size_t)b * N, out + (size_t)b * N);
    }
    return NULL;
}

static void orc_run_batch(const void *plan, const void *in, void *out, int batch, int nthreads, int kind)
{
    if (nthreads <= 0) nthreads = 1;
    if (nthreads > batch) nthreads = batch;
    if (nthreads <= 1) {
        orc_job j = {plan, in, out, 0, batch, kind};
        orc_worker(&j);
        return;
    }
    pthread_t th[256];
    orc_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (orc_job){plan, in, out, (int)((long)batch * t / nthreads), (int)((long)batch * (t + 1) / nthreads), kind};
        pthread_create(&th[t], NULL, orc_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void orc_exec_batch(const orc_plan *p, const orc_cplx *in, orc_cplx *out, int batch, int nthreads)
{
    orc_run_batch(p, in, out, batch, nthreads, 0);
}

/* ------------------------------------------------------------------------------------ */
/* digit reversal of the recursion (the index permutation the Stockham passes absorb)    */
/* ------------------------------------------------------------------------------------ */

static void drmap(const orc_plan *p, int *map, int oo, int io, int stride, int n, int fi)
{
    if (n == 1 || is_leaf(n)) {
        for (int i = 0; i < n; i++) map[oo + i] = io + i * stride;
        return;
    }
    int r = p->fac[fi], L = n / r;
    for (int i = 0; i < r; i++) drmap(p, map, oo + i * L, io + i * stride, stride * r, L, fi + 1);
}

void orc_digit_reverse_map(const orc_plan *p, int *map) { drmap(p, map, 0, 0, 1, p->M, 0); }

/* ------------------------------------------------------------------------------------ */
/* real transforms, real.c:26-193                                                        */
/* ------------------------------------------------------------------------------------ */


orc_real_plan *orc_real_create(int N, int sgn, int flags)
{
    if (N <= 0 || N % 2) return NULL;
    orc_real_plan *rp = calloc(1, sizeof *rp);
    rp->N = N;
    rp->c = orc_plan_create(N / 2, sgn, flags);
    rp->w2 = malloc(sizeof(orc_cplx) * (size_t)(N / 2));
    for (int k = 0; k < N / 2; k++) {
        double a = ORC_PI2 * k / N, s, c;
        sincos(a, &s, &c);
        rp->w2[k].re = c;
        rp->w2[k].im = s;
    }
    return rp;
}

void orc_real_destroy(orc_real_plan *rp)
{
    if (!rp) return;
    orc_plan_destroy(rp->c);
    free(rp->w2);
    free(rp);
}

void orc_r2c(const orc_real_plan *rp, const double *in, orc_cplx *out)
{
    int h = rp->N / 2, N = rp->N;
    orc_cplx *z = calloc((size_t)h, sizeof *z);
    orc_exec(rp->c, (const orc_cplx *)in, z); /* packing x[2k], x[2k+1] is a reinterpretation */
    out[0].re = z[0].re + z[0].im;
    out[0].im = 0.0;
    for (int k = 1; k < h; k++) {
        const orc_cplx a = z[k], b = z[h - k], w = rp->w2[k];
        double t1 = a.im + b.im, t2 = b.re - a.re;
        out[k].re = (a.re + b.re + (t1 * w.re) + (t2 * w.im)) / 2.0;
        out[k].im = (a.im - b.im + (t2 * w.re) - (t1 * w.im)) / 2.0;
    }
    out[h].re = z[0].re - z[0].im;
    out[h].im = 0.0;
    for (int k = 1; k < h; k++) { /* Hermitian mirror to all N bins (D8) */
        out[N - k].re = out[k].re;
        out[N - k].im = -out[k].im;
    }
    free(z);
}

void orc_c2r(const orc_real_plan *rp, const orc_cplx *in, double *out)
{
    int h = rp->N / 2;
    orc_cplx *zi = malloc(sizeof(orc_cplx) * (size_t)h), *z = calloc((size_t)h, sizeof *z);
    for (int k = 0; k < h; k++) {
        const orc_cplx a = in[k], b = in[h - k], w = rp->w2[k];
        double t1 = -a.im - b.im, t2 = -b.re + a.re;
        zi[k].re = a.re + b.re + (t1 * w.re) - (t2 * w.im);
        zi[k].im = a.im - b.im + (t2 * w.re) + (t1 * w.im);
    }
    orc_exec(rp->c, zi, z);
    memcpy(out, z, sizeof(orc_cplx) * (size_t)h);
    free(zi);
    free(z);
}

void orc_r2c_batch(const orc_real_plan *rp, const double *in, orc_cplx *out, int batch, int nthreads)
{
    orc_run_batch(rp, in, out, batch, nthreads, 1);
}

/* ------------------------------------------------------------------------------------ */
/* convolution, convolve.c:20-214                                                        */
/* ------------------------------------------------------------------------------------ */

static int orc_next_pow2(int n) { return n <= 0 ? 1 : (int)pow(2, ceil(log2(n))); }

int orc_convolve(const char *type, const char *conv_type, const double *a, int n, const double *b,
                 int m, double *out, int flags)
{
    if (!a || !b || !out || n <= 0 || m <= 0 || !conv_type) return -1;
    int linear = strcmp(conv_type, "linear") == 0, circular = strcmp(conv_type, "circular") == 0;
    if (!linear && !circular) return -1;
    int clen = linear ? n + m - 1 : (n > m ? n : m);
    int P = orc_next_pow2(linear ? clen : (n > m ? n : m));
    orc_real_plan *f = orc_real_create(P, 1, flags), *iv = orc_real_create(P, -1, flags);
    double *pa = calloc((size_t)P, sizeof(double)), *pb = calloc((size_t)P, sizeof(double));
    orc_cplx *A = malloc(sizeof(orc_cplx) * (size_t)P), *B = malloc(sizeof(orc_cplx) * (size_t)P);
    orc_cplx *C = malloc(sizeof(orc_cplx) * (size_t)P);
    double *res = malloc(sizeof(double) * (size_t)P);
    memcpy(pa, a, sizeof(double) * (size_t)n);
    memcpy(pb, b, sizeof(double) * (size_t)m);
    orc_r2c(f, pa, A);
    orc_r2c(f, pb, B);
    for (int i = 0; i < P; i++) {
        C[i].re = A[i].re * B[i].re - A[i].im * B[i].im;
        C[i].im = A[i].re * B[i].im + A[i].im * B[i].re;
    }
    orc_c2r(iv, C, res);
    for (int i = 0; i < P; i++) res[i] /= P;
    int start = 0, len = 0;
    if (linear) {
        /* the reference strcmp()s `type` before its NULL test (D9); NULL means "full" here */
        if (type == NULL || strcmp(type, "full") == 0) { start = 0; len = clen; }
        else if (strcmp(type, "same") == 0) {
            int big = n > m ? n : m;
            start = (clen - big) / 2;
            len = big;
        } else if (strcmp(type, "valid") == 0) {
            int sm = n < m ? n : m, big = n > m ? n : m;
            start = sm - 1;
            len = big - sm + 1;
        } else {
            len = -1;
        }
    } else {
        start = 0;
        len = P;
    }
    if (len > 0) memcpy(out, res + start, sizeof(double) * (size_t)len);
    free(pa); free(pb); free(A); free(B); free(C); free(res);
    orc_real_destroy(f);
    orc_real_destroy(iv);
    return len;
}

/* ------------------------------------------------------------------------------------ */
/* synthetic inputs                                                                      */
/* ------------------------------------------------------------------------------------ */

double orc_uniform(uint64_t seed, uint64_t i)
{
    uint64_t z = (seed ^ i) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 4503599627370496.0) - 1.0; /* 2^-52 -> [0,2) - 1 */
}

void orc_fill_complex(orc_cplx *x, int64_t count, uint64_t seed, uint64_t offset)
{
    for (int64_t j = 0; j < count; j++) {
        uint64_t e = (uint64_t)j + offset;
        x[j].re = orc_uniform(seed, 2 * e);
        x[j].im = orc_uniform(seed, 2 * e + 1);
    }
}

void orc_fill_real(double *x, int64_t count, uint64_t seed, uint64_t offset)
{
    for (int64_t j = 0; j < count; j++) x[j] = orc_uniform(seed, (uint64_t)j + offset);
}
