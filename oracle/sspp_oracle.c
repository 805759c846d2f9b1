/*
 * sspp_oracle.c — CPU restatement of Geryyy/sspp's candidate-scoring path.
 * TEST INFRASTRUCTURE ONLY (see sspp_oracle.h for the contract and citations).
 *
 * Build: oracle/Makefile  (gcc -O2 -fopenmp -ffp-contract=off -mfma).  Every
 * floating-point expression is written out operation by operation (explicit fma()
 * where a fused multiply-add is meant, -ffp-contract=off everywhere else) so that the
 * GPU kernels, which follow the same operation order, can be compared bit for bit.
 */
#include "sspp_oracle.h"
#include "../sspp_amd/csrc/sspp_logtab.h" /* data only: the sampler's ln table */

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_MAXP 8
#define OR_MAXD 16
#define OR_MINVAL 1e-15 /* mjMINVAL */

/* ------------------------------------------------------------------ small math */
static double dot3(const double* a, const double* b) {
    return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]));
}
/* row i of a row-major 3x3 times v */
static void matvec3(const double* m, const double* v, double* r) {
    r[0] = dot3(m + 0, v);
    r[1] = dot3(m + 3, v);
    r[2] = dot3(m + 6, v);
}
static void col3(const double* m, int j, double* c) {
    c[0] = m[j];
    c[1] = m[3 + j];
    c[2] = m[6 + j];
}
/* mju_normalize4 (MuJoCo engine_util_blas.c) */
static void normalize4(double* q) {
    double s = q[0] * q[0];
    s = fma(q[1], q[1], s);
    s = fma(q[2], q[2], s);
    s = fma(q[3], q[3], s);
    double n = sqrt(s);
    if (n < OR_MINVAL) {
        q[0] = 1.0; q[1] = q[2] = q[3] = 0.0;
    } else if (fabs(n - 1.0) > OR_MINVAL) {
        double inv = 1.0 / n;
        q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
    }
}
/* mju_mulQuat */
static void mulquat(const double* a, const double* b, double* r) {
    double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
/* mju_quat2Mat, row-major (without MuJoCo's identity shortcut: the general formula gives
   the same matrix for q = (1,0,0,0), and a single code path keeps the GPU off scratch) */
static void quat2mat(const double* q, double* m) {
    double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
    double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
    double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
    m[0] = q00 + q11 - q22 - q33;
    m[4] = q00 - q11 + q22 - q33;
    m[8] = q00 - q11 - q22 + q33;
    m[1] = 2.0 * (q12 - q03);
    m[2] = 2.0 * (q13 + q02);
    m[3] = 2.0 * (q12 + q03);
    m[5] = 2.0 * (q23 - q01);
    m[6] = 2.0 * (q13 - q02);
    m[7] = 2.0 * (q23 + q01);
}

/* ------------------------------------------------------------------ splines */
void or_knot_averaging(const double* u, int n, int p, double* knots) {
    /* Eigen KnotAveraging: interior knot t_{j+p} = mean(u_j..u_{j+p-1}), j=1..n-p-1 */
    int nk = n + p + 1;
    for (int j = 1; j < n - p; ++j) {
        double s = 0.0;
        for (int r = 0; r < p; ++r) s = s + u[j + r];
        knots[j + p] = s / (double)p;
    }
    for (int i = 0; i <= p; ++i) knots[i] = 0.0;
    for (int i = nk - p - 1; i < nk; ++i) knots[i] = 1.0;
}

int or_span(double u, int p, const double* knots, int nknots) {
    /* Eigen Spline::Span (Piegl & Tiller A2.1 via std::upper_bound) */
    if (u <= knots[0]) return p;
    int lo = p - 1, hi = nknots - p - 1; /* search [lo, hi) */
    int first = lo, count = hi - lo;
    while (count > 0) { /* upper_bound */
        int step = count / 2, it = first + step;
        if (!(u < knots[it])) { first = it + 1; count -= step + 1; }
        else count = step;
    }
    return first - 1;
}

void or_basis(double u, int p, const double* knots, int nknots, double* N) {
    /* Eigen Spline::BasisFunctions (Piegl & Tiller A2.2) */
    int i = or_span(u, p, knots, nknots);
    double left[OR_MAXP + 1], right[OR_MAXP + 1];
    left[0] = 0.0; right[0] = 0.0;
    for (int j = 1; j <= p; ++j) {
        left[j] = u - knots[i + 1 - j];
        right[j] = knots[i + j] - u;
    }
    N[0] = 1.0;
    for (int j = 1; j <= p; ++j) {
        double saved = 0.0;
        for (int r = 0; r < j; ++r) {
            double tmp = N[r] / (right[r + 1] + left[j - r]);
            N[r] = saved + right[r + 1] * tmp;
            saved = left[j - r] * tmp;
        }
        N[j] = saved;
    }
}

void or_spline_eval(const double* knots, int nknots, int p, const double* ctrl, int D, double u,
                    double* out) {
    int span = or_span(u, p, knots, nknots);
    double N[OR_MAXP + 1];
    or_basis(u, p, knots, nknots, N);
    const double* c0 = ctrl + (size_t)(span - p) * D;
    for (int d = 0; d < D; ++d) {
        double acc = N[0] * c0[d];
        for (int r = 1; r <= p; ++r) acc = fma(N[r], c0[(size_t)r * D + d], acc);
        out[d] = acc;
    }
}

/* Householder QR least squares solve A X = B (A n x n row-major, B n x D row-major) */
static int qr_solve(double* A, double* B, int n, int D) {
    double* v = (double*)malloc(sizeof(double) * n);
    if (!v) return -1;
    for (int k = 0; k < n; ++k) {
        double norm = 0.0;
        for (int i = k; i < n; ++i) norm = fma(A[i * n + k], A[i * n + k], norm);
        norm = sqrt(norm);
        if (norm == 0.0) continue;
        double alpha = A[k * n + k] > 0 ? -norm : norm;
        for (int i = k; i < n; ++i) v[i] = A[i * n + k];
        v[k] -= alpha;
        double vn = 0.0;
        for (int i = k; i < n; ++i) vn = fma(v[i], v[i], vn);
        if (vn == 0.0) continue;
        for (int j = k; j < n; ++j) {
            double s = 0.0;
            for (int i = k; i < n; ++i) s = fma(v[i], A[i * n + j], s);
            s = 2.0 * s / vn;
            for (int i = k; i < n; ++i) A[i * n + j] -= s * v[i];
        }
        for (int j = 0; j < D; ++j) {
            double s = 0.0;
            for (int i = k; i < n; ++i) s = fma(v[i], B[i * D + j], s);
            s = 2.0 * s / vn;
            for (int i = k; i < n; ++i) B[i * D + j] -= s * v[i];
        }
    }
    free(v);
    for (int j = 0; j < D; ++j) {
        for (int i = n - 1; i >= 0; --i) {
            double s = B[i * D + j];
            for (int c = i + 1; c < n; ++c) s -= A[i * n + c] * B[c * D + j];
            if (A[i * n + i] == 0.0) return -2;
            B[i * D + j] = s / A[i * n + i];
        }
    }
    return 0;
}

int or_interpolate(const double* pts, int n, int D, int p, const double* u, double* knots,
                   double* ctrl) {
    /* Eigen SplineFitting::Interpolate(pts, degree, knot_parameters) */
    if (n < p + 1 || p > OR_MAXP) return -1;
    int nk = n + p + 1;
    or_knot_averaging(u, n, p, knots);
    double* A = (double*)calloc((size_t)n * n, sizeof(double));
    if (!A) return -1;
    for (int i = 1; i < n - 1; ++i) {
        int span = or_span(u[i], p, knots, nk);
        double N[OR_MAXP + 1];
        or_basis(u[i], p, knots, nk, N);
        for (int r = 0; r <= p; ++r) A[i * n + span - p + r] = N[r];
    }
    A[0] = 1.0;
    A[(n - 1) * n + n - 1] = 1.0;
    memcpy(ctrl, pts, sizeof(double) * (size_t)n * D);
    int rc = qr_solve(A, ctrl, n, D);
    free(A);
    return rc;
}

/* ------------------------------------------------------------------ BSplines.py */
void or_py_knot_vector(int n, int k, double* t) {
    int m = n + 1 - k; /* np.linspace(0, 1, n_knots - 2k) */
    int o = 0;
    for (int i = 0; i < k; ++i) t[o++] = 0.0;
    double step = 1.0 / (double)(m - 1);
    for (int i = 0; i < m; ++i) t[o++] = (i == m - 1) ? 1.0 : (double)i * step + 0.0;
    for (int i = 0; i < k; ++i) t[o++] = 1.0;
}

double or_py_B(double theta, int k, int i, const double* t) {
    if (k == 0) return (t[i] <= theta && theta < t[i + 1]) ? 1.0 : 0.0;
    double c1, c2;
    if (t[i + k] == t[i]) c1 = 0.0;
    else c1 = (theta - t[i]) / (t[i + k] - t[i]) * or_py_B(theta, k - 1, i, t);
    if (t[i + k + 1] == t[i + 1]) c2 = 0.0;
    else c2 = (t[i + k + 1] - theta) / (t[i + k + 1] - t[i + 1]) * or_py_B(theta, k - 1, i + 1, t);
    return c1 + c2;
}

void or_py_bspline(double theta, const double* t, int nt, const double* c, int D, int k,
                   double* out) {
    int n = nt - k - 1;
    if (theta < 0) {
        double b = or_py_B(0.0, k, 0, t);
        for (int d = 0; d < D; ++d) out[d] = c[d] * b;
        return;
    }
    if (theta >= 1) {
        for (int d = 0; d < D; ++d) out[d] = c[(size_t)(n - 1) * D + d];
        return;
    }
    for (int d = 0; d < D; ++d) out[d] = 0.0;
    for (int i = 0; i < n; ++i) {
        double b = or_py_B(theta, k, i, t);
        for (int d = 0; d < D; ++d) out[d] = out[d] + c[(size_t)i * D + d] * b;
    }
}

/* ------------------------------------------------------------------ Philox4x32-10 */
static uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    *hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}
void or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, &hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, &hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void philox_words(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream, uint32_t o[4]) {
    uint32_t ctr[4] = {idx, stream, (uint32_t)cand, (uint32_t)(cand >> 32)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    or_philox4x32_10(ctr, key, o);
}
#define TWO_M53 1.1102230246251565e-16 /* 2^-53 */
#define TWO_PI 6.283185307179586

/* sin(pi x), cos(pi x) for the Box-Muller angle: exact quarter-turn reduction (x*2 and
   x - q/2 are exact for the multiples of 2^-52 used here), then libm on |pi r| <= pi/4.
   Agrees with the device sincospi to ~1 ulp (the samplers' parity bar is 1e-12). */
static void or_sincospi(double x, double* s, double* c) {
    const double q = nearbyint(2.0 * x);
    const double r = x - 0.5 * q;
    const double a = 3.141592653589793 * r;
    const double sa = sin(a), ca = cos(a);
    switch (((long long)q) & 3) {
        case 0: *s = sa; *c = ca; break;
        case 1: *s = ca; *c = -sa; break;
        case 2: *s = -sa; *c = -ca; break;
        default: *s = -ca; *c = sa; break;
    }
}

/* FP64 Box-Muller, the default normals of both planners (reference: std::normal_distribution
   <double>, include/sspp.h:116,125 and include/sspp/tsp_sampler.h:17): the kernels' normal_pair
   (sspp_amd/csrc/sspp_kern.h) operation for operation — ln u1 division-free: k = round(64 m),
   r = RN(64/k) and -ln r = hi + lo from the shared data table (sspp_amd/csrc/sspp_logtab.h,
   generated by tools/gen_log_table.py and checked entry by entry in
   tests/test_oracle_golden.py::test_log_table), t = fma(m, r, -1), ln(1 + t) by its series to
   t^8; sin / cos of 2 pi u2 by Taylor polynomials on |a| <= pi/4 (to a^17 / a^16) after an exact
   quarter-turn reduction; explicit fma, IEEE sqrt — so every normal is bit-identical.
   Accuracy against libm: tests/test_oracle_golden.py::test_normal_pair64_accuracy. */
static const double bm_logtab[64][4] = {SSPP_LOGTAB_ENTRIES};
static double bm_log64(double u) {
    uint64_t bits;
    memcpy(&bits, &u, 8);
    const uint64_t mb = bits & 0x000fffffffffffffull;
    int e = (int)(bits >> 52) - 1023;
    int k = (int)((mb + (1ull << 45)) >> 46);
    const uint64_t mbits = mb | 0x3ff0000000000000ull;
    double m;
    memcpy(&m, &mbits, 8);
    if (k == 64) { k = 0; e += 1; m = m * 0.5; }
    const double t = fma(m, bm_logtab[k][0], -1.0);
    const double t2 = t * t;
    double p = -0.125;
    p = fma(t, p, 0x1.2492492492492p-3);
    p = fma(t, p, -0x1.5555555555555p-3);
    p = fma(t, p, 0x1.999999999999ap-3);
    p = fma(t, p, -0.25);
    p = fma(t, p, 0x1.5555555555555p-2);
    p = fma(t, p, -0.5);
    const double l1 = fma(t2, p, t);
    const double de = (double)e;
    const double hi = fma(de, 0x1.62e42fefa3800p-1, bm_logtab[k][1]);
    const double lo = fma(de, 0x1.ef35793c76730p-45, bm_logtab[k][2]) + l1;
    return hi + lo;
}
static void bm_sincos2pi64(double u, double* sn, double* cs) {
    const double q = rint(4.0 * u);
    const double r = fma(-0.25, q, u);
    const double a = r * 0x1.921fb54442d18p+2;
    const double a2 = a * a;
    double sp = 0x1.952c77030ad4ap-49;
    sp = fma(a2, sp, -0x1.ae7f3e733b81fp-41);
    sp = fma(a2, sp, 0x1.6124613a86d09p-33);
    sp = fma(a2, sp, -0x1.ae64567f544e4p-26);
    sp = fma(a2, sp, 0x1.71de3a556c734p-19);
    sp = fma(a2, sp, -0x1.a01a01a01a01ap-13);
    sp = fma(a2, sp, 0x1.1111111111111p-7);
    sp = fma(a2, sp, -0x1.5555555555555p-3);
    const double sa = fma(a * a2, sp, a);
    double cp = 0x1.ae7f3e733b81fp-45;
    cp = fma(a2, cp, -0x1.93974a8c07c9dp-37);
    cp = fma(a2, cp, 0x1.1eed8eff8d898p-29);
    cp = fma(a2, cp, -0x1.27e4fb7789f5cp-22);
    cp = fma(a2, cp, 0x1.a01a01a01a01ap-16);
    cp = fma(a2, cp, -0x1.6c16c16c16c17p-10);
    cp = fma(a2, cp, 0x1.5555555555555p-5);
    cp = fma(a2, cp, -0x1.0000000000000p-1);
    const double ca = fma(a2, cp, 1.0);
    const int qi = (int)q & 3;
    *sn = qi == 0 ? sa : (qi == 1 ? ca : (qi == 2 ? -sa : -ca));
    *cs = qi == 0 ? ca : (qi == 1 ? -sa : (qi == 2 ? -ca : sa));
}
void or_normal_pair(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream, double* z0,
                    double* z1) {
    uint32_t o[4];
    philox_words(seed, cand, idx, stream, o);
    uint64_t a = (((uint64_t)o[0] << 32) | o[1]) >> 11;
    uint64_t b = (((uint64_t)o[2] << 32) | o[3]) >> 11;
    double u1 = (double)(a + 1) * TWO_M53; /* (0,1] */
    double u2 = (double)b * TWO_M53;       /* [0,1) */
    double r = sqrt(-2.0 * bm_log64(u1));
    double sn, cs;
    bm_sincos2pi64(u2, &sn, &cs);
    *z0 = r * cs;
    *z1 = r * sn;
}
double or_bm_log64_test(double u) { return bm_log64(u); } /* tests: ln u against libm */
/* the libm form of the same transform (log, sin/cos): the accuracy reference of the tests */
void or_normal_pair_libm(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream, double* z0,
                         double* z1) {
    uint32_t o[4];
    philox_words(seed, cand, idx, stream, o);
    uint64_t a = (((uint64_t)o[0] << 32) | o[1]) >> 11;
    uint64_t b = (((uint64_t)o[2] << 32) | o[3]) >> 11;
    double u1 = (double)(a + 1) * TWO_M53;
    double u2 = (double)b * TWO_M53;
    double r = sqrt(-2.0 * log(u1));
    double sn, cs;
    or_sincospi(2.0 * u2, &sn, &cs);
    *z0 = r * cs;
    *z1 = r * sn;
}

/* SamplingPathPlanner normals: the kernels' normal_quad (sspp_amd/csrc/sspp_kernels.hip), the
   same FP32 operations in the same order (explicit fmaf, correctly rounded division and sqrtf,
   round-half-even rintf), so the result is bit-identical: one Philox4x32-10 call -> four
   24-bit uniforms -> two Box-Muller pairs; ln u by the atanh series on the mantissa, sin / cos
   of 2 pi u after an exact quarter-turn reduction. */
static float bm_log(float u) {
    uint32_t bits;
    memcpy(&bits, &u, 4);
    int e = (int)(bits >> 23) - 127;
    uint32_t mb = (bits & 0x7fffffu) | 0x3f800000u;
    float m;
    memcpy(&m, &mb, 4);
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    const float s = (m - 1.0f) / (m + 1.0f);
    const float s2 = s * s;
    float p = fmaf(s2, 0.111111111f, 0.142857143f);
    p = fmaf(s2, p, 0.2f);
    p = fmaf(s2, p, 0.333333333f);
    p = fmaf(s2, p, 1.0f);
    return fmaf((float)e, 0.693147181f, (s + s) * p);
}
static void bm_sincos2pi(float u, float* sn, float* cs) {
    const float q = rintf(4.0f * u);
    const float r = fmaf(-0.25f, q, u);
    const float a = r * 6.28318531f;
    const float a2 = a * a;
    float sp = fmaf(a2, 2.75573192e-6f, -1.98412698e-4f);
    sp = fmaf(a2, sp, 8.33333333e-3f);
    sp = fmaf(a2, sp, -0.166666667f);
    const float sa = fmaf(a * a2, sp, a);
    float cp = fmaf(a2, 2.48015873e-5f, -1.38888889e-3f);
    cp = fmaf(a2, cp, 4.16666667e-2f);
    cp = fmaf(a2, cp, -0.5f);
    const float ca = fmaf(a2, cp, 1.0f);
    const int qi = (int)q & 3;
    *sn = qi == 0 ? sa : (qi == 1 ? ca : (qi == 2 ? -sa : -ca));
    *cs = qi == 0 ? ca : (qi == 1 ? -sa : (qi == 2 ? -ca : sa));
}
void or_normal_quad(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream, double z[4]) {
    uint32_t o[4];
    philox_words(seed, cand, idx, stream, o);
    for (int h = 0; h < 2; ++h) {
        const float u1 = (float)((o[2 * h] >> 8) + 1u) * 5.96046448e-8f;
        const float u2 = (float)(o[2 * h + 1] >> 8) * 5.96046448e-8f;
        const float r = sqrtf(-2.0f * bm_log(u1));
        float sn, cs;
        bm_sincos2pi(u2, &sn, &cs);
        z[2 * h] = (double)(r * cs);
        z[2 * h + 1] = (double)(r * sn);
    }
}

static double uniform01(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream) {
    uint32_t o[4];
    philox_words(seed, cand, idx, stream, o);
    uint64_t b = (((uint64_t)o[2] << 32) | o[3]) >> 11;
    return (double)b * TWO_M53;
}

void or_sample_sspp(const double* init_ctrl, int n, int D, int p, double sigma,
                    const double* limits, uint64_t seed, int64_t first, int64_t B,
                    double* ctrl_out, int sampler) {
    /* include/sspp.h:114-130: ctrl(d, j) += N(0, sigma) * limits(d), j in [p, n-p).  Normal k of
       a candidate: sampler 0 (FP64, default) component k & 1 of Philox pair k >> 1; sampler 1
       (FP32 quads, opt-in) component k & 3 of quad k >> 2. */
    for (int64_t b = 0; b < B; ++b) {
        uint64_t g = (uint64_t)(first + b);
        double* c = ctrl_out + (size_t)b * n * D;
        memcpy(c, init_ctrl, sizeof(double) * (size_t)n * D);
        for (int j = p; j < n - p; ++j) {
            for (int d = 0; d < D; ++d) {
                int k = (j - p) * D + d;
                double z;
                if (sampler == 0) {
                    double z0, z1;
                    or_normal_pair(seed, g, (uint32_t)(k >> 1), 0u, &z0, &z1);
                    z = (k & 1) ? z1 : z0;
                } else {
                    double zq[4];
                    or_normal_quad(seed, g, (uint32_t)(k >> 2), 0u, zq);
                    z = zq[k & 3];
                }
                double noise = (sigma * z) * limits[d];
                c[(size_t)j * D + d] = c[(size_t)j * D + d] + noise;
            }
        }
    }
}

void or_sample_tsp(const double* mean, const double* sigma, int K, const double* lo,
                   const double* hi, double z_min, uint64_t seed, int64_t first, int64_t B,
                   double* vias_out) {
    /* include/sspp/tsp_sampler.h:12-51 */
    for (int64_t b = 0; b < B; ++b) {
        uint64_t g = (uint64_t)(first + b);
        for (int v = 0; v < K; ++v) {
            double* pt = vias_out + ((size_t)b * K + v) * 4;
            const double* m = mean + v * 4;
            const double* s = sigma + v * 4;
            for (int i = 0; i < 3; ++i) {
                double val = 0.0;
                int ok = 0;
                for (int t = 0; t < 99; ++t) {
                    double z0, z1;
                    or_normal_pair(seed, g, (uint32_t)(((v * 4 + i) << 7) | t), 1u, &z0, &z1);
                    val = z0 * s[i];
                    val = val + m[i];
                    if (!(val < lo[i] || val > hi[i])) { ok = 1; break; }
                }
                if (!ok) {
                    double u = uniform01(seed, g, (uint32_t)(((v * 4 + i) << 7) | 127), 1u);
                    val = u * (hi[i] - lo[i]);
                    val = val + lo[i];
                }
                pt[i] = val;
            }
            if (lo[3] != hi[3]) {
                double z0, z1;
                or_normal_pair(seed, g, (uint32_t)((v * 4 + 3) << 7), 1u, &z0, &z1);
                double yaw = z0 * s[3];
                yaw = yaw + m[3];
                double range = hi[3] - lo[3];
                while (yaw < lo[3]) yaw += range;
                while (yaw > hi[3]) yaw -= range;
                pt[3] = yaw;
            } else {
                pt[3] = m[3];
            }
            if (pt[2] < z_min) pt[2] = z_min;
        }
    }
}

/* ------------------------------------------------------------------ scene */
typedef struct { int g1, g2, is_static; double margin; } or_pair;

struct or_scene {
    int mode, arg;
    int nbody, ngeom, nq;
    int32_t *body_parent, *body_jnt_type, *body_qpos_adr, *weld, *moving;
    double *body_pos, *body_quat;
    int32_t *geom_type, *geom_body;
    double *geom_size, *geom_pos, *geom_quat, *geom_margin, *rbound;
    double* qpos0;
    int npair;
    or_pair* pairs;
};

static void* dupmem(const void* p, size_t n) {
    void* r = malloc(n ? n : 1);
    if (r && n) memcpy(r, p, n);
    return r;
}

static double geom_rbound(int type, const double* s) {
    switch (type) {
        case OR_GEOM_BOX: return sqrt(fma(s[2], s[2], fma(s[1], s[1], s[0] * s[0])));
        case OR_GEOM_CYLINDER: return sqrt(fma(s[1], s[1], s[0] * s[0]));
        case OR_GEOM_SPHERE: return s[0];
        case OR_GEOM_CAPSULE: return s[0] + s[1];
        default: return 0.0; /* plane: infinite */
    }
}

or_scene* or_scene_create(const or_model* m, int mode, int arg) {
    or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
    if (!s) return NULL;
    s->mode = mode; s->arg = arg;
    s->nbody = m->nbody; s->ngeom = m->ngeom; s->nq = m->nq;
    size_t nb = (size_t)m->nbody, ng = (size_t)m->ngeom;
    s->body_parent = (int32_t*)dupmem(m->body_parent, nb * 4);
    s->body_jnt_type = (int32_t*)dupmem(m->body_jnt_type, nb * 4);
    s->body_qpos_adr = (int32_t*)dupmem(m->body_qpos_adr, nb * 4);
    s->body_pos = (double*)dupmem(m->body_pos, nb * 24);
    s->body_quat = (double*)dupmem(m->body_quat, nb * 32);
    s->geom_type = (int32_t*)dupmem(m->geom_type, ng * 4);
    s->geom_body = (int32_t*)dupmem(m->geom_body, ng * 4);
    s->geom_size = (double*)dupmem(m->geom_size, ng * 24);
    s->geom_pos = (double*)dupmem(m->geom_pos, ng * 24);
    s->geom_quat = (double*)dupmem(m->geom_quat, ng * 32);
    s->geom_margin = (double*)dupmem(m->geom_margin, ng * 8);
    s->qpos0 = (double*)dupmem(m->qpos0, (size_t)m->nq * 8);
    s->weld = (int32_t*)calloc(nb, 4);
    s->moving = (int32_t*)calloc(nb, 4);
    s->rbound = (double*)calloc(ng ? ng : 1, 8);
    /* weld bodies: a body without joints is welded to its parent (MuJoCo body_weldid) */
    for (int b = 0; b < m->nbody; ++b) {
        if (b == 0) s->weld[b] = 0;
        else if (m->body_jnt_type[b] != OR_JNT_NONE) s->weld[b] = b;
        else s->weld[b] = s->weld[m->body_parent[b]];
    }
    /* moving weld roots */
    for (int b = 1; b < m->nbody; ++b) {
        if (m->body_jnt_type[b] != OR_JNT_FREE) continue;
        if (mode == 0) { if (m->body_qpos_adr[b] < arg) s->moving[b] = 1; }
        else if (b == arg) s->moving[b] = 1;
    }
    for (int g = 0; g < m->ngeom; ++g) s->rbound[g] = geom_rbound(m->geom_type[g], m->geom_size + 3 * g);
    /* pair list in (g1 < g2) order — mj_collision filter */
    s->pairs = (or_pair*)malloc(sizeof(or_pair) * (ng * ng / 2 + 1));
    s->npair = 0;
    for (int g1 = 0; g1 < m->ngeom; ++g1) {
        for (int g2 = g1 + 1; g2 < m->ngeom; ++g2) {
            int b1 = m->geom_body[g1], b2 = m->geom_body[g2];
            int w1 = s->weld[b1], w2 = s->weld[b2];
            if (w1 == w2) continue; /* same weld body (incl. static-static) */
            int ct1 = m->geom_contype[g1], ca1 = m->geom_conaffinity[g1];
            int ct2 = m->geom_contype[g2], ca2 = m->geom_conaffinity[g2];
            if (!((ct1 & ca2) || (ct2 & ca1))) continue;
            if (w1 != 0 && w2 != 0) { /* filterparent */
                if (w1 == s->weld[m->body_parent[w2]] || w2 == s->weld[m->body_parent[w1]]) continue;
            }
            int excl = 0;
            for (int e = 0; e < m->nexclude; ++e) {
                int e1 = m->exclude[2 * e], e2 = m->exclude[2 * e + 1];
                if ((e1 == b1 && e2 == b2) || (e1 == b2 && e2 == b1)) { excl = 1; break; }
            }
            if (excl) continue;
            or_pair pr;
            pr.g1 = g1; pr.g2 = g2;
            pr.is_static = !(s->moving[w1] || s->moving[w2]);
            double m1 = m->geom_margin[g1], m2 = m->geom_margin[g2];
            pr.margin = m1 > m2 ? m1 : m2;
            s->pairs[s->npair++] = pr;
        }
    }
    return s;
}

void or_scene_destroy(or_scene* s) {
    if (!s) return;
    free(s->body_parent); free(s->body_jnt_type); free(s->body_qpos_adr); free(s->weld);
    free(s->moving); free(s->body_pos); free(s->body_quat); free(s->geom_type);
    free(s->geom_body); free(s->geom_size); free(s->geom_pos); free(s->geom_quat);
    free(s->geom_margin); free(s->rbound); free(s->qpos0); free(s->pairs); free(s);
}

int or_scene_npairs(const or_scene* s, int* n_moving, int* n_static) {
    int nm = 0, ns = 0;
    for (int i = 0; i < s->npair; ++i) { if (s->pairs[i].is_static) ns++; else nm++; }
    if (n_moving) *n_moving = nm;
    if (n_static) *n_static = ns;
    return s->npair;
}

/* mj_kinematics restated for free joints + fixed bodies */
static void fk(const or_scene* s, const double* qpos, double* xpos, double* xquat, double* xmat,
               double* gxpos, double* gxmat) {
    xpos[0] = xpos[1] = xpos[2] = 0.0;
    xquat[0] = 1.0; xquat[1] = xquat[2] = xquat[3] = 0.0;
    quat2mat(xquat, xmat);
    for (int b = 1; b < s->nbody; ++b) {
        double* p = xpos + 3 * b;
        double* q = xquat + 4 * b;
        if (s->body_jnt_type[b] == OR_JNT_FREE) {
            const double* qp = qpos + s->body_qpos_adr[b];
            p[0] = qp[0]; p[1] = qp[1]; p[2] = qp[2];
            q[0] = qp[3]; q[1] = qp[4]; q[2] = qp[5]; q[3] = qp[6];
        } else {
            int pa = s->body_parent[b];
            double t[3];
            matvec3(xmat + 9 * pa, s->body_pos + 3 * b, t);
            p[0] = xpos[3 * pa] + t[0];
            p[1] = xpos[3 * pa + 1] + t[1];
            p[2] = xpos[3 * pa + 2] + t[2];
            mulquat(xquat + 4 * pa, s->body_quat + 4 * b, q);
        }
        normalize4(q);
        quat2mat(q, xmat + 9 * b);
    }
    for (int g = 0; g < s->ngeom; ++g) {
        int b = s->geom_body[g];
        double t[3], gq[4];
        matvec3(xmat + 9 * b, s->geom_pos + 3 * g, t);
        gxpos[3 * g] = xpos[3 * b] + t[0];
        gxpos[3 * g + 1] = xpos[3 * b + 1] + t[1];
        gxpos[3 * g + 2] = xpos[3 * b + 2] + t[2];
        mulquat(xquat + 4 * b, s->geom_quat + 4 * g, gq);
        normalize4(gq);
        quat2mat(gq, gxmat + 9 * g);
    }
}

static void set_qpos(const or_scene* s, const double* q, double* qpos) {
    memcpy(qpos, s->qpos0, sizeof(double) * (size_t)s->nq);
    if (s->mode == 0) {
        for (int i = 0; i < s->arg && i < s->nq; ++i) qpos[i] = q[i];
    } else {
        /* Utility::mj_set_point + yaw_to_quat (include/utility.h:149-206) */
        int adr = s->body_qpos_adr[s->arg];
        double half = q[3] * 0.5;
        qpos[adr] = q[0]; qpos[adr + 1] = q[1]; qpos[adr + 2] = q[2];
        qpos[adr + 3] = cos(half); qpos[adr + 4] = 0.0; qpos[adr + 5] = 0.0; qpos[adr + 6] = sin(half);
    }
}

void or_fk_geoms(const or_scene* s, const double* q, double* gxpos, double* gxmat) {
    double* qpos = (double*)malloc(sizeof(double) * (size_t)(s->nq ? s->nq : 1));
    double* xpos = (double*)malloc(sizeof(double) * 3 * s->nbody);
    double* xquat = (double*)malloc(sizeof(double) * 4 * s->nbody);
    double* xmat = (double*)malloc(sizeof(double) * 9 * s->nbody);
    set_qpos(s, q, qpos);
    fk(s, qpos, xpos, xquat, xmat, gxpos, gxmat);
    free(qpos); free(xpos); free(xquat); free(xmat);
}

/* ------------------------------------------------------------------ narrowphase
 * Each function returns the number of contacts (dist < margin) and, in *ndeep,
 * how many of them have dist < -1e-3 (include/Collision.h:93).                */
#define DEEP (-1e-3)

static int col_plane_box(const double* pp, const double* pm, const double* bp, const double* bm,
                         const double* e, double margin, int* ndeep) {
    double n[3], d[3], ax[3], a[3];
    col3(pm, 2, n);
    d[0] = bp[0] - pp[0]; d[1] = bp[1] - pp[1]; d[2] = bp[2] - pp[2];
    double d0 = dot3(d, n);
    for (int j = 0; j < 3; ++j) { col3(bm, j, ax); a[j] = dot3(n, ax) * e[j]; }
    int nc = 0, nd = 0;
    for (int k = 0; k < 8; ++k) {
        double l = (k & 1) ? a[0] : -a[0];  // corner height over the box centre (MuJoCo's ldist)
        l = l + ((k & 2) ? a[1] : -a[1]);
        l = l + ((k & 4) ? a[2] : -a[2]);
        const double t = d0 + l;
        // mjc_PlaneBox: a corner counts unless dist + ldist > margin or ldist > 0 (the corners
        // of the half turned away from the plane never count), at most 4
        if (!(t > margin) && !(l > 0.0) && nc < 4) { nc++; if (t < DEEP) nd++; }
    }
    *ndeep = nd;
    return nc;
}

static int col_plane_sphere(const double* pp, const double* pm, const double* sp, double r,
                            double margin, int* ndeep) {
    double n[3], d[3];
    col3(pm, 2, n);
    d[0] = sp[0] - pp[0]; d[1] = sp[1] - pp[1]; d[2] = sp[2] - pp[2];
    double dist = dot3(d, n) - r;
    *ndeep = dist < DEEP;
    return dist <= margin;  // mjc_PlaneSphere: no contact only when dist > margin
}

static int col_plane_cyl(const double* pp, const double* pm, const double* cp, const double* cm,
                         const double* sz, double margin, int* ndeep) {
    // mjc_PlaneCylinder: the deepest rim point of the cap nearer the plane (p1) decides whether
    // there is any contact (dist <= margin); then the matching rim point of the far cap (p2) and
    // two "triangle" points on the near cap at +-120 degrees from p1 (pt, height -prjvec / 2),
    // each counted when within the margin: up to 4 contacts
    double n[3], a[3], d[3];
    col3(pm, 2, n);
    col3(cm, 2, a);
    d[0] = cp[0] - pp[0]; d[1] = cp[1] - pp[1]; d[2] = cp[2] - pp[2];
    const double dn = dot3(d, n), na = dot3(n, a);
    const double s = 1.0 - na * na;
    const double rim = sz[0] * sqrt(s > 0.0 ? s : 0.0);
    const double ha = sz[1] * fabs(na);
    const double nearc = dn - ha;
    const double p1 = nearc - rim, p2 = (dn + ha) - rim, pt = nearc + 0.5 * rim;
    if (p1 > margin) { *ndeep = 0; return 0; }
    *ndeep = (p1 < DEEP) + (p2 < DEEP) + 2 * (pt < DEEP);
    return 1 + (p2 <= margin) + 2 * (pt <= margin);
}

static int col_sphere_sphere(const double* p1, double r1, const double* p2, double r2,
                             double margin, int* ndeep) {
    double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    double dist = sqrt(dot3(d, d)) - (r1 + r2);
    *ndeep = dist < DEEP;
    return dist <= margin;  // MuJoCo: no contact only when dist > margin
}

static int col_sphere_box(const double* sp, double r, const double* bp, const double* bm,
                          const double* e, double margin, int* ndeep) {
    double d[3] = {sp[0] - bp[0], sp[1] - bp[1], sp[2] - bp[2]}, ax[3], l[3];
    int inside = 1;
    double mind = 1e300, out2 = 0.0;
    for (int j = 0; j < 3; ++j) {
        col3(bm, j, ax);
        l[j] = dot3(ax, d);
        double al = fabs(l[j]);
        if (al > e[j]) { inside = 0; double o = al - e[j]; out2 = fma(o, o, out2); }
        double f = e[j] - al;
        if (f < mind) mind = f;
    }
    double dist = inside ? (-mind - r) : (sqrt(out2) - r);
    *ndeep = dist < DEEP;
    return dist <= margin;  // MuJoCo: no contact only when dist > margin
}

static int col_sphere_cyl(const double* sp, double r, const double* cp, const double* cm,
                          const double* sz, double margin, int* ndeep) {
    double d[3] = {sp[0] - cp[0], sp[1] - cp[1], sp[2] - cp[2]}, a[3];
    col3(cm, 2, a);
    double z = dot3(a, d);
    double rr = dot3(d, d) - z * z;
    double rho = sqrt(rr > 0.0 ? rr : 0.0);
    double dz = fabs(z) - sz[1], dr = rho - sz[0];
    double dist;
    if (dz <= 0.0 && dr <= 0.0) dist = (dz > dr ? dz : dr) - r;
    else {
        double oz = dz > 0.0 ? dz : 0.0, orr = dr > 0.0 ? dr : 0.0;
        dist = sqrt(fma(orr, orr, oz * oz)) - r;
    }
    *ndeep = dist < DEEP;
    return dist <= margin;  // MuJoCo: no contact only when dist > margin
}

/* Separating-axis test for two boxes: dist = max over the 15 axes of the signed
 * separation; the pair is "in contact" when dist < margin and "deep" when dist < -1e-3.
 * Early exit as soon as one axis reaches thr (exact: only the booleans are used).   */
static int sat_box_box(const double* pa, const double* ma, const double* ea, const double* pb,
                       const double* mb, const double* eb, double thr) {
    double A[3][3], Bc[3][3], T[3], t[3], R[3][3], AR[3][3];
    for (int j = 0; j < 3; ++j) { col3(ma, j, A[j]); col3(mb, j, Bc[j]); }
    T[0] = pb[0] - pa[0]; T[1] = pb[1] - pa[1]; T[2] = pb[2] - pa[2];
    for (int i = 0; i < 3; ++i) {
        t[i] = dot3(A[i], T);
        for (int j = 0; j < 3; ++j) { R[i][j] = dot3(A[i], Bc[j]); AR[i][j] = fabs(R[i][j]); }
    }
    for (int i = 0; i < 3; ++i) { /* faces of A */
        double rb = fma(eb[2], AR[i][2], fma(eb[1], AR[i][1], eb[0] * AR[i][0]));
        double sep = fabs(t[i]) - (ea[i] + rb);
        if (sep >= thr) return 0;
    }
    for (int j = 0; j < 3; ++j) { /* faces of B */
        double pr = fabs(fma(t[2], R[2][j], fma(t[1], R[1][j], t[0] * R[0][j])));
        double ra = fma(ea[2], AR[2][j], fma(ea[1], AR[1][j], ea[0] * AR[0][j]));
        double sep = pr - (ra + eb[j]);
        if (sep >= thr) return 0;
    }
    for (int i = 0; i < 3; ++i) { /* edge x edge */
        for (int j = 0; j < 3; ++j) {
            double v[3] = {R[0][j], R[1][j], R[2][j]}, L[3];
            if (i == 0) { L[0] = 0.0; L[1] = -v[2]; L[2] = v[1]; }
            else if (i == 1) { L[0] = v[2]; L[1] = 0.0; L[2] = -v[0]; }
            else { L[0] = -v[1]; L[1] = v[0]; L[2] = 0.0; }
            double len2 = dot3(L, L);
            if (len2 < 1e-12) continue;
            double pr = fabs(dot3(t, L));
            double ra = fma(ea[2], fabs(L[2]), fma(ea[1], fabs(L[1]), ea[0] * fabs(L[0])));
            double rb = 0.0;
            for (int k = 0; k < 3; ++k) {
                double bk[3] = {R[0][k], R[1][k], R[2][k]};
                rb = fma(eb[k], fabs(dot3(bk, L)), rb);
            }
            /* separation along the unit axis L/|L| >= thr, without the division */
            double num = pr - (ra + rb);
            if (num >= thr * sqrt(len2)) return 0;
        }
    }
    return 1;
}

/* Box-box deep contacts for the TaskSpacePlanner cost (include/Collision.h:89-101 adds one
 * term per MuJoCo contact with dist < -1e-3; MuJoCo's box-box collider reports up to 8).  One
 * pass: the 15-axis SAT at thr = -1e-3 exactly as sat_box_box (0 = not deep); then an edge-edge
 * axis separating by more than every face axis + 1e-12 gives one contact; else the face axis of
 * least penetration is the reference face, the most anti-parallel face of the other box the
 * incident face, and the contacts are the vertices of the incident face clipped to the
 * reference rectangle, dist = -(depth below the reference face): each incident edge clipped by
 * Liang-Barsky (one reciprocal per direction, boundary inclusive) gives its entry point and, if
 * it leaves early, its exit point; reference corners strictly inside the incident face are
 * vertices too.  Returns the count with dist < -1e-3, at least 1.  DESIGN.md §4.             */
static int box_box_deep_count(const double* pa, const double* ma, const double* ea,
                              const double* pb, const double* mb, const double* eb) {
    double A[3][3], Bc[3][3], T[3], t[3], R[3][3], AR[3][3];
    for (int j = 0; j < 3; ++j) { col3(ma, j, A[j]); col3(mb, j, Bc[j]); }
    T[0] = pb[0] - pa[0]; T[1] = pb[1] - pa[1]; T[2] = pb[2] - pa[2];
    for (int i = 0; i < 3; ++i) {
        t[i] = dot3(A[i], T);
        for (int j = 0; j < 3; ++j) { R[i][j] = dot3(A[i], Bc[j]); AR[i][j] = fabs(R[i][j]); }
    }
    double best_face = -1e300;
    int fi = 0;
    for (int i = 0; i < 3; ++i) {
        double rb = fma(eb[2], AR[i][2], fma(eb[1], AR[i][1], eb[0] * AR[i][0]));
        double sep = fabs(t[i]) - (ea[i] + rb);
        if (sep >= DEEP) return 0;
        if (sep > best_face) { best_face = sep; fi = i; }
    }
    for (int j = 0; j < 3; ++j) {
        double pr = fabs(fma(t[2], R[2][j], fma(t[1], R[1][j], t[0] * R[0][j])));
        double ra = fma(ea[2], AR[2][j], fma(ea[1], AR[1][j], ea[0] * AR[0][j]));
        double sep = pr - (ra + eb[j]);
        if (sep >= DEEP) return 0;
        if (sep > best_face) { best_face = sep; fi = 3 + j; }
    }
    int edge = 0;
    double fthr = best_face + 1e-12;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) {
            double v[3] = {R[0][j], R[1][j], R[2][j]}, L[3];
            if (i == 0) { L[0] = 0.0; L[1] = -v[2]; L[2] = v[1]; }
            else if (i == 1) { L[0] = v[2]; L[1] = 0.0; L[2] = -v[0]; }
            else { L[0] = -v[1]; L[1] = v[0]; L[2] = 0.0; }
            double len2 = dot3(L, L);
            if (len2 < 1e-12) continue;
            double pr = fabs(dot3(t, L));
            double ra = fma(ea[2], fabs(L[2]), fma(ea[1], fabs(L[1]), ea[0] * fabs(L[0])));
            double rb = 0.0;
            for (int k = 0; k < 3; ++k) {
                double bk[3] = {R[0][k], R[1][k], R[2][k]};
                rb = fma(eb[k], fabs(dot3(bk, L)), rb);
            }
            double num = pr - (ra + rb), len = sqrt(len2);
            if (num >= DEEP * len) return 0;
            edge = edge || num > fthr * len;
        }
    }
    if (edge) return 1;
    int refA = fi < 3, f = refA ? fi : fi - 3;
    const double *pR = refA ? pa : pb, *pI = refA ? pb : pa;
    const double *eR = refA ? ea : eb, *eI = refA ? eb : ea;
    double RA[3][3], IA[3][3];
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) { RA[j][i] = refA ? A[j][i] : Bc[j][i]; IA[j][i] = refA ? Bc[j][i] : A[j][i]; }
    double n[3] = {RA[f][0], RA[f][1], RA[f][2]};
    double dRI[3] = {pI[0] - pR[0], pI[1] - pR[1], pI[2] - pR[2]};
    if (dot3(dRI, n) < 0.0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    int k = 0;
    double kb = fabs(dot3(IA[0], n));
    { double v = fabs(dot3(IA[1], n)); if (v > kb) { kb = v; k = 1; } }
    { double v = fabs(dot3(IA[2], n)); if (v > kb) { kb = v; k = 2; } }
    double sg = dot3(IA[k], n) > 0.0 ? -eI[k] : eI[k];
    int k1 = k == 2 ? 0 : k + 1, k2 = k == 0 ? 2 : k - 1;
    int ta = f == 2 ? 0 : f + 1, tb = f == 0 ? 2 : f - 1;
    double off = dot3(pR, n) + eR[f];
    double cu[4], cv[4], cd[4];
    for (int v = 0; v < 4; ++v) {
        double c1 = (v == 0 || v == 3) ? eI[k1] : -eI[k1];
        double c2 = (v < 2) ? eI[k2] : -eI[k2];
        double P[3], dp[3];
        for (int i = 0; i < 3; ++i) {
            P[i] = fma(c2, IA[k2][i], fma(c1, IA[k1][i], fma(sg, IA[k][i], pI[i])));
            dp[i] = P[i] - pR[i];
        }
        cu[v] = dot3(dp, RA[ta]);
        cv[v] = dot3(dp, RA[tb]);
        cd[v] = off - dot3(P, n);
    }
    double eu = eR[ta], ev = eR[tb];
    int nd = 0;
    for (int e = 0; e < 4; ++e) {
        int e2 = (e + 1) & 3;
        double du = cu[e2] - cu[e], dv = cv[e2] - cv[e];
        double t0 = 0.0, t1 = 1.0;
        int ok = 1;
        if (du == 0.0) {
            ok = ok && !(cu[e] + eu < 0.0) && !(eu - cu[e] < 0.0);
        } else {
            double r = 1.0 / du;
            double a0 = -(cu[e] + eu) * r, a1 = (eu - cu[e]) * r;
            double lo = du > 0.0 ? a0 : a1, hi = du > 0.0 ? a1 : a0;
            if (lo > t0) t0 = lo;
            if (hi < t1) t1 = hi;
        }
        if (dv == 0.0) {
            ok = ok && !(cv[e] + ev < 0.0) && !(ev - cv[e] < 0.0);
        } else {
            double r = 1.0 / dv;
            double b0 = -(cv[e] + ev) * r, b1 = (ev - cv[e]) * r;
            double lo = dv > 0.0 ? b0 : b1, hi = dv > 0.0 ? b1 : b0;
            if (lo > t0) t0 = lo;
            if (hi < t1) t1 = hi;
        }
        if (ok && t0 <= t1) {
            double dd = cd[e2] - cd[e];
            if (-fma(t0, dd, cd[e]) < DEEP) ++nd;
            if (t1 < 1.0 && -fma(t1, dd, cd[e]) < DEEP) ++nd;
        }
    }
    double au = cu[1] - cu[0], av = cv[1] - cv[0], bu = cu[3] - cu[0], bv = cv[3] - cv[0];
    double idet = 1.0 / (au * bv - av * bu);
    for (int q = 0; q < 4; ++q) {
        double qu = (q & 1) ? eu : -eu, qv = (q & 2) ? ev : -ev;
        double wu = qu - cu[0], wv = qv - cv[0];
        double al = (wu * bv - wv * bu) * idet, be = (au * wv - av * wu) * idet;
        if (al > 0.0 && al < 1.0 && be > 0.0 && be < 1.0) {
            double d = fma(be, cd[3] - cd[0], fma(al, cd[1] - cd[0], cd[0]));
            if (-d < DEEP) ++nd;
        }
    }
    return nd > 0 ? nd : 1;
}

/* ---------------------------------------------------------------- cylinder-box, exact
 * The signed distance of two convex bodies is the maximum over directions n of their
 * separation along n (negative: minus the penetration depth), attained at the normal of the
 * closest feature pair.  Candidate families (cylinder cap / lateral surface / rim circles vs
 * box faces / edges / vertices), DESIGN.md §4:
 *   (a) box face normals  (b) cylinder axis a  (c) a x b_k
 *   (d) perp_a(w - c) per box vertex w     (f) w - (nearest rim point), both rims
 *   (e) rim vs box edge: normal of the rim projected along the edge (an ellipse) at its point
 *       nearest the projected edge (Eberly's bisection); for a depth also the other locally
 *       nearest ellipse point.
 * Any direction bounds the signed distance from below, so "dist < thr" holds exactly when no
 * candidate separates by >= thr.                                                          */
typedef struct {
    double a[3], T[3], B[3][3], e[3], R, H;
} or_cylbox;

static or_cylbox make_cylbox(const double* pa, const double* ma, const double* sz, const double* pb,
                             const double* mb, const double* eb) {
    or_cylbox c;
    col3(ma, 2, c.a);
    for (int j = 0; j < 3; ++j) { col3(mb, j, c.B[j]); c.e[j] = eb[j]; }
    c.T[0] = pb[0] - pa[0]; c.T[1] = pb[1] - pa[1]; c.T[2] = pb[2] - pa[2];
    c.R = sz[0]; c.H = sz[1];
    return c;
}

static int cb_sep(const or_cylbox* c, const double* L, double thr) {
    double len2 = dot3(L, L);
    if (!(len2 > 1e-30)) return 0;
    double aL = dot3(c->a, L);
    double rr = len2 - aL * aL;
    double rc = fma(c->H, fabs(aL), c->R * sqrt(rr > 0.0 ? rr : 0.0));
    double rb = 0.0;
    for (int k = 0; k < 3; ++k) rb = fma(c->e[k], fabs(dot3(c->B[k], L)), rb);
    double num = fabs(dot3(c->T, L)) - (rc + rb);
    return thr == 0.0 ? num >= 0.0 : num >= thr * sqrt(len2);
}

static int cb_base_sep(const or_cylbox* c, double thr) {
    for (int ax = 0; ax < 7; ++ax) {
        double L[3];
        if (ax < 3) { L[0] = c->B[ax][0]; L[1] = c->B[ax][1]; L[2] = c->B[ax][2]; }
        else if (ax == 3) { L[0] = c->a[0]; L[1] = c->a[1]; L[2] = c->a[2]; }
        else {
            const double* b = c->B[ax - 4];
            L[0] = c->a[1] * b[2] - c->a[2] * b[1];
            L[1] = c->a[2] * b[0] - c->a[0] * b[2];
            L[2] = c->a[0] * b[1] - c->a[1] * b[0];
            if (dot3(L, L) < 1e-20) continue;
        }
        if (cb_sep(c, L, thr)) return 1;
    }
    return 0;
}

static double ell_F(double r0, double z0, double z1, double s) {
    double t0 = (r0 * z0) / (s + r0), t1 = z1 / (s + 1.0);
    return fma(t1, t1, t0 * t0) - 1.0;
}
/* root of F on (lo, hi), sign(F(lo)) = sgn_lo, F convex + monotone: safeguarded Newton */
static double ell_bisect(double r0, double z0, double z1, double lo, double hi, double sgn_lo) {
    double n0 = r0 * z0;
    double s = 0.5 * (lo + hi);
    for (int i = 0; i < 48; ++i) {
        double a0 = s + r0, a1 = s + 1.0;
        double t0 = n0 / a0, t1 = z1 / a1;
        double f = fma(t1, t1, t0 * t0) - 1.0;
        if (f == 0.0) break;
        if ((f > 0.0) == (sgn_lo > 0.0)) lo = s; else hi = s;
        double fp = -2.0 * ((t0 * t0) / a0 + (t1 * t1) / a1);
        double sn = s - f / fp;
        if (!(sn > lo && sn < hi)) sn = 0.5 * (lo + hi);
        if (sn == s) break;
        s = sn;
    }
    return s;
}
/* Eberly, "Distance from a point to an ellipse" (2013): nearest point, first quadrant */
static void ellipse_q1(double e0, double e1, double y0, double y1, double* x0, double* x1) {
    if (y1 > 0.0) {
        if (y0 > 0.0) {
            double z0 = y0 / e0, z1 = y1 / e1;
            double g = fma(z1, z1, z0 * z0) - 1.0;
            if (g != 0.0) {
                double q = e0 / e1, r0 = q * q, n0 = r0 * z0;
                double hi = g < 0.0 ? 0.0 : sqrt(fma(z1, z1, n0 * n0)) - 1.0;
                double s = ell_bisect(r0, z0, z1, z1 - 1.0, hi, 1.0);
                *x0 = (r0 * y0) / (s + r0);
                *x1 = y1 / (s + 1.0);
            } else {
                *x0 = y0; *x1 = y1;
            }
        } else {
            *x0 = 0.0; *x1 = e1;
        }
    } else {
        double num = e0 * y0, den = e0 * e0 - e1 * e1;
        if (num < den) {
            double xd = num / den;
            *x0 = e0 * xd;
            *x1 = e1 * sqrt(1.0 - xd * xd);
        } else {
            *x0 = e0; *x1 = 0.0;
        }
    }
}
static int cb_ell_axis(const or_cylbox* c, const double* u1, const double* u2, double x, double y,
                       double e0, double e1, double thr) {
    double nx = x / (e0 * e0), ny = y / (e1 * e1);
    double L[3] = {fma(ny, u2[0], nx * u1[0]), fma(ny, u2[1], nx * u1[1]), fma(ny, u2[2], nx * u1[2])};
    return cb_sep(c, L, thr);
}
static int cb_ell_other(const or_cylbox* c, const double* u1, const double* u2, double px, double py,
                        double e0, double e1, double thr) {
    double y0 = fabs(px), y1 = fabs(py), sx = px < 0.0 ? -1.0 : 1.0, sy = py < 0.0 ? -1.0 : 1.0;
    double den = e0 * e0 - e1 * e1;
    if (y1 == 0.0) {
        if (cb_ell_axis(c, u1, u2, e0, 0.0, e0, e1, thr)) return 1;
        if (e0 * y0 < den) {
            double xd = (e0 * y0) / den, x0 = sx * e0 * xd, x1 = e1 * sqrt(1.0 - xd * xd);
            if (cb_ell_axis(c, u1, u2, x0, x1, e0, e1, thr) || cb_ell_axis(c, u1, u2, x0, -x1, e0, e1, thr))
                return 1;
        }
        return 0;
    }
    if (y0 == 0.0) {
        if (cb_ell_axis(c, u1, u2, 0.0, e1, e0, e1, thr)) return 1;
        if (e1 * y1 < den) {
            double x1 = -sy * (e1 * e1 * y1) / den, t = x1 / e1;
            double x0 = e0 * sqrt(1.0 - t * t);
            if (cb_ell_axis(c, u1, u2, x0, x1, e0, e1, thr) || cb_ell_axis(c, u1, u2, -x0, x1, e0, e1, thr))
                return 1;
        }
        return 0;
    }
    double z0 = y0 / e0, z1 = y1 / e1, q = e0 / e1, r0 = q * q, n0 = r0 * z0;
    double lo = -r0, hi = -1.0, s = 0.5 * (lo + hi);
    for (int i = 0; i < 48; ++i) {
        double a0 = s + r0, a1 = s + 1.0;
        double q0 = (n0 * n0) / (a0 * a0 * a0), q1 = (z1 * z1) / (a1 * a1 * a1);
        double D = q0 + q1;
        if (D == 0.0) break;
        if (D > 0.0) lo = s; else hi = s;
        double Dp = -3.0 * (q0 / a0 + q1 / a1);
        double sn = s - D / Dp;
        if (!(sn > lo && sn < hi)) sn = 0.5 * (lo + hi);
        if (sn == s) break;
        s = sn;
    }
    if (!(ell_F(r0, z0, z1, s) < 0.0)) return 0;
    double ss[2];
    ss[0] = ell_bisect(r0, z0, z1, -r0, s, 1.0);
    ss[1] = ell_bisect(r0, z0, z1, s, -1.0, -1.0);
    for (int k = 0; k < 2; ++k) {
        double x0 = sx * ((r0 * y0) / (ss[k] + r0)), x1 = sy * (y1 / (ss[k] + 1.0));
        if (cb_ell_axis(c, u1, u2, x0, x1, e0, e1, thr)) return 1;
    }
    return 0;
}

static int cb_ext_sep(const or_cylbox* c, double thr, int all_roots) {
    for (int v = 0; v < 8; ++v) {
        double s0 = (v & 1) ? c->e[0] : -c->e[0], s1 = (v & 2) ? c->e[1] : -c->e[1],
               s2 = (v & 4) ? c->e[2] : -c->e[2];
        double w[3], u[3];
        for (int i = 0; i < 3; ++i) w[i] = fma(s2, c->B[2][i], fma(s1, c->B[1][i], fma(s0, c->B[0][i], c->T[i])));
        double z = dot3(c->a, w);
        for (int i = 0; i < 3; ++i) u[i] = w[i] - z * c->a[i];
        double uu = dot3(u, u);
        if (!(uu > 1e-30)) continue;
        if (cb_sep(c, u, thr)) return 1;
        double f = 1.0 - c->R / sqrt(uu);
        for (int r = 0; r < 2; ++r) {
            double dz = z - (r ? c->H : -c->H);
            double L[3] = {fma(dz, c->a[0], f * u[0]), fma(dz, c->a[1], f * u[1]), fma(dz, c->a[2], f * u[2])};
            if (cb_sep(c, L, thr)) return 1;
        }
    }
    for (int j = 0; j < 3; ++j) {
        const double* e = c->B[j];
        double u1[3] = {c->a[1] * e[2] - c->a[2] * e[1], c->a[2] * e[0] - c->a[0] * e[2], c->a[0] * e[1] - c->a[1] * e[0]};
        double S2 = dot3(u1, u1);
        if (S2 < 1e-20) continue;
        double iS = 1.0 / sqrt(S2);
        u1[0] *= iS; u1[1] *= iS; u1[2] *= iS;
        double u2[3] = {e[1] * u1[2] - e[2] * u1[1], e[2] * u1[0] - e[0] * u1[2], e[0] * u1[1] - e[1] * u1[0]};
        double e0 = c->R, e1 = c->R * fabs(dot3(c->a, e));
        int k1 = j == 2 ? 0 : j + 1, k2 = j == 0 ? 2 : j - 1;
        for (int q = 0; q < 4; ++q) {
            double s1 = (q & 1) ? c->e[k1] : -c->e[k1], s2 = (q & 2) ? c->e[k2] : -c->e[k2];
            double w0[3];
            for (int i = 0; i < 3; ++i) w0[i] = fma(s2, c->B[k2][i], fma(s1, c->B[k1][i], c->T[i]));
            for (int r = 0; r < 2; ++r) {
                double hs = r ? c->H : -c->H;
                double d[3] = {w0[0] - hs * c->a[0], w0[1] - hs * c->a[1], w0[2] - hs * c->a[2]};
                double px = dot3(d, u1), py = dot3(d, u2);
                if (e1 < 1e-9 * e0) {
                    if (fabs(px) <= e0) continue;
                    double ex = px - (px < 0.0 ? -e0 : e0);
                    double L[3] = {fma(py, u2[0], ex * u1[0]), fma(py, u2[1], ex * u1[1]), fma(py, u2[2], ex * u1[2])};
                    if (cb_sep(c, L, thr)) return 1;
                    continue;
                }
                double x0, x1;
                ellipse_q1(e0, e1, fabs(px), fabs(py), &x0, &x1);
                if (cb_ell_axis(c, u1, u2, px < 0.0 ? -x0 : x0, py < 0.0 ? -x1 : x1, e0, e1, thr)) return 1;
                if (all_roots && cb_ell_other(c, u1, u2, px, py, e0, e1, thr)) return 1;
            }
        }
    }
    return 0;
}

/* Witnesses: they only prove overlap (a separation needs the candidate directions). */
static int cb_proj_box(const or_cylbox* c, const double* e, const double* x, double* y) {
    double d[3] = {x[0] - c->T[0], x[1] - c->T[1], x[2] - c->T[2]}, l[3];
    int in = 1;
    for (int k = 0; k < 3; ++k) {
        double t = dot3(c->B[k], d);
        if (!(t < e[k] && t > -e[k])) in = 0;
        l[k] = t > e[k] ? e[k] : (t < -e[k] ? -e[k] : t);
    }
    for (int i = 0; i < 3; ++i) y[i] = fma(l[2], c->B[2][i], fma(l[1], c->B[1][i], fma(l[0], c->B[0][i], c->T[i])));
    return in;
}
static int cb_proj_cyl(const or_cylbox* c, double R, double H, const double* x, double* y) {
    double z = dot3(c->a, x);
    double r[3] = {x[0] - z * c->a[0], x[1] - z * c->a[1], x[2] - z * c->a[2]};
    double rr = dot3(r, r);
    int in = rr < R * R && z < H && z > -H;
    double zc = z > H ? H : (z < -H ? -H : z);
    double f = rr > R * R ? R / sqrt(rr) : 1.0;
    for (int i = 0; i < 3; ++i) y[i] = fma(zc, c->a[i], f * r[i]);
    return in;
}
/* dist < thr (thr >= 0): alternating projections, x on the cylinder strictly inside the box
   or closer than thr to its projection y on the box */
static int cb_touch_witness(const or_cylbox* c, double thr) {
    double x[3], y[3] = {c->T[0], c->T[1], c->T[2]};
    for (int it = 0; it < 3; ++it) {
        cb_proj_cyl(c, c->R, c->H, y, x);
        if (cb_proj_box(c, c->e, x, y)) return 1;
        double d[3] = {x[0] - y[0], x[1] - y[1], x[2] - y[2]};
        if (thr > 0.0 && dot3(d, d) < thr * thr) return 1;
    }
    return 0;
}
/* dist < -dl: a point of the cylinder shrunk by dl strictly inside the box, or of the box
   shrunk by dl strictly inside the cylinder ((A (-) ball) - B lies in (A - B) (-) ball) */
static int cb_deep_witness(const or_cylbox* c, double dl) {
    double x[3], y[3];
    if (c->R > dl && c->H > dl) {
        y[0] = c->T[0]; y[1] = c->T[1]; y[2] = c->T[2];
        for (int it = 0; it < 3; ++it) {
            cb_proj_cyl(c, c->R - dl, c->H - dl, y, x);
            if (cb_proj_box(c, c->e, x, y)) return 1;
        }
    }
    if (c->e[0] > dl && c->e[1] > dl && c->e[2] > dl) {
        double es[3] = {c->e[0] - dl, c->e[1] - dl, c->e[2] - dl};
        x[0] = 0.0; x[1] = 0.0; x[2] = 0.0;
        for (int it = 0; it < 3; ++it) {
            cb_proj_box(c, es, x, y);
            if (cb_proj_cyl(c, c->R, c->H, y, x)) return 1;
        }
    }
    return 0;
}

/* the candidate search runs in the box's frame (box axes = identity), as on the device */
static or_cylbox cb_box_frame(const or_cylbox* c) {
    or_cylbox b;
    for (int k = 0; k < 3; ++k) {
        b.T[k] = dot3(c->B[k], c->T);
        b.a[k] = dot3(c->B[k], c->a);
        b.e[k] = c->e[k];
        for (int i = 0; i < 3; ++i) b.B[k][i] = k == i ? 1.0 : 0.0;
    }
    b.R = c->R; b.H = c->H;
    return b;
}

/* Vertical cylinder (ma[2] = ma[5] = 0) vs upright box (mb[2] = mb[5] = mb[6] = mb[7] = 0): both
   are prisms along z, so the signed distance is that of the centre offset (box frame) to
   (rectangle + disc R) x [-(ez + H), ez + H]; the device's sspd::cb_upright_sd, operation for
   operation (the yaw-only TaskSpacePlanner mover keeps such pairs upright). */
static int cb_upright(const double* ma, const double* mb) {
    return ma[2] == 0.0 && ma[5] == 0.0 && mb[2] == 0.0 && mb[5] == 0.0 && mb[6] == 0.0 && mb[7] == 0.0;
}
static double cb_upright_sd(const double* pa, const double* sz, const double* pb, const double* mb,
                            const double* eb) {
    const double d0 = pa[0] - pb[0], d1 = pa[1] - pb[1], d2 = pa[2] - pb[2];
    const double cx = fma(mb[3], d1, mb[0] * d0), cy = fma(mb[4], d1, mb[1] * d0), cz = mb[8] * d2;
    const double ax = fabs(cx) - eb[0], ay = fabs(cy) - eb[1];
    double dr;
    if (ax > 0.0 || ay > 0.0) {
        const double ox = ax > 0.0 ? ax : 0.0, oy = ay > 0.0 ? ay : 0.0;
        dr = sqrt(fma(ox, ox, oy * oy));
    } else {
        dr = ax > ay ? ax : ay;
    }
    const double dxy = dr - sz[0], dz = fabs(cz) - (sz[1] + eb[2]);
    if (dxy > 0.0 && dz > 0.0) return sqrt(fma(dxy, dxy, dz * dz));
    return dxy > dz ? dxy : dz;
}

/* cylinder (A) vs box (B): signed distance < thr; SAT axes, then witnesses, then the
   remaining candidate directions */
static int cyl_box_overlap(const double* pa, const double* ma, const double* sz, const double* pb,
                           const double* mb, const double* eb, double thr) {
    or_cylbox c = make_cylbox(pa, ma, sz, pb, mb, eb);
    if (cb_base_sep(&c, thr)) return 0;
    /* past the SAT axes everything runs in the box's frame, as on the device */
    or_cylbox b = cb_box_frame(&c);
    int deep = thr < 0.0;
    if (deep ? cb_deep_witness(&b, -thr) : cb_touch_witness(&b, thr)) return 1;
    return !cb_ext_sep(&b, thr, deep);
}

/* dispatch; returns contact count, *ndeep deep count, -1 if unsupported */
static int collide(int t1, const double* p1, const double* m1, const double* s1, int t2,
                   const double* p2, const double* m2, const double* s2, double margin, int* ndeep) {
    *ndeep = 0;
    if (t1 > t2) { /* order by type like mj_collision's table */
        int tt = t1; t1 = t2; t2 = tt;
        const double* x;
        x = p1; p1 = p2; p2 = x;
        x = m1; m1 = m2; m2 = x;
        x = s1; s1 = s2; s2 = x;
    }
    if (t1 == OR_GEOM_PLANE) {
        if (t2 == OR_GEOM_BOX) return col_plane_box(p1, m1, p2, m2, s2, margin, ndeep);
        if (t2 == OR_GEOM_SPHERE) return col_plane_sphere(p1, m1, p2, s2[0], margin, ndeep);
        if (t2 == OR_GEOM_CYLINDER) return col_plane_cyl(p1, m1, p2, m2, s2, margin, ndeep);
        if (t2 == OR_GEOM_PLANE) return 0;
        return -1;
    }
    if (t1 == OR_GEOM_SPHERE) {
        if (t2 == OR_GEOM_SPHERE) return col_sphere_sphere(p1, s1[0], p2, s2[0], margin, ndeep);
        if (t2 == OR_GEOM_BOX) return col_sphere_box(p1, s1[0], p2, m2, s2, margin, ndeep);
        if (t2 == OR_GEOM_CYLINDER) return col_sphere_cyl(p1, s1[0], p2, m2, s2, margin, ndeep);
        return -1;
    }
    if (t1 == OR_GEOM_CYLINDER && t2 == OR_GEOM_BOX) { /* exact; one contact (MuJoCo convex) */
        if (cb_upright(m1, m2)) {
            const double sd = cb_upright_sd(p1, s1, p2, m2, s2);
            if (!(sd < margin)) return 0;
            *ndeep = sd < DEEP;
            return 1;
        }
        int c = cyl_box_overlap(p1, m1, s1, p2, m2, s2, margin);
        if (!c) return 0;
        *ndeep = cyl_box_overlap(p1, m1, s1, p2, m2, s2, DEEP);
        return 1;
    }
    if (t1 == OR_GEOM_BOX && t2 == OR_GEOM_BOX) { /* SAT decides; deep count from the manifold */
        int c = sat_box_box(p1, m1, s1, p2, m2, s2, margin);
        if (!c) return 0;
        *ndeep = box_box_deep_count(p1, m1, s1, p2, m2, s2); /* 0 unless deep (its SAT pass) */
        return 1;
    }
    return -1;
}

int or_point_contacts(const or_scene* s, const double* q, int count_static, double* deep_cost,
                      int* n_deep) {
    int nb = s->nbody, ng = s->ngeom;
    double qpos_buf[256], xpos_b[3 * 64], xquat_b[4 * 64], xmat_b[9 * 64], gxpos_b[3 * 128],
        gxmat_b[9 * 128];
    double *qpos = qpos_buf, *xpos = xpos_b, *xquat = xquat_b, *xmat = xmat_b, *gxpos = gxpos_b,
           *gxmat = gxmat_b;
    int heap = (s->nq > 256 || nb > 64 || ng > 128);
    if (heap) {
        qpos = (double*)malloc(8 * (size_t)(s->nq + 1));
        xpos = (double*)malloc(24 * (size_t)nb); xquat = (double*)malloc(32 * (size_t)nb);
        xmat = (double*)malloc(72 * (size_t)nb);
        gxpos = (double*)malloc(24 * (size_t)(ng + 1)); gxmat = (double*)malloc(72 * (size_t)(ng + 1));
    }
    set_qpos(s, q, qpos);
    fk(s, qpos, xpos, xquat, xmat, gxpos, gxmat);
    int ncon = 0, ndeep_tot = 0;
    double cost = 0.0;
    for (int k = 0; k < s->npair; ++k) {
        const or_pair* pr = s->pairs + k;
        if (pr->is_static && !(count_static || s->mode == 1)) continue;
        int g1 = pr->g1, g2 = pr->g2;
        double dc[3] = {gxpos[3 * g2] - gxpos[3 * g1], gxpos[3 * g2 + 1] - gxpos[3 * g1 + 1],
                        gxpos[3 * g2 + 2] - gxpos[3 * g1 + 2]};
        double r1 = s->rbound[g1], r2 = s->rbound[g2];
        if (r1 > 0.0 && r2 > 0.0) { /* bounding-sphere broadphase with margin */
            double thr = r1 + r2 + pr->margin;
            if (dot3(dc, dc) > thr * thr) continue;
        }
        int nd = 0;
        int nc = collide(s->geom_type[g1], gxpos + 3 * g1, gxmat + 9 * g1, s->geom_size + 3 * g1,
                         s->geom_type[g2], gxpos + 3 * g2, gxmat + 9 * g2, s->geom_size + 3 * g2,
                         pr->margin, &nd);
        if (nc < 0) { ncon = -1000000; break; }
        ncon += nc;
        if (nd > 0) {
            double cd = sqrt(dot3(dc, dc));
            double term = -1.0 / (cd + 1e-4);
            for (int i = 0; i < nd; ++i) cost = cost + term;
            ndeep_tot += nd;
        }
    }
    if (heap) { free(qpos); free(xpos); free(xquat); free(xmat); free(gxpos); free(gxmat); }
    if (deep_cost) *deep_cost = cost;
    if (n_deep) *n_deep = ndeep_tot;
    return ncon;
}

/* Analysis hook (tools/ only): contact count of every pair at q, in the scene's pair order
 * (static pairs included), plus the pair's geoms.  Same FK and narrowphase as above. */
int or_point_pair_contacts(const or_scene* s, const double* q, int* counts, int* g1_out, int* g2_out) {
    int nb = s->nbody, ng = s->ngeom;
    if (s->nq > 256 || nb > 64 || ng > 128) return -1;
    double qpos[256], xpos[3 * 64], xquat[4 * 64], xmat[9 * 64], gxpos[3 * 128], gxmat[9 * 128];
    set_qpos(s, q, qpos);
    fk(s, qpos, xpos, xquat, xmat, gxpos, gxmat);
    for (int k = 0; k < s->npair; ++k) {
        const or_pair* pr = s->pairs + k;
        int g1 = pr->g1, g2 = pr->g2;
        if (g1_out) g1_out[k] = g1;
        if (g2_out) g2_out[k] = g2;
        counts[k] = 0;
        double dc[3] = {gxpos[3 * g2] - gxpos[3 * g1], gxpos[3 * g2 + 1] - gxpos[3 * g1 + 1],
                        gxpos[3 * g2 + 2] - gxpos[3 * g1 + 2]};
        double r1 = s->rbound[g1], r2 = s->rbound[g2];
        if (r1 > 0.0 && r2 > 0.0) {
            double thr = r1 + r2 + pr->margin;
            if (dot3(dc, dc) > thr * thr) continue;
        }
        int nd = 0;
        counts[k] = collide(s->geom_type[g1], gxpos + 3 * g1, gxmat + 9 * g1, s->geom_size + 3 * g1,
                            s->geom_type[g2], gxpos + 3 * g2, gxmat + 9 * g2, s->geom_size + 3 * g2,
                            pr->margin, &nd);
    }
    return s->npair;
}

/* ------------------------------------------------------------------ reductions
 * Canonical order (shared with the GPU kernels): `lanes` lanes, lane l accumulates
 * x[l], x[l+lanes], ... sequentially from 0.0; each 64-lane wave reduces its lanes by
 * an xor butterfly (offsets 32,16,8,4,2,1); the wave sums are added in wave order. */
int or_lanes_for(int items) {
    int l = ((items + 63) / 64) * 64;
    if (l < 64) l = 64;
    if (l > 256) l = 256; /* workgroup size of the GPU kernels */
    return l;
}

double or_canon_sum(const double* x, int n, int lanes) {
    double part[1024], tmp[64];
    for (int l = 0; l < lanes; ++l) {
        double acc = 0.0;
        for (int i = l; i < n; i += lanes) acc = acc + x[i];
        part[l] = acc;
    }
    double total = 0.0;
    for (int w = 0; w < lanes / 64; ++w) {
        double* v = part + 64 * w;
        for (int off = 32; off >= 1; off >>= 1) {
            for (int l = 0; l < 64; ++l) tmp[l] = v[l] + v[l ^ off];
            memcpy(v, tmp, sizeof(tmp));
        }
        total = (w == 0) ? v[0] : total + v[0];
    }
    return total;
}

static double seq_sum(const double* x, int n) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc = acc + x[i];
    return acc;
}

static double dist_nd(const double* a, const double* b, int D) {
    double d0 = b[0] - a[0];
    double s = d0 * d0;
    for (int d = 1; d < D; ++d) { double dd = b[d] - a[d]; s = fma(dd, dd, s); }
    return sqrt(s);
}

/* ------------------------------------------------------------------ SamplingPathPlanner */
int or_sspp_score(const or_scene* s, const double* knots, int nknots, int p, const double* ctrl,
                  int n, int D, int64_t B, int W, int count_static, int sequential_sum,
                  int nthreads, int arc_all, double* arc_out, uint8_t* feasible_out) {
    if (W < 2 || D > OR_MAXD || p > OR_MAXP || nknots != n + p + 1) return -1;
    if (s && s->mode == 0 && s->arg != D) return -2;
    int bad = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : bad)
#endif
    for (int64_t b = 0; b < B; ++b) {
        const double* c = ctrl + (size_t)b * n * D;
        double q[OR_MAXD], q2[OR_MAXD];
        /* include/sspp.h:132-150 checkCollision: points u = i/W, i = 0..W */
        int feasible = 1;
        if (s) {
            for (int i = 0; i <= W; ++i) {
                double u = (double)i / W;
                or_spline_eval(knots, nknots, p, c, D, u, q);
                int nc = or_point_contacts(s, q, count_static, NULL, NULL);
                if (nc < 0) { bad = 1; break; }
                if (nc > 0) { feasible = 0; break; }
            }
        }
        feasible_out[b] = (uint8_t)feasible;
        /* include/sspp.h:171-192 findBestPath scores only the successful paths */
        if (!feasible && !arc_all) { arc_out[b] = INFINITY; continue; }
        /* include/sspp.h:152-169 computeArcLength: chords between u=(i-1)/(W-1), i/(W-1) */
        double chords[4096];
        double* ch = W - 1 <= 4096 ? chords : (double*)malloc(sizeof(double) * (size_t)(W - 1));
        for (int i = 1; i < W; ++i) {
            double u1 = (double)(i - 1) / (W - 1);
            double u2 = (double)i / (W - 1);
            or_spline_eval(knots, nknots, p, c, D, u1, q);
            or_spline_eval(knots, nknots, p, c, D, u2, q2);
            ch[i - 1] = dist_nd(q, q2, D);
        }
        arc_out[b] = sequential_sum ? seq_sum(ch, W - 1) : or_canon_sum(ch, W - 1, or_lanes_for(W - 1));
        if (ch != chords) free(ch);
    }
    return bad ? -3 : 0;
}

int64_t or_argmin(const double* cost, const uint8_t* feasible, int64_t B, double* best_cost) {
    /* include/sspp.h:171-192 findBestPath: strict '<' from +inf; lowest index on ties */
    double best = INFINITY;
    int64_t idx = -1;
    for (int64_t b = 0; b < B; ++b) {
        if (!feasible[b]) continue;
        if (cost[b] < best) { best = cost[b]; idx = b; }
    }
    if (best_cost) *best_cost = best;
    return idx;
}

/* ------------------------------------------------------------------ TaskSpacePlanner */
int or_tsp_score(const or_scene* s, const double* start, const double* end, const double* vias,
                 int K, int64_t B, int cp, double w_collision, int sequential_sum, int nthreads,
                 double* Lo, double* Cnfo, double* Cwfo, uint8_t* status, double* cost) {
    if (cp < 1 || K < 0 || K > 62 || !s || s->mode != 1) return -1;
    const int P = 2, D = 4, n = K + 2;
    int bad = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(| : bad)
#endif
    for (int64_t b = 0; b < B; ++b) {
        double pts[64 * 4], u[64], knots[64 + 3], ctrl[64 * 4];
        /* tsp_path_model.h:11-43: [start, vias..., end] at u_i = i/(total-1) */
        for (int i = 0; i < n; ++i) u[i] = (double)i / (n - 1);
        for (int d = 0; d < D; ++d) { pts[d] = start[d]; pts[(n - 1) * D + d] = end[d]; }
        for (int v = 0; v < K; ++v)
            for (int d = 0; d < D; ++d) pts[(1 + v) * D + d] = vias[((size_t)b * K + v) * D + d];
        if (or_interpolate(pts, n, D, P, u, knots, ctrl) != 0) { bad = 1; continue; }
        int nk = n + P + 1;
        /* tsp_evaluator.h:18-32 eval_one_pass */
        double du = 1.0 / cp;
        double prev[4], cur[4];
        double Lb[4096], Cb[4096], Wb[4096];
        double *Lv = Lb, *Cv = Cb, *Wv = Wb;
        if (cp > 4096) {
            Lv = (double*)malloc(8 * (size_t)cp); Cv = (double*)malloc(8 * (size_t)cp);
            Wv = (double*)malloc(8 * (size_t)cp);
        }
        or_spline_eval(knots, nk, P, ctrl, D, 0.0, prev);
        for (int i = 1; i <= cp; ++i) {
            /* the reference evaluates s(i*du) and s((i-1)*du) as consecutive points;
               each lane of the GPU kernel evaluates both, so do the same here */
            double up = (double)(i - 1) * du, uc = (double)i * du;
            or_spline_eval(knots, nk, P, ctrl, D, up, prev);
            or_spline_eval(knots, nk, P, ctrl, D, uc, cur);
            Lv[i - 1] = dist_nd(prev, cur, D);
            double c = 0.0;
            int nc = or_point_contacts(s, cur, 1, &c, NULL);
            if (nc < 0) bad = 1;
            /* floorPenalty with the evaluator's defaults */
            double deficit = (0.0 + 0.01) - cur[2];
            double fp = deficit > 0.0 ? (10.0 * deficit) * deficit : 0.0;
            Cv[i - 1] = c;
            Wv[i - 1] = c + fp;
        }
        double L, Cnf, Cwf;
        if (sequential_sum) { L = seq_sum(Lv, cp); Cnf = seq_sum(Cv, cp); Cwf = seq_sum(Wv, cp); }
        else {
            int lanes = or_lanes_for(cp);
            L = or_canon_sum(Lv, cp, lanes); Cnf = or_canon_sum(Cv, cp, lanes);
            Cwf = or_canon_sum(Wv, cp, lanes);
        }
        if (Lv != Lb) { free(Lv); free(Cv); free(Wv); }
        Lo[b] = L; Cnfo[b] = Cnf; Cwfo[b] = Cwf;
        status[b] = (uint8_t)(Cnf == 0.0); /* tsp_planner.h:110 */
        cost[b] = L + w_collision * Cwf;   /* tsp_planner.h:123 */
    }
    return bad ? -3 : 0;
}

int64_t or_tsp_best(const double* cost, const uint8_t* status, int64_t B, double* best_cost) {
    /* tsp_planner.h:131-134 min_element over successes; lowest index on ties */
    return or_argmin(cost, status, B, best_cost);
}

/* ================================================================ TaskSpacePlanner CES update
 * tsp::Planner::plan after the evaluation loop (include/sspp/tsp_planner.h:121-142):
 *   successes -> EliteSelector::select (tsp_elites.h:13-22: top k = max(1, int(n * frac)) by
 *   L + w * C_wf), ::weights (24-32: log(k + 0.5) - log(i + 1), normalised),
 *   Distribution::update (tsp_distribution.h:52-83), best = std::min_element, adapt (31-38).
 * Candidate order = slot order and ties go to the lowest slot.  sequential = 1
 * sums in the reference's order; 0 in the GPU's canonical order (or_canon_sum, 512 lanes). */
typedef struct { double cost; int64_t slot; } or_ces_key;

static int or_ces_cmp(const void* a, const void* b) {
    const or_ces_key* x = (const or_ces_key*)a;
    const or_ces_key* y = (const or_ces_key*)b;
    if (x->cost < y->cost) return -1;
    if (y->cost < x->cost) return 1;
    return (x->slot > y->slot) - (x->slot < y->slot);
}

static double or_ces_clamp_sd(double s, const or_ces_cfg* c) {
    s = s < c->sd_min ? c->sd_min : s;
    s = s > c->sd_max ? c->sd_max : s;
    return s < c->sigma_floor ? c->sigma_floor : s;
}

static double or_wrap_diff(double a, double b, double mn, double mx) {
    const double range = mx - mn;
    double d = a - b;
    while (d > 0.5 * range) d -= range;
    while (d < -0.5 * range) d += range;
    return d;
}

static double or_ces_sum(const double* x, int n, int sequential) {
    return sequential ? seq_sum(x, n) : or_canon_sum(x, n, 512);  /* k_ces_update: 512 lanes */
}

int or_ces_update(const or_ces_cfg* c, const double* cost, const uint8_t* status,
                  const double* vias, int64_t n, double* mean, double* sigma, double* last_best,
                  int* has_best, int32_t* elites, int* n_elite, int64_t* best_slot) {
    const int K = c->K, KD = 4 * K;
    int64_t ns = 0;
    for (int64_t i = 0; i < n; ++i) ns += status[i] != 0;
    *n_elite = 0;
    *best_slot = -1;
    if (ns == 0) {
        for (int q = 0; q < KD; ++q) sigma[q] = or_ces_clamp_sd(sigma[q] * c->inc, c);
        return 0;
    }
    or_ces_key* keys = (or_ces_key*)malloc(sizeof(or_ces_key) * (size_t)ns);
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i)
        if (status[i]) { keys[m].cost = cost[i]; keys[m].slot = i; ++m; }
    qsort(keys, (size_t)ns, sizeof(or_ces_key), or_ces_cmp);
    int k = (int)((double)ns * c->frac);
    if (k < 1) k = 1;
    double* w = (double*)malloc(sizeof(double) * (size_t)k);
    double* x = (double*)malloc(sizeof(double) * (size_t)k);
    const double lk = log((double)k + 0.5);
    for (int j = 0; j < k; ++j) x[j] = lk - log((double)j + 1.0);
    const double sumw = or_ces_sum(x, k, c->sequential);
    for (int j = 0; j < k; ++j) w[j] = x[j] / sumw;
    for (int q = 0; q < KD; ++q) {
        const int d = q & 3;
        for (int j = 0; j < k; ++j) x[j] = w[j] * vias[keys[j].slot * KD + q];
        const double em = or_ces_sum(x, k, c->sequential);
        const double m0 = mean[q];
        double nm = m0 + c->mean_lr * (em - m0);
        if (d == 2) nm = nm < c->dist_z_min ? c->dist_z_min : nm;
        nm = nm < c->lo[d] ? c->lo[d] : (c->hi[d] < nm ? c->hi[d] : nm);
        const int wrap = d == 3 && c->lo[3] != c->hi[3];
        for (int j = 0; j < k; ++j) {
            const double v = vias[keys[j].slot * KD + q];
            const double df = wrap ? or_wrap_diff(v, nm, c->lo[3], c->hi[3]) : v - nm;
            x[j] = w[j] * (df * df);
        }
        const double ve = or_ces_sum(x, k, c->sequential);
        const double pv = sigma[q] * sigma[q];
        const double blend = (1.0 - c->var_beta) * pv + c->var_beta * ve;
        double sg = or_ces_clamp_sd(sqrt(blend), c);
        sigma[q] = or_ces_clamp_sd(sg * c->dec, c);
        mean[q] = nm;
    }
    for (int q = 0; q < KD; ++q) last_best[q] = vias[keys[0].slot * KD + q];
    *has_best = 1;
    *best_slot = keys[0].slot;
    for (int j = 0; j < k; ++j) elites[j] = (int32_t)keys[j].slot;
    *n_elite = k;
    free(keys); free(w); free(x);
    return (int)ns;
}
