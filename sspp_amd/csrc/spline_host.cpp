// spline_host.cpp — host-side B-spline construction (Eigen unsupported/Splines semantics).
//
// Reference call sites: include/sspp.h:95 (SplineFitting::Interpolate, degree 3, parameters
// u_i = i/(n-1)), include/sspp/tsp_path_model.h:25-28,38-42 (degree 2).  The knot vector is
// Eigen's KnotAveraging; rows of the collocation matrix are Piegl & Tiller A2.2 basis values at
// the parameters with A(0,0) = A(n-1,n-1) = 1; the system is solved by Householder QR as Eigen's
// SplineFitting::Interpolate does (HouseholderQR), in exactly the operation order of
// oracle/sspp_oracle.c::qr_solve.  The factorisation depends only on the parameters, so it is
// kept as a "QR program" (reflectors + R) that the TaskSpacePlanner kernel replays per
// candidate: device and oracle control points agree bit for bit.
#include <cmath>
#include <vector>

#include "model.h"

namespace sspp {

void knot_averaging(const double* u, int n, int p, double* knots) {
    int nk = n + p + 1;
    for (int j = 1; j < n - p; ++j) {
        double s = 0.0;
        for (int r = 0; r < p; ++r) s = s + u[j + r];
        knots[j + p] = s / (double)p;
    }
    for (int i = 0; i <= p; ++i) knots[i] = 0.0;
    for (int i = nk - p - 1; i < nk; ++i) knots[i] = 1.0;
}

int span_of(double u, int p, const double* knots, int nknots) {
    if (u <= knots[0]) return p;
    int first = p - 1, count = (nknots - p - 1) - (p - 1);
    while (count > 0) {
        int step = count / 2, it = first + step;
        if (!(u < knots[it])) { first = it + 1; count -= step + 1; }
        else count = step;
    }
    return first - 1;
}

void basis_funcs(double u, int p, const double* knots, int nknots, double* N) {
    int i = span_of(u, p, knots, nknots);
    double left[16], right[16];
    left[0] = right[0] = 0.0;
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

static void collocation(const double* u, int n, int p, const double* knots, std::vector<double>& A) {
    int nk = n + p + 1;
    A.assign((size_t)n * n, 0.0);
    for (int i = 1; i < n - 1; ++i) {
        int sp = span_of(u[i], p, knots, nk);
        double N[16];
        basis_funcs(u[i], p, knots, nk, N);
        for (int r = 0; r <= p; ++r) A[(size_t)i * n + sp - p + r] = N[r];
    }
    A[0] = 1.0;
    A[(size_t)(n - 1) * n + n - 1] = 1.0;
}

// Householder QR of A (oracle qr_solve, A part): prog = [n][n] reflectors v_k (row k, entries
// k..n-1) | [n] |v_k|^2 (0 = no reflection at step k) | [n][n] R.
static int qr_factor(std::vector<double>& A, int n, double* prog) {
    double* V = prog;
    double* vn_out = prog + (size_t)n * n;
    double* R = vn_out + n;
    std::vector<double> v((size_t)n);
    for (size_t e = 0; e < (size_t)n * n; ++e) V[e] = 0.0;
    for (int k = 0; k < n; ++k) {
        vn_out[k] = 0.0;
        double norm = 0.0;
        for (int i = k; i < n; ++i) norm = std::fma(A[(size_t)i * n + k], A[(size_t)i * n + k], norm);
        norm = std::sqrt(norm);
        if (norm == 0.0) continue;
        const double alpha = A[(size_t)k * n + k] > 0 ? -norm : norm;
        for (int i = k; i < n; ++i) v[i] = A[(size_t)i * n + k];
        v[k] -= alpha;
        double vn = 0.0;
        for (int i = k; i < n; ++i) vn = std::fma(v[i], v[i], vn);
        if (vn == 0.0) continue;
        for (int j = k; j < n; ++j) {
            double s = 0.0;
            for (int i = k; i < n; ++i) s = std::fma(v[i], A[(size_t)i * n + j], s);
            s = 2.0 * s / vn;
            for (int i = k; i < n; ++i) A[(size_t)i * n + j] -= s * v[i];
        }
        vn_out[k] = vn;
        for (int i = k; i < n; ++i) V[(size_t)k * n + i] = v[i];
    }
    for (size_t e = 0; e < (size_t)n * n; ++e) R[e] = A[e];
    for (int i = 0; i < n; ++i)
        if (R[(size_t)i * n + i] == 0.0) return -2;
    return 0;
}

void qr_apply(const double* prog, int n, double* B, int D) {
    const double* V = prog;
    const double* vn = prog + (size_t)n * n;
    const double* R = vn + n;
    for (int k = 0; k < n; ++k) {
        if (vn[k] == 0.0) continue;
        const double* v = V + (size_t)k * n;
        for (int j = 0; j < D; ++j) {
            double s = 0.0;
            for (int i = k; i < n; ++i) s = std::fma(v[i], B[(size_t)i * D + j], s);
            s = 2.0 * s / vn[k];
            for (int i = k; i < n; ++i) B[(size_t)i * D + j] -= s * v[i];
        }
    }
    for (int j = 0; j < D; ++j) {
        for (int i = n - 1; i >= 0; --i) {
            double s = B[(size_t)i * D + j];
            for (int c = i + 1; c < n; ++c) s -= R[(size_t)i * n + c] * B[(size_t)c * D + j];
            B[(size_t)i * D + j] = s / R[(size_t)i * n + i];
        }
    }
}

int interpolate(const double* pts, int n, int D, int p, const double* u, double* knots,
                double* ctrl) {
    if (n < p + 1 || p < 1 || p > 15 || D < 1) return -1;
    knot_averaging(u, n, p, knots);
    std::vector<double> A, prog((size_t)2 * n * n + n);
    collocation(u, n, p, knots, A);
    if (qr_factor(A, n, prog.data()) != 0) return -1;
    for (size_t k = 0; k < (size_t)n * D; ++k) ctrl[k] = pts[k];
    qr_apply(prog.data(), n, ctrl, D);
    return 0;
}

int qr_program(const double* u, int n, int p, double* knots, double* prog) {
    if (n < p + 1 || p < 1 || p > 15) return -1;
    knot_averaging(u, n, p, knots);
    std::vector<double> A;
    collocation(u, n, p, knots, A);
    return qr_factor(A, n, prog);
}

}  // namespace sspp
