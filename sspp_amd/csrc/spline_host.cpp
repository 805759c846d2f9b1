// spline_host.cpp — host-side B-spline construction (Eigen unsupported/Splines semantics).
//
// Reference call sites: include/sspp.h:95 (SplineFitting::Interpolate, degree 3, parameters
// u_i = i/(n-1)), include/sspp/tsp_path_model.h:25-28,38-42 (degree 2).  The knot vector is
// Eigen's KnotAveraging; rows of the collocation matrix are Piegl & Tiller A2.2 basis values at
// the parameters with A(0,0) = A(n-1,n-1) = 1; the system is solved by LU with partial
// pivoting (Eigen uses HouseholderQR: same solution up to rounding).
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

// Solve A X = B in place (A n x n, B n x m), partial pivoting.
static int lu_solve(std::vector<double>& A, double* B, int n, int m) {
    for (int k = 0; k < n; ++k) {
        int piv = k;
        double best = std::fabs(A[(size_t)k * n + k]);
        for (int i = k + 1; i < n; ++i) {
            double v = std::fabs(A[(size_t)i * n + k]);
            if (v > best) { best = v; piv = i; }
        }
        if (best == 0.0) return -1;
        if (piv != k) {
            for (int j = 0; j < n; ++j) std::swap(A[(size_t)k * n + j], A[(size_t)piv * n + j]);
            for (int j = 0; j < m; ++j) std::swap(B[(size_t)k * m + j], B[(size_t)piv * m + j]);
        }
        for (int i = k + 1; i < n; ++i) {
            double f = A[(size_t)i * n + k] / A[(size_t)k * n + k];
            if (f == 0.0) continue;
            for (int j = k; j < n; ++j) A[(size_t)i * n + j] -= f * A[(size_t)k * n + j];
            for (int j = 0; j < m; ++j) B[(size_t)i * m + j] -= f * B[(size_t)k * m + j];
        }
    }
    for (int j = 0; j < m; ++j) {
        for (int i = n - 1; i >= 0; --i) {
            double s = B[(size_t)i * m + j];
            for (int c = i + 1; c < n; ++c) s -= A[(size_t)i * n + c] * B[(size_t)c * m + j];
            B[(size_t)i * m + j] = s / A[(size_t)i * n + i];
        }
    }
    return 0;
}

int interpolate(const double* pts, int n, int D, int p, const double* u, double* knots,
                double* ctrl) {
    if (n < p + 1 || p < 1 || p > 15 || D < 1) return -1;
    knot_averaging(u, n, p, knots);
    std::vector<double> A;
    collocation(u, n, p, knots, A);
    for (size_t k = 0; k < (size_t)n * D; ++k) ctrl[k] = pts[k];
    return lu_solve(A, ctrl, n, D);
}

int collocation_inverse(const double* u, int n, int p, double* knots, double* Minv) {
    if (n < p + 1 || p < 1 || p > 15) return -1;
    knot_averaging(u, n, p, knots);
    std::vector<double> A;
    collocation(u, n, p, knots, A);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) Minv[(size_t)i * n + j] = (i == j) ? 1.0 : 0.0;
    return lu_solve(A, Minv, n, n);
}

}  // namespace sspp
