// sspp_device.h — FP64 geometry for the candidate-scoring kernels (CDNA4, wave64).
//
// Restates, per waypoint, what the reference gets from one mj_forward call
// (include/sspp.h:139-147, include/Collision.h:84-103): free-joint forward kinematics,
// the bounding-sphere broadphase and the primitive narrowphase, with the contact rules
// documented in DESIGN.md §Collision semantics.  Every expression is written operation by
// operation (explicit fma, compiled with -ffp-contract=off) in the same order as the CPU
// restatement in oracle/, so GPU and oracle agree bit for bit wherever their inputs do.
//
// __host__ __device__ so the scene builder evaluates env-env pairs with the same code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SSPP_HD __host__ __device__ __forceinline__

namespace sspd {

constexpr double kDeep = -1e-3;     // include/Collision.h:93 "col_dist < -1e-3"
constexpr double kMinVal = 1e-15;   // mjMINVAL
constexpr int kMaxP = 7;            // max spline degree in kernels

// Geom table entry in device memory.  Static geoms: world pose.  Moving geoms: pose
// relative to their mover's root body frame.
struct DGeom {
    double pos[3];
    double mat[9];   // row-major, columns = geom axes
    double size[3];
    double rbound;   // bounding-sphere radius (0 = infinite, planes)
    double reach;    // moving geoms: |pos| (centre offset from the mover root), else 0
    int32_t type;
    int32_t mover;   // -1 static
    int32_t orig;    // model geom index (orders same-type pairs like the oracle)
    int32_t relrot;  // moving geoms: 0 when mat is exactly the identity (pose = mover rotation)
};

// One filter-passing pair with the partner's data inlined, so the wave-uniform pair loop
// reads one contiguous record per pair (scalar loads, no dependent index chain).
struct DPair {
    int32_t gm;      // index of the moving geom in the DGeom table
    int32_t go;      // index of the partner geom
    int32_t otype;   // partner type
    int32_t oorig;   // partner model index
    int32_t omover;  // partner mover (-1 static)
    int32_t pad;
    double margin;   // max(margin1, margin2)
    double opos[3];  // partner pose: world (static) or relative to its mover
    double omat[9];
    double osize[3];
    double orbound;
};

struct DMover {
    int32_t qpos_adr;
    int32_t pad;
    double qpos0[7];
};

SSPP_HD double dot3(const double* a, const double* b) {
    return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]));
}
SSPP_HD void matvec3(const double* m, const double* v, double* r) {
    r[0] = dot3(m + 0, v);
    r[1] = dot3(m + 3, v);
    r[2] = dot3(m + 6, v);
}
SSPP_HD void col3(const double* m, int j, double* c) {
    c[0] = m[j];
    c[1] = m[3 + j];
    c[2] = m[6 + j];
}
// r = a * b (3x3 row-major); r_ij = row_i(a) . col_j(b)
SSPP_HD void matmul3(const double* a, const double* b, double* r) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double c[3] = {b[j], b[3 + j], b[6 + j]};
            r[3 * i + j] = dot3(a + 3 * i, c);
        }
    }
}
SSPP_HD void normalize4(double* q) {
    double s = q[0] * q[0];
    s = fma(q[1], q[1], s);
    s = fma(q[2], q[2], s);
    s = fma(q[3], q[3], s);
    double n = sqrt(s);
    if (n < kMinVal) {
        q[0] = 1.0; q[1] = 0.0; q[2] = 0.0; q[3] = 0.0;
    } else if (fabs(n - 1.0) > kMinVal) {
        double inv = 1.0 / n;
        q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
    }
}
SSPP_HD void mulquat(const double* a, const double* b, double* r) {
    double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
// mju_quat2Mat without MuJoCo's identity shortcut (same matrix; one code path, no scratch)
SSPP_HD void quat2mat(const double* q, double* m) {
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

// ---------------------------------------------------------------- B-spline basis (A2.1/A2.2)
SSPP_HD int span_of(double u, int p, const double* knots, int nknots) {
    if (u <= knots[0]) return p;
    int first = p - 1, count = (nknots - p - 1) - (p - 1);
    while (count > 0) {
        int step = count / 2, it = first + step;
        if (!(u < knots[it])) { first = it + 1; count -= step + 1; }
        else count = step;
    }
    return first - 1;
}
SSPP_HD void basis_funcs(double u, int p, int span, const double* knots, double* N) {
    double left[kMaxP + 1], right[kMaxP + 1];
    left[0] = 0.0; right[0] = 0.0;
    for (int j = 1; j <= p; ++j) {
        left[j] = u - knots[span + 1 - j];
        right[j] = knots[span + j] - u;
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

// ---------------------------------------------------------------- narrowphase
// Each returns the contact count (dist < margin); *nd = contacts with dist < -1e-3.
SSPP_HD int col_plane_box(const double* pp, const double* pm, const double* bp, const double* bm,
                          const double* e, double margin, int* nd) {
    double n[3], d[3], ax[3], a[3];
    col3(pm, 2, n);
    d[0] = bp[0] - pp[0]; d[1] = bp[1] - pp[1]; d[2] = bp[2] - pp[2];
    double d0 = dot3(d, n);
#pragma unroll
    for (int j = 0; j < 3; ++j) { col3(bm, j, ax); a[j] = dot3(n, ax) * e[j]; }
    int nc = 0, ndd = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        double t = d0 + ((k & 1) ? a[0] : -a[0]);
        t = t + ((k & 2) ? a[1] : -a[1]);
        t = t + ((k & 4) ? a[2] : -a[2]);
        if (t < margin && nc < 4) { nc++; if (t < kDeep) ndd++; }
    }
    *nd = ndd;
    return nc;
}
SSPP_HD int col_plane_sphere(const double* pp, const double* pm, const double* sp, double r,
                             double margin, int* nd) {
    double n[3], d[3];
    col3(pm, 2, n);
    d[0] = sp[0] - pp[0]; d[1] = sp[1] - pp[1]; d[2] = sp[2] - pp[2];
    double dist = dot3(d, n) - r;
    *nd = dist < kDeep;
    return dist < margin;
}
SSPP_HD int col_plane_cyl(const double* pp, const double* pm, const double* cp, const double* cm,
                          const double* sz, double margin, int* nd) {
    double n[3], a[3], d[3];
    col3(pm, 2, n);
    col3(cm, 2, a);
    d[0] = cp[0] - pp[0]; d[1] = cp[1] - pp[1]; d[2] = cp[2] - pp[2];
    double dn = dot3(d, n), na = dot3(n, a);
    double s = 1.0 - na * na;
    double rim = sz[0] * sqrt(s > 0.0 ? s : 0.0);
    double ha = sz[1] * na;
    int nc = 0, ndd = 0;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        double t = (c == 0) ? dn - ha : dn + ha;
        t = t - rim;
        if (t < margin) { nc++; if (t < kDeep) ndd++; }
    }
    *nd = ndd;
    return nc;
}
SSPP_HD int col_sphere_sphere(const double* p1, double r1, const double* p2, double r2,
                              double margin, int* nd) {
    double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    double dist = sqrt(dot3(d, d)) - (r1 + r2);
    *nd = dist < kDeep;
    return dist < margin;
}
SSPP_HD int col_sphere_box(const double* sp, double r, const double* bp, const double* bm,
                           const double* e, double margin, int* nd) {
    double d[3] = {sp[0] - bp[0], sp[1] - bp[1], sp[2] - bp[2]}, ax[3];
    bool inside = true;
    double mind = 1e300, out2 = 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        col3(bm, j, ax);
        double l = dot3(ax, d);
        double al = fabs(l);
        if (al > e[j]) { inside = false; double o = al - e[j]; out2 = fma(o, o, out2); }
        double f = e[j] - al;
        if (f < mind) mind = f;
    }
    double dist = inside ? (-mind - r) : (sqrt(out2) - r);
    *nd = dist < kDeep;
    return dist < margin;
}
SSPP_HD int col_sphere_cyl(const double* sp, double r, const double* cp, const double* cm,
                           const double* sz, double margin, int* nd) {
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
    *nd = dist < kDeep;
    return dist < margin;
}

// Separating-axis test, two boxes: true iff every one of the 15 axis separations < thr.
// Rows of R = A^T B are formed lazily so that an early separating face of A (the common
// case: the moving box hovering over a static box) skips the rest.  Edge axes compare the
// unnormalised separation with thr * |L| (no division; the oracle does the same).
SSPP_HD bool sat_box_box(const double* pa, const double* ma, const double* ea, const double* pb,
                         const double* mb, const double* eb, double thr) {
    const double T[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    double B0[3], B1[3], B2[3];
    col3(mb, 0, B0);
    col3(mb, 1, B1);
    col3(mb, 2, B2);
    double t[3], R[3][3], AR[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double Ai[3];
        col3(ma, i, Ai);
        t[i] = dot3(Ai, T);
        R[i][0] = dot3(Ai, B0);
        R[i][1] = dot3(Ai, B1);
        R[i][2] = dot3(Ai, B2);
        AR[i][0] = fabs(R[i][0]);
        AR[i][1] = fabs(R[i][1]);
        AR[i][2] = fabs(R[i][2]);
        double rb = fma(eb[2], AR[i][2], fma(eb[1], AR[i][1], eb[0] * AR[i][0]));
        double sep = fabs(t[i]) - (ea[i] + rb);
        if (sep >= thr) return false;
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        double pr = fabs(fma(t[2], R[2][j], fma(t[1], R[1][j], t[0] * R[0][j])));
        double ra = fma(ea[2], AR[2][j], fma(ea[1], AR[1][j], ea[0] * AR[0][j]));
        double sep = pr - (ra + eb[j]);
        if (sep >= thr) return false;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double v0 = R[0][j], v1 = R[1][j], v2 = R[2][j], L[3];
            if (i == 0) { L[0] = 0.0; L[1] = -v2; L[2] = v1; }
            else if (i == 1) { L[0] = v2; L[1] = 0.0; L[2] = -v0; }
            else { L[0] = -v1; L[1] = v0; L[2] = 0.0; }
            double len2 = dot3(L, L);
            if (len2 < 1e-12) continue;
            double pr = fabs(dot3(t, L));
            double ra = fma(ea[2], fabs(L[2]), fma(ea[1], fabs(L[1]), ea[0] * fabs(L[0])));
            double rb = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                double bk[3] = {R[0][k], R[1][k], R[2][k]};
                rb = fma(eb[k], fabs(dot3(bk, L)), rb);
            }
            double num = pr - (ra + rb);
            if (thr == 0.0 ? num >= 0.0 : num >= thr * sqrt(len2)) return false;
        }
    }
    return true;
}

// cylinder (A) vs box (B) over the 7 finite axes {box faces, cylinder axis, axis x box edges}.
SSPP_HD bool sat_cyl_box(const double* pa, const double* ma, const double* sz, const double* pb,
                         const double* mb, const double* eb, double thr) {
    double a[3], Bc[3][3];
    col3(ma, 2, a);
#pragma unroll
    for (int j = 0; j < 3; ++j) col3(mb, j, Bc[j]);
    double T[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
#pragma unroll
    for (int ax = 0; ax < 7; ++ax) {
        double L[3];
        if (ax < 3) { L[0] = Bc[ax][0]; L[1] = Bc[ax][1]; L[2] = Bc[ax][2]; }
        else if (ax == 3) { L[0] = a[0]; L[1] = a[1]; L[2] = a[2]; }
        else {
            const double* b = Bc[ax - 4];
            L[0] = a[1] * b[2] - a[2] * b[1];
            L[1] = a[2] * b[0] - a[0] * b[2];
            L[2] = a[0] * b[1] - a[1] * b[0];
        }
        double len2 = dot3(L, L);
        if (len2 < 1e-12) continue;
        double aL = dot3(a, L);
        double rr = len2 - aL * aL;
        double rc = fma(sz[1], fabs(aL), sz[0] * sqrt(rr > 0.0 ? rr : 0.0));
        double rb = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) rb = fma(eb[k], fabs(dot3(Bc[k], L)), rb);
        double num = fabs(dot3(T, L)) - (rc + rb);
        if (thr == 0.0 ? num >= 0.0 : num >= thr * sqrt(len2)) return false;
    }
    return true;
}

// Supported narrowphase pair? (types ordered t1 <= t2)
SSPP_HD bool pair_supported(int t1, int t2) {
    if (t1 > t2) { int t = t1; t1 = t2; t2 = t; }
    if (t1 == 0) return t2 == 0 || t2 == 2 || t2 == 5 || t2 == 6;
    if (t1 == 2) return t2 == 2 || t2 == 5 || t2 == 6;
    return (t1 == 5 && t2 == 6) || (t1 == 6 && t2 == 6);
}

// Narrowphase dispatch.  Geom 1 must be the first by (type, model index), like the oracle.
// NEED_DEEP=false: returns the contact count (SamplingPathPlanner feasibility needs > 0).
// NEED_DEEP=true:  only *nd (contacts with dist < -1e-3, Collision.h cost) is meaningful.
template <bool NEED_DEEP>
SSPP_HD int collide(int t1, const double* p1, const double* m1, const double* s1, int t2,
                    const double* p2, const double* m2, const double* s2, double margin, int* nd) {
    *nd = 0;
    if (t1 == 0) {
        if (t2 == 6) return col_plane_box(p1, m1, p2, m2, s2, margin, nd);
        if (t2 == 2) return col_plane_sphere(p1, m1, p2, s2[0], margin, nd);
        if (t2 == 5) return col_plane_cyl(p1, m1, p2, m2, s2, margin, nd);
        return 0;
    }
    if (t1 == 2) {
        if (t2 == 2) return col_sphere_sphere(p1, s1[0], p2, s2[0], margin, nd);
        if (t2 == 6) return col_sphere_box(p1, s1[0], p2, m2, s2, margin, nd);
        if (t2 == 5) return col_sphere_cyl(p1, s1[0], p2, m2, s2, margin, nd);
        return 0;
    }
    if (t1 == 5) {  // cylinder-box
        if (NEED_DEEP) {
            int d = (margin >= kDeep) ? (int)sat_cyl_box(p1, m1, s1, p2, m2, s2, kDeep)
                                      : (int)(sat_cyl_box(p1, m1, s1, p2, m2, s2, margin) &&
                                              sat_cyl_box(p1, m1, s1, p2, m2, s2, kDeep));
            *nd = d;
            return d;
        }
        return sat_cyl_box(p1, m1, s1, p2, m2, s2, margin) ? 1 : 0;
    }
    // box-box
    if (NEED_DEEP) {
        int d = (margin >= kDeep) ? (int)sat_box_box(p1, m1, s1, p2, m2, s2, kDeep)
                                  : (int)(sat_box_box(p1, m1, s1, p2, m2, s2, margin) &&
                                          sat_box_box(p1, m1, s1, p2, m2, s2, kDeep));
        *nd = d;
        return d;
    }
    return sat_box_box(p1, m1, s1, p2, m2, s2, margin) ? 1 : 0;
}

SSPP_HD double geom_rbound(int type, const double* s) {
    switch (type) {
        case 6: return sqrt(fma(s[2], s[2], fma(s[1], s[1], s[0] * s[0])));
        case 5: return sqrt(fma(s[1], s[1], s[0] * s[0]));
        case 2: return s[0];
        case 3: return s[0] + s[1];
        default: return 0.0;
    }
}

}  // namespace sspd
