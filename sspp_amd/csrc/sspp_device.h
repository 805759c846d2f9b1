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
// profiling counters of the narrowphase paths (SSPP_C2F_STATS builds; slots 10-13)
#if defined(SSPP_CB_STAT) && defined(__HIP_DEVICE_COMPILE__)
#define SSPP_NP_STAT(i) SSPP_CB_STAT(i)
#else
#define SSPP_NP_STAT(i) do { } while (0)
#endif

namespace sspd {

constexpr double kDeep = -1e-3;     // include/Collision.h:93 "col_dist < -1e-3"
// kDeep as a scalar-register value at each use: a 64-bit constant in VALU code is materialised in
// a VGPR pair, which the compiler hoisted out of the pair loops and then spilled to scratch in the
// multi-goal / stacking kernels; through an empty asm it is two s_mov at the use instead
#ifndef SSPP_DEEP_SGPR
#define SSPP_DEEP_SGPR 1
#endif
__host__ __device__ __forceinline__ double in_sgpr(double c) {
#if defined(__HIP_DEVICE_COMPILE__) && SSPP_DEEP_SGPR
    asm volatile("" : "+s"(c));
#endif
    return c;
}
__host__ __device__ __forceinline__ double deep_thr() { return in_sgpr(kDeep); }
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
    // FP32 copies for the filtered scan (sspp_filter.h): the doubles above rounded to nearest
    float fpos[3], fmat[9], fsize[3], frbound;
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
    // FP32 copies for the filtered scan (sspp_filter.h): the doubles above rounded to nearest
    float fmargin, fopos[3], fomat[9], fosize[3], forbound;
};

// fill the FP32 copies of a geom / pair record from its doubles (host, at table creation)
inline void fill_f32(DGeom& g) {
    for (int k = 0; k < 3; ++k) { g.fpos[k] = (float)g.pos[k]; g.fsize[k] = (float)g.size[k]; }
    for (int k = 0; k < 9; ++k) g.fmat[k] = (float)g.mat[k];
    g.frbound = (float)g.rbound;
}
inline void fill_f32(DPair& p) {
    p.fmargin = (float)p.margin;
    for (int k = 0; k < 3; ++k) { p.fopos[k] = (float)p.opos[k]; p.fosize[k] = (float)p.osize[k]; }
    for (int k = 0; k < 9; ++k) p.fomat[k] = (float)p.omat[k];
    p.forbound = (float)p.orbound;
}

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
        double l = (k & 1) ? a[0] : -a[0];  // corner height over the box centre (MuJoCo's ldist)
        l = l + ((k & 2) ? a[1] : -a[1]);
        l = l + ((k & 4) ? a[2] : -a[2]);
        const double t = d0 + l;
        // mjc_PlaneBox: a corner counts unless dist + ldist > margin or ldist > 0 (the corners
        // of the half turned away from the plane never count), at most 4
        if (!(t > margin) && !(l > 0.0) && nc < 4) { nc++; if (t < deep_thr()) ndd++; }
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
    *nd = dist < deep_thr();
    return dist <= margin;  // mjc_PlaneSphere: no contact only when dist > margin
}
SSPP_HD int col_plane_cyl(const double* pp, const double* pm, const double* cp, const double* cm,
                          const double* sz, double margin, int* nd) {
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
    if (p1 > margin) { *nd = 0; return 0; }
    *nd = (p1 < deep_thr()) + (p2 < deep_thr()) + 2 * (pt < deep_thr());
    return 1 + (p2 <= margin) + 2 * (pt <= margin);
}
SSPP_HD int col_sphere_sphere(const double* p1, double r1, const double* p2, double r2,
                              double margin, int* nd) {
    double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
    double dist = sqrt(dot3(d, d)) - (r1 + r2);
    *nd = dist < deep_thr();
    return dist <= margin;  // MuJoCo: no contact only when dist > margin
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
    *nd = dist < deep_thr();
    return dist <= margin;  // MuJoCo: no contact only when dist > margin
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
    *nd = dist < deep_thr();
    return dist <= margin;  // MuJoCo: no contact only when dist > margin
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

// The contact polygon of box_box_deep_count's face case (reference face fi: 0-2 faces of A,
// 3-5 faces of B): the deep vertices of the incident face clipped to the reference rectangle.
// The clipping of bb_clip_count in the reference face's (u, v) frame: the incident corners
// (cu, cv, depth-defining cd), the rectangle |u| <= eu, |v| <= ev.
SSPP_HD int bb_clip_2d(const double* cu, const double* cv, const double* cd, double eu, double ev) {
    int nd = 0;
    // each incident edge clipped to the rectangle |u| <= eu, |v| <= ev (Liang-Barsky with one
    // reciprocal per direction): its entry point, and its exit point when it leaves early
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int e2 = (e + 1) & 3;
        const double du = cu[e2] - cu[e], dv = cv[e2] - cv[e];
        double t0 = 0.0, t1 = 1.0;
        bool ok = true;
        if (du == 0.0) {
            ok = ok && !(cu[e] + eu < 0.0) && !(eu - cu[e] < 0.0);
        } else {
            const double r = 1.0 / du;
            const double ta0 = -(cu[e] + eu) * r, ta1 = (eu - cu[e]) * r;  // u = -eu, u = eu
            const double lo = du > 0.0 ? ta0 : ta1, hi = du > 0.0 ? ta1 : ta0;
            if (lo > t0) t0 = lo;
            if (hi < t1) t1 = hi;
        }
        if (dv == 0.0) {
            ok = ok && !(cv[e] + ev < 0.0) && !(ev - cv[e] < 0.0);
        } else {
            const double r = 1.0 / dv;
            const double tb0 = -(cv[e] + ev) * r, tb1 = (ev - cv[e]) * r;
            const double lo = dv > 0.0 ? tb0 : tb1, hi = dv > 0.0 ? tb1 : tb0;
            if (lo > t0) t0 = lo;
            if (hi < t1) t1 = hi;
        }
        if (ok && t0 <= t1) {
            const double dd = cd[e2] - cd[e];
            if (-fma(t0, dd, cd[e]) < deep_thr()) ++nd;
            if (t1 < 1.0 && -fma(t1, dd, cd[e]) < deep_thr()) ++nd;
        }
    }
    // ... and the rectangle's corners strictly inside the incident parallelogram
    const double au = cu[1] - cu[0], av = cv[1] - cv[0], bu = cu[3] - cu[0], bv = cv[3] - cv[0];
    const double idet = 1.0 / (au * bv - av * bu);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double qu = (q & 1) ? eu : -eu, qv = (q & 2) ? ev : -ev;
        const double wu = qu - cu[0], wv = qv - cv[0];
        const double al = (wu * bv - wv * bu) * idet, be = (au * wv - av * wu) * idet;
        if (al > 0.0 && al < 1.0 && be > 0.0 && be < 1.0) {
            const double d = fma(be, cd[3] - cd[0], fma(al, cd[1] - cd[0], cd[0]));
            if (-d < deep_thr()) ++nd;
        }
    }
    return nd > 0 ? nd : 1;
}


SSPP_HD int bb_clip_count(const double* pa, const double* ma, const double* ea, const double* pb,
                          const double* mb, const double* eb, int fi) {
    double A[3][3], Bc[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) { col3(ma, j, A[j]); col3(mb, j, Bc[j]); }
    auto pick3 = [](int i, double x0, double x1, double x2) { return i == 0 ? x0 : (i == 1 ? x1 : x2); };
    const bool refA = fi < 3;
    const int f = refA ? fi : fi - 3;
    double pR[3], pI[3], eR[3], eI[3], RA[3][3], IA[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        pR[j] = refA ? pa[j] : pb[j]; pI[j] = refA ? pb[j] : pa[j];
        eR[j] = refA ? ea[j] : eb[j]; eI[j] = refA ? eb[j] : ea[j];
#pragma unroll
        for (int i = 0; i < 3; ++i) { RA[j][i] = refA ? A[j][i] : Bc[j][i]; IA[j][i] = refA ? Bc[j][i] : A[j][i]; }
    }
    double n[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) n[c] = pick3(f, RA[0][c], RA[1][c], RA[2][c]);
    const double dRI[3] = {pI[0] - pR[0], pI[1] - pR[1], pI[2] - pR[2]};
    if (dot3(dRI, n) < 0.0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    // incident face: the first most anti-parallel face normal of the other box
    int k = 0;
    double kb = fabs(dot3(IA[0], n));
    { const double v = fabs(dot3(IA[1], n)); if (v > kb) { kb = v; k = 1; } }
    { const double v = fabs(dot3(IA[2], n)); if (v > kb) { kb = v; k = 2; } }
    const int k1 = k == 2 ? 0 : k + 1, k2 = k == 0 ? 2 : k - 1;
    const int ta = f == 2 ? 0 : f + 1, tb = f == 0 ? 2 : f - 1;
    double Ik[3], Ik1[3], Ik2[3], Ta[3], Tb[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        Ik[c] = pick3(k, IA[0][c], IA[1][c], IA[2][c]);
        Ik1[c] = pick3(k1, IA[0][c], IA[1][c], IA[2][c]);
        Ik2[c] = pick3(k2, IA[0][c], IA[1][c], IA[2][c]);
        Ta[c] = pick3(ta, RA[0][c], RA[1][c], RA[2][c]);
        Tb[c] = pick3(tb, RA[0][c], RA[1][c], RA[2][c]);
    }
    const double eIk = pick3(k, eI[0], eI[1], eI[2]), eIk1 = pick3(k1, eI[0], eI[1], eI[2]),
                 eIk2 = pick3(k2, eI[0], eI[1], eI[2]);
    const double sg = dot3(Ik, n) > 0.0 ? -eIk : eIk;
    // incident face corners (cyclic) in the reference face's frame: (u, v) along its two axes,
    // d = depth below the face
    const double off = dot3(pR, n) + pick3(f, eR[0], eR[1], eR[2]);
    double cu[4], cv[4], cd[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        const double c1 = (v == 0 || v == 3) ? eIk1 : -eIk1;
        const double c2 = (v < 2) ? eIk2 : -eIk2;
        double P[3], dp[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            P[i] = fma(c2, Ik2[i], fma(c1, Ik1[i], fma(sg, Ik[i], pI[i])));
            dp[i] = P[i] - pR[i];
        }
        cu[v] = dot3(dp, Ta);
        cv[v] = dot3(dp, Tb);
        cd[v] = off - dot3(P, n);
    }
    const double eu = pick3(ta, eR[0], eR[1], eR[2]), ev = pick3(tb, eR[0], eR[1], eR[2]);
    return bb_clip_2d(cu, cv, cd, eu, ev);
}

// bb_clip_count for two upright boxes (see box_box_deep_count_up): the same operations with the
// products of the rotations' exact zeros dropped.  A z reference face (fi = 2, 5) has the other
// box's z face as incident face; a side reference face has a side face of the other box as
// incident face (its z face is exactly orthogonal to n, so never the most anti-parallel).
SSPP_HD int bb_clip_count_up(const double* pa, const double* ma, const double* ea, const double* pb,
                             const double* mb, const double* eb, int fi) {
    // every operand is selected by value (a pointer select or a run-time index into these
    // register-resident arrays would put them in scratch memory)
    const bool refA = fi < 3;
    const int f = refA ? fi : fi - 3;
    const double R0 = refA ? ma[0] : mb[0], R1 = refA ? ma[1] : mb[1], R3 = refA ? ma[3] : mb[3],
                 R4 = refA ? ma[4] : mb[4], R8 = refA ? ma[8] : mb[8];
    const double I0 = refA ? mb[0] : ma[0], I1 = refA ? mb[1] : ma[1], I3 = refA ? mb[3] : ma[3],
                 I4 = refA ? mb[4] : ma[4], I8 = refA ? mb[8] : ma[8];
    const double pR0 = refA ? pa[0] : pb[0], pR1 = refA ? pa[1] : pb[1], pR2 = refA ? pa[2] : pb[2];
    const double pI0 = refA ? pb[0] : pa[0], pI1 = refA ? pb[1] : pa[1], pI2 = refA ? pb[2] : pa[2];
    const double eR0 = refA ? ea[0] : eb[0], eR1 = refA ? ea[1] : eb[1], eR2 = refA ? ea[2] : eb[2];
    const double eI0 = refA ? eb[0] : ea[0], eI1 = refA ? eb[1] : ea[1], eI2 = refA ? eb[2] : ea[2];
    const double dRI0 = pI0 - pR0, dRI1 = pI1 - pR1, dRI2 = pI2 - pR2;
    double cu[4], cv[4], cd[4], eu, ev;
    if (f == 2) {
        double n2 = R8;
        if (dRI2 * n2 < 0.0) n2 = -n2;
        const double sg = I8 * n2 > 0.0 ? -eI2 : eI2;
        const double off = pR2 * n2 + eR2;
        const double P2 = fma(sg, I8, pI2);
        const double cdz = off - P2 * n2;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const double c1 = (v == 0 || v == 3) ? eI0 : -eI0;
            const double c2 = (v < 2) ? eI1 : -eI1;
            const double P0 = fma(c2, I1, fma(c1, I0, pI0));
            const double P1 = fma(c2, I4, fma(c1, I3, pI1));
            const double dp0 = P0 - pR0, dp1 = P1 - pR1;
            cu[v] = fma(dp1, R3, dp0 * R0);
            cv[v] = fma(dp1, R4, dp0 * R1);
            cd[v] = cdz;
        }
        eu = eR0;
        ev = eR1;
    } else {
        double n0 = f ? R1 : R0, n1 = f ? R4 : R3;
        if (fma(dRI1, n1, dRI0 * n0) < 0.0) { n0 = -n0; n1 = -n1; }
        const double d0 = fma(I3, n1, I0 * n0), d1 = fma(I4, n1, I1 * n0);
        const bool k = fabs(d1) > fabs(d0);
        // Ik: the incident horizontal axis k; Hh: the other horizontal axis (coefficient c1 for
        // k = 0, c2 for k = 1); the vertical axis takes the other coefficient
        const double Ik0 = k ? I1 : I0, Ik1 = k ? I4 : I3;
        const double Hh0 = k ? I0 : I1, Hh1 = k ? I3 : I4;
        const double eIk = k ? eI1 : eI0;
        const double sg = (k ? d1 : d0) > 0.0 ? -eIk : eIk;
        const double eK1 = k ? eI2 : eI1, eK2 = k ? eI0 : eI2;  // eI[k1], eI[k2]
        const double off = fma(pR1, n1, pR0 * n0) + (f ? eR1 : eR0);
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const double c1 = (v == 0 || v == 3) ? eK1 : -eK1;
            const double c2 = (v < 2) ? eK2 : -eK2;
            const double ch = k ? c2 : c1, cz = k ? c1 : c2;
            const double P0 = fma(ch, Hh0, fma(sg, Ik0, pI0));
            const double P1 = fma(ch, Hh1, fma(sg, Ik1, pI1));
            const double P2 = fma(cz, I8, pI2);
            const double dp0 = P0 - pR0, dp1 = P1 - pR1, dp2 = P2 - pR2;
            const double hz = dp2 * R8;  // along the reference box's z axis
            // f = 0: Ta = axis 1 (horizontal), Tb = z;  f = 1: Ta = z, Tb = axis 0 (horizontal)
            const double hh = f == 0 ? fma(dp1, R4, dp0 * R1) : fma(dp1, R3, dp0 * R0);
            cu[v] = f == 0 ? hh : hz;
            cv[v] = f == 0 ? hz : hh;
            cd[v] = off - fma(P1, n1, P0 * n0);
        }
        eu = f == 0 ? eR1 : eR2;
        ev = f == 0 ? eR2 : eR0;
    }
    return bb_clip_2d(cu, cv, cd, eu, ev);
}

// Box-box deep contacts (TaskSpacePlanner cost: Collision.h:89-101 adds one term per contact
// with dist < -1e-3, and MuJoCo's box-box collider reports up to 8).  One pass:
// * the 15-axis SAT at thr = -1e-3 exactly as sat_box_box (returns 0 at the first axis whose
//   separation reaches it: not deep);
// * otherwise MuJoCo-style: an edge-edge axis whose separation exceeds every face
//   axis's by more than 1e-12 gives one contact; else the face axis of least penetration makes
//   that face the reference face and the most anti-parallel face of the other box the incident
//   face, and the contacts are the vertices of the incident face clipped to the reference face's
//   rectangle (<= 8), dist = -(depth below the reference face): every incident edge's clipped
//   segment (Liang-Barsky, boundary inclusive) gives its entry point and, if it leaves early,
//   its exit point; reference corners strictly inside the incident face are vertices too.
// Returns the number of those with dist < -1e-3, at least 1 (no clipped point is deeper than the
// SAT depth).  Every array is indexed with compile-time indices (run-time choices are selects),
// so everything stays in registers.
// box_box_deep_class: the decision part — -1 not deep, 6 one contact (edge-edge axis), 0..5 the
// reference face fi whose contact polygon bb_clip_count counts; box_box_deep_count composes the
// two (k_tsp's deferred form runs the polygon later, for the compacted deep items only).
SSPP_HD int box_box_deep_class(const double* pa, const double* ma, const double* ea,
                               const double* pb, const double* mb, const double* eb) {
    double A[3][3], Bc[3][3], T[3], t[3], R[3][3], AR[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) { col3(ma, j, A[j]); col3(mb, j, Bc[j]); }
    T[0] = pb[0] - pa[0]; T[1] = pb[1] - pa[1]; T[2] = pb[2] - pa[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        t[i] = dot3(A[i], T);
#pragma unroll
        for (int j = 0; j < 3; ++j) { R[i][j] = dot3(A[i], Bc[j]); AR[i][j] = fabs(R[i][j]); }
    }
    double best_face = -1e300;
    int fi = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // faces of A
        const double rb = fma(eb[2], AR[i][2], fma(eb[1], AR[i][1], eb[0] * AR[i][0]));
        const double sep = fabs(t[i]) - (ea[i] + rb);
        if (sep >= deep_thr()) return -1;
        if (sep > best_face) { best_face = sep; fi = i; }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // faces of B
        const double pr = fabs(fma(t[2], R[2][j], fma(t[1], R[1][j], t[0] * R[0][j])));
        const double ra = fma(ea[2], AR[2][j], fma(ea[1], AR[1][j], ea[0] * AR[0][j]));
        const double sep = pr - (ra + eb[j]);
        if (sep >= deep_thr()) return -1;
        if (sep > best_face) { best_face = sep; fi = 3 + j; }
    }
    bool edge = false;  // some edge axis separates by more than best_face + 1e-12
    const double fthr = best_face + 1e-12;
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // edge x edge
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double v0 = R[0][j], v1 = R[1][j], v2 = R[2][j];
            double L[3];
            if (i == 0) { L[0] = 0.0; L[1] = -v2; L[2] = v1; }
            else if (i == 1) { L[0] = v2; L[1] = 0.0; L[2] = -v0; }
            else { L[0] = -v1; L[1] = v0; L[2] = 0.0; }
            const double len2 = dot3(L, L);
            if (len2 < 1e-12) continue;
            const double pr = fabs(dot3(t, L));
            const double ra = fma(ea[2], fabs(L[2]), fma(ea[1], fabs(L[1]), ea[0] * fabs(L[0])));
            double rb = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double bk[3] = {R[0][k], R[1][k], R[2][k]};
                rb = fma(eb[k], fabs(dot3(bk, L)), rb);
            }
            const double num = pr - (ra + rb), len = sqrt(len2);
            if (num >= deep_thr() * len) return -1;
            edge = edge || num > fthr * len;
        }
    }
    return edge ? 6 : fi;
}
SSPP_HD int box_box_deep_count(const double* pa, const double* ma, const double* ea,
                               const double* pb, const double* mb, const double* eb) {
    const int c = box_box_deep_class(pa, ma, ea, pb, mb, eb);
    if (c < 0) return 0;
    if (c == 6) return 1;
#ifdef SSPP_NO_MANIFOLD  // measurement variant only: the SAT decision without the contact polygon
    return 1;
#endif
    return bb_clip_count(pa, ma, ea, pb, mb, eb, c);
}

// box_box_deep_count for two UPRIGHT boxes: each rotation has m[2] = m[5] = m[6] = m[7] = 0
// exactly (z axis = world z up to its sign and length, x / y axes horizontal), which holds for a
// yaw-only mover (TaskSpacePlanner, utility.h:198-206) against z-aligned static boxes.  Then
// R = A^T B has R02 = R12 = R20 = R21 = 0 exactly and every product with those zeros drops out
// of box_box_deep_count's fma chains without changing any other rounding (adding an exact zero
// is exact), so this returns bit for bit what box_box_deep_count returns on such boxes, with a
// quarter of the SAT arithmetic: the 8 non-degenerate edge axes are z (4), A's and B's
// horizontal axes (2 + 2); the ninth (A_z x B_z) has length 0 and is skipped there too.
SSPP_HD int box_box_deep_class_up(const double* pa, const double* ma, const double* ea,
                                  const double* pb, const double* mb, const double* eb) {
    const double T0 = pb[0] - pa[0], T1 = pb[1] - pa[1], T2 = pb[2] - pa[2];
    const double t0 = fma(ma[3], T1, ma[0] * T0), t1 = fma(ma[4], T1, ma[1] * T0), t2 = ma[8] * T2;
    const double R00 = fma(ma[3], mb[3], ma[0] * mb[0]), R01 = fma(ma[3], mb[4], ma[0] * mb[1]);
    const double R10 = fma(ma[4], mb[3], ma[1] * mb[0]), R11 = fma(ma[4], mb[4], ma[1] * mb[1]);
    const double R22 = ma[8] * mb[8];
    const double A00 = fabs(R00), A01 = fabs(R01), A10 = fabs(R10), A11 = fabs(R11), A22 = fabs(R22);
    double best_face, sep;
    int fi;
    // faces of A
    sep = fabs(t0) - (ea[0] + fma(eb[1], A01, eb[0] * A00));
    if (sep >= deep_thr()) return -1;
    best_face = sep; fi = 0;
    sep = fabs(t1) - (ea[1] + fma(eb[1], A11, eb[0] * A10));
    if (sep >= deep_thr()) return -1;
    if (sep > best_face) { best_face = sep; fi = 1; }
    sep = fabs(t2) - (ea[2] + eb[2] * A22);
    if (sep >= deep_thr()) return -1;
    if (sep > best_face) { best_face = sep; fi = 2; }
    // faces of B
    sep = fabs(fma(t1, R10, t0 * R00)) - (fma(ea[1], A10, ea[0] * A00) + eb[0]);
    if (sep >= deep_thr()) return -1;
    if (sep > best_face) { best_face = sep; fi = 3; }
    sep = fabs(fma(t1, R11, t0 * R01)) - (fma(ea[1], A11, ea[0] * A01) + eb[1]);
    if (sep >= deep_thr()) return -1;
    if (sep > best_face) { best_face = sep; fi = 4; }
    sep = fabs(t2 * R22) - (ea[2] * A22 + eb[2]);
    if (sep >= deep_thr()) return -1;
    if (sep > best_face) { best_face = sep; fi = 5; }
    bool edge = false;
    const double fthr = best_face + 1e-12;
    // one edge axis: separation numerator num against thr * |L|, len2 = |L|^2 as formed there
    auto ax = [&](double len2, double pr, double ra, double rb) -> int {
        if (len2 < 1e-12) return 1;
        const double num = pr - (ra + rb), len = sqrt(len2);
        if (num >= deep_thr() * len) return 0;
        edge = edge || num > fthr * len;
        return 1;
    };
    // (i, j) = (0, 0), (0, 1): L = (0, -0, R1j), along z
    if (!ax(R10 * R10, fabs(t2 * R10), ea[2] * fabs(R10), eb[2] * fabs(R22 * R10))) return -1;
    if (!ax(R11 * R11, fabs(t2 * R11), ea[2] * fabs(R11), eb[2] * fabs(R22 * R11))) return -1;
    // (0, 2): L = (0, -R22, 0)
    if (!ax(R22 * R22, fabs(t1 * -R22), ea[1] * A22,
            fma(eb[1], fabs(R11 * -R22), eb[0] * fabs(R10 * -R22)))) return -1;
    // (1, 0), (1, 1): L = (0, 0, -R0j), along z
    if (!ax(R00 * R00, fabs(t2 * -R00), ea[2] * A00, eb[2] * fabs(R22 * -R00))) return -1;
    if (!ax(R01 * R01, fabs(t2 * -R01), ea[2] * A01, eb[2] * fabs(R22 * -R01))) return -1;
    // (1, 2): L = (R22, 0, -0)
    if (!ax(R22 * R22, fabs(t0 * R22), ea[0] * A22,
            fma(eb[1], fabs(R01 * R22), eb[0] * fabs(R00 * R22)))) return -1;
    // (2, 0), (2, 1): L = (-R1j, R0j, 0), horizontal; (2, 2) has L = 0
    if (!ax(fma(R00, R00, -R10 * -R10), fabs(fma(t1, R00, t0 * -R10)), fma(ea[1], A00, ea[0] * A10),
            fma(eb[1], fabs(fma(R11, R00, R01 * -R10)), eb[0] * fabs(fma(R10, R00, R00 * -R10))))) return -1;
    if (!ax(fma(R01, R01, -R11 * -R11), fabs(fma(t1, R01, t0 * -R11)), fma(ea[1], A01, ea[0] * A11),
            fma(eb[1], fabs(fma(R11, R01, R01 * -R11)), eb[0] * fabs(fma(R10, R01, R00 * -R11))))) return -1;
    return edge ? 6 : fi;
}
SSPP_HD int box_box_deep_count_up(const double* pa, const double* ma, const double* ea,
                                  const double* pb, const double* mb, const double* eb) {
    const int c = box_box_deep_class_up(pa, ma, ea, pb, mb, eb);
    if (c < 0) return 0;
    if (c == 6) return 1;
#ifdef SSPP_NO_MANIFOLD
    return 1;
#endif
    return bb_clip_count_up(pa, ma, ea, pb, mb, eb, c);
}

// Both rotations upright (see box_box_deep_count_up)?
SSPP_HD bool upright3(const double* m) {
    return m[2] == 0.0 && m[5] == 0.0 && m[6] == 0.0 && m[7] == 0.0;
}

// ---------------------------------------------------------------- cylinder-box, exact
// The signed distance of two convex bodies is the maximum over directions n of their
// separation along n (negative: minus the penetration depth), attained at the normal of the
// closest feature pair.  A cylinder has a cap disc, a lateral surface and two rim circles; a
// box has faces, edges and vertices.  Every feature pair that can be closest has its normal
// in one of these families:
//   (a) box face normals b_k           (b) the cylinder axis a      (c) a x b_k
//   (d) perp_a(w - c) for each box vertex w (lateral surface vs vertex or vertical edge)
//   (f) w - (rim point nearest w), both rims (rim circle vs vertex, separated bodies)
//   (e) rim circle vs box edge: the common normal of a circle and a line = the normal of the
//       rim's projection along the edge (an ellipse) at its point nearest the projected edge
//       (Eberly's robust bisection); for a penetration depth also the ellipse's other
//       locally-nearest point (the deepest point of the Minkowski difference can be one).
// Every direction gives a lower bound of the signed distance, so "dist < thr" is exact when
// no candidate separates by >= thr.  (a)-(c) are the finite SAT axes and go first; the rest
// runs only when those cannot separate.
struct CylBox {
    double a[3];     // cylinder axis (world)
    double T[3];     // box centre - cylinder centre
    double B[3][3];  // box axes (rows)
    double e[3];     // box half extents
    double R, H;     // cylinder radius, half height
};

SSPP_HD CylBox make_cylbox(const double* pa, const double* ma, const double* sz, const double* pb,
                           const double* mb, const double* eb) {
    CylBox c;
    col3(ma, 2, c.a);
#pragma unroll
    for (int j = 0; j < 3; ++j) { col3(mb, j, c.B[j]); c.e[j] = eb[j]; }
    c.T[0] = pb[0] - pa[0]; c.T[1] = pb[1] - pa[1]; c.T[2] = pb[2] - pa[2];
    c.R = sz[0]; c.H = sz[1];
    return c;
}

// true iff the separation along L (any length) is >= thr
SSPP_HD bool cb_sep(const CylBox& c, const double* L, double thr) {
    const double len2 = dot3(L, L);
    if (!(len2 > 1e-30)) return false;
    const double aL = dot3(c.a, L);
    const double rr = len2 - aL * aL;
    const double rc = fma(c.H, fabs(aL), c.R * sqrt(rr > 0.0 ? rr : 0.0));
    double rb = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) rb = fma(c.e[k], fabs(dot3(c.B[k], L)), rb);
    const double num = fabs(dot3(c.T, L)) - (rc + rb);
    return thr == 0.0 ? num >= 0.0 : num >= thr * sqrt(len2);
}

// families (a)-(c): box faces, cylinder axis, axis x box edges
SSPP_HD bool cb_base_sep(const CylBox& c, double thr) {
#pragma unroll
    for (int ax = 0; ax < 7; ++ax) {
        double L[3];
        if (ax < 3) { L[0] = c.B[ax][0]; L[1] = c.B[ax][1]; L[2] = c.B[ax][2]; }
        else if (ax == 3) { L[0] = c.a[0]; L[1] = c.a[1]; L[2] = c.a[2]; }
        else {
            const double* b = c.B[ax - 4];
            L[0] = c.a[1] * b[2] - c.a[2] * b[1];
            L[1] = c.a[2] * b[0] - c.a[0] * b[2];
            L[2] = c.a[0] * b[1] - c.a[1] * b[0];
            if (dot3(L, L) < 1e-20) continue;  // edge parallel to the axis: family (d)
        }
        if (cb_sep(c, L, thr)) return true;
    }
    return false;
}

// Eberly's F(s) = (r0 z0 / (s + r0))^2 + (z1 / (s + 1))^2 - 1
SSPP_HD double ell_F(double r0, double z0, double z1, double s) {
    const double t0 = (r0 * z0) / (s + r0), t1 = z1 / (s + 1.0);
    return fma(t1, t1, t0 * t0) - 1.0;
}
// Root of F on (lo, hi) with sign(F(lo)) = sgn_lo, F convex and monotone there: Newton steps
// safeguarded by the shrinking bracket (bisection whenever a step leaves it), <= 48 iterations.
SSPP_HD double ell_bisect(double r0, double z0, double z1, double lo, double hi, double sgn_lo) {
    const double n0 = r0 * z0;
    double s = 0.5 * (lo + hi);
#pragma unroll 1
    for (int i = 0; i < 48; ++i) {
        const double a0 = s + r0, a1 = s + 1.0;
        const double t0 = n0 / a0, t1 = z1 / a1;
        const double f = fma(t1, t1, t0 * t0) - 1.0;
        if (f == 0.0) break;
        if ((f > 0.0) == (sgn_lo > 0.0)) lo = s; else hi = s;
        const double fp = -2.0 * ((t0 * t0) / a0 + (t1 * t1) / a1);
        double sn = s - f / fp;
        if (!(sn > lo && sn < hi)) sn = 0.5 * (lo + hi);
        if (sn == s) break;
        s = sn;
    }
    return s;
}
// nearest point (x0, x1) of the ellipse x0^2/e0^2 + x1^2/e1^2 = 1 (e0 >= e1 > 0) to (y0, y1) >= 0
SSPP_HD void ellipse_q1(double e0, double e1, double y0, double y1, double* x0, double* x1) {
    if (y1 > 0.0) {
        if (y0 > 0.0) {
            const double z0 = y0 / e0, z1 = y1 / e1;
            const double g = fma(z1, z1, z0 * z0) - 1.0;
            if (g != 0.0) {
                const double q = e0 / e1, r0 = q * q, n0 = r0 * z0;
                const double hi = g < 0.0 ? 0.0 : sqrt(fma(z1, z1, n0 * n0)) - 1.0;
                const double s = ell_bisect(r0, z0, z1, z1 - 1.0, hi, 1.0);
                *x0 = (r0 * y0) / (s + r0);
                *x1 = y1 / (s + 1.0);
            } else {
                *x0 = y0; *x1 = y1;
            }
        } else {
            *x0 = 0.0; *x1 = e1;
        }
    } else {
        const double num = e0 * y0, den = e0 * e0 - e1 * e1;
        if (num < den) {
            const double xd = num / den;
            *x0 = e0 * xd;
            *x1 = e1 * sqrt(1.0 - xd * xd);
        } else {
            *x0 = e0; *x1 = 0.0;
        }
    }
}

// family (e) axis from an ellipse point (x, y) in the (u1, u2) frame: the ellipse normal
SSPP_HD bool cb_ell_axis(const CylBox& c, const double* u1, const double* u2, double x, double y,
                         double e0, double e1, double thr) {
    const double nx = x / (e0 * e0), ny = y / (e1 * e1);
    const double L[3] = {fma(ny, u2[0], nx * u1[0]), fma(ny, u2[1], nx * u1[1]), fma(ny, u2[2], nx * u1[2])};
    return cb_sep(c, L, thr);
}

// The ellipse's other locally-nearest points to p = (px, py) (penetration depth only): the
// roots of F on (-r0, -1), where F is convex — its minimiser by bisection on F', then one
// bisection on each side when the minimum is negative; exact-zero coordinates by hand.
SSPP_HD bool cb_ell_other(const CylBox& c, const double* u1, const double* u2, double px, double py,
                          double e0, double e1, double thr) {
    const double y0 = fabs(px), y1 = fabs(py), sx = px < 0.0 ? -1.0 : 1.0, sy = py < 0.0 ? -1.0 : 1.0;
    const double den = e0 * e0 - e1 * e1;
    if (y1 == 0.0) {  // on the major axis: (+-e0, 0) and the off-axis pair
        if (cb_ell_axis(c, u1, u2, e0, 0.0, e0, e1, thr)) return true;
        if (e0 * y0 < den) {
            const double xd = (e0 * y0) / den, x0 = sx * e0 * xd, x1 = e1 * sqrt(1.0 - xd * xd);
            if (cb_ell_axis(c, u1, u2, x0, x1, e0, e1, thr) || cb_ell_axis(c, u1, u2, x0, -x1, e0, e1, thr))
                return true;
        }
        return false;
    }
    if (y0 == 0.0) {  // on the minor axis: (0, +-e1) and the off-axis pair
        if (cb_ell_axis(c, u1, u2, 0.0, e1, e0, e1, thr)) return true;
        if (e1 * y1 < den) {
            const double x1 = -sy * (e1 * e1 * y1) / den, t = x1 / e1;
            const double x0 = e0 * sqrt(1.0 - t * t);
            if (cb_ell_axis(c, u1, u2, x0, x1, e0, e1, thr) || cb_ell_axis(c, u1, u2, -x0, x1, e0, e1, thr))
                return true;
        }
        return false;
    }
    const double z0 = y0 / e0, z1 = y1 / e1, q = e0 / e1, r0 = q * q, n0 = r0 * z0;
    // minimiser of F on (-r0, -1): root of the decreasing D(s) = n0^2/(s+r0)^3 + z1^2/(s+1)^3,
    // safeguarded Newton as in ell_bisect
    double lo = -r0, hi = -1.0, s = 0.5 * (lo + hi);
#pragma unroll 1
    for (int i = 0; i < 48; ++i) {
        const double a0 = s + r0, a1 = s + 1.0;
        const double q0 = (n0 * n0) / (a0 * a0 * a0), q1 = (z1 * z1) / (a1 * a1 * a1);
        const double D = q0 + q1;
        if (D == 0.0) break;
        if (D > 0.0) lo = s; else hi = s;
        const double Dp = -3.0 * (q0 / a0 + q1 / a1);
        double sn = s - D / Dp;
        if (!(sn > lo && sn < hi)) sn = 0.5 * (lo + hi);
        if (sn == s) break;
        s = sn;
    }
    if (!(ell_F(r0, z0, z1, s) < 0.0)) return false;
    const double sa = ell_bisect(r0, z0, z1, -r0, s, 1.0);
    const double sb = ell_bisect(r0, z0, z1, s, -1.0, -1.0);
    const double ss[2] = {sa, sb};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const double x0 = sx * ((r0 * y0) / (ss[k] + r0)), x1 = sy * (y1 / (ss[k] + 1.0));
        if (cb_ell_axis(c, u1, u2, x0, x1, e0, e1, thr)) return true;
    }
    return false;
}

// families (d), (f) and (e); all_roots adds (e)'s non-global critical points
SSPP_HD bool cb_ext_sep(const CylBox& c, double thr, bool all_roots) {
#pragma unroll 1
    for (int v = 0; v < 8; ++v) {  // (d), (f): box vertices
        const double s0 = (v & 1) ? c.e[0] : -c.e[0], s1 = (v & 2) ? c.e[1] : -c.e[1],
                     s2 = (v & 4) ? c.e[2] : -c.e[2];
        double w[3], u[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) w[i] = fma(s2, c.B[2][i], fma(s1, c.B[1][i], fma(s0, c.B[0][i], c.T[i])));
        const double z = dot3(c.a, w);
#pragma unroll
        for (int i = 0; i < 3; ++i) u[i] = w[i] - z * c.a[i];
        const double uu = dot3(u, u);
        if (!(uu > 1e-30)) continue;
        if (cb_sep(c, u, thr)) return true;
        const double f = 1.0 - c.R / sqrt(uu);
#pragma unroll 1
        for (int r = 0; r < 2; ++r) {
            const double dz = z - (r ? c.H : -c.H);
            const double L[3] = {fma(dz, c.a[0], f * u[0]), fma(dz, c.a[1], f * u[1]), fma(dz, c.a[2], f * u[2])};
            if (cb_sep(c, L, thr)) return true;
        }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // (e): rim circles vs box edges along b_j (unrolled: static indices)
        const double* e = c.B[j];
        double u1[3] = {c.a[1] * e[2] - c.a[2] * e[1], c.a[2] * e[0] - c.a[0] * e[2], c.a[0] * e[1] - c.a[1] * e[0]};
        const double S2 = dot3(u1, u1);
        if (S2 < 1e-20) continue;  // edge parallel to the axis: family (d)
        const double iS = 1.0 / sqrt(S2);
        u1[0] *= iS; u1[1] *= iS; u1[2] *= iS;
        const double u2[3] = {e[1] * u1[2] - e[2] * u1[1], e[2] * u1[0] - e[0] * u1[2], e[0] * u1[1] - e[1] * u1[0]};
        const double e0 = c.R, e1 = c.R * fabs(dot3(c.a, e));
        const int k1 = j == 2 ? 0 : j + 1, k2 = j == 0 ? 2 : j - 1;
#pragma unroll 1
        for (int q = 0; q < 4; ++q) {
            const double s1 = (q & 1) ? c.e[k1] : -c.e[k1], s2 = (q & 2) ? c.e[k2] : -c.e[k2];
            double w0[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) w0[i] = fma(s2, c.B[k2][i], fma(s1, c.B[k1][i], c.T[i]));
#pragma unroll 1
            for (int r = 0; r < 2; ++r) {
                const double hs = r ? c.H : -c.H;
                const double d[3] = {w0[0] - hs * c.a[0], w0[1] - hs * c.a[1], w0[2] - hs * c.a[2]};
                const double px = dot3(d, u1), py = dot3(d, u2);
                if (e1 < 1e-9 * e0) {  // the rim's plane contains the edge: a segment
                    if (fabs(px) <= e0) continue;  // normal = the axis, family (b)
                    const double ex = px - (px < 0.0 ? -e0 : e0);
                    const double L[3] = {fma(py, u2[0], ex * u1[0]), fma(py, u2[1], ex * u1[1]), fma(py, u2[2], ex * u1[2])};
                    if (cb_sep(c, L, thr)) return true;
                    continue;
                }
                double x0, x1;
                ellipse_q1(e0, e1, fabs(px), fabs(py), &x0, &x1);
                if (cb_ell_axis(c, u1, u2, px < 0.0 ? -x0 : x0, py < 0.0 ? -x1 : x1, e0, e1, thr)) return true;
                if (all_roots && cb_ell_other(c, u1, u2, px, py, e0, e1, thr)) return true;
            }
        }
    }
    return false;
}

// dist < thr (thr >= 0: MuJoCo's contact test with margin thr)
// Witnesses (they only prove overlap; a separation always needs the candidate directions).
// Nearest point of the box to x, and whether x lies strictly inside it.
SSPP_HD bool cb_proj_box(const CylBox& c, const double* e, const double* x, double* y) {
    const double d[3] = {x[0] - c.T[0], x[1] - c.T[1], x[2] - c.T[2]};
    double l[3];
    bool in = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double t = dot3(c.B[k], d);
        if (!(t < e[k] && t > -e[k])) in = false;
        l[k] = t > e[k] ? e[k] : (t < -e[k] ? -e[k] : t);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = fma(l[2], c.B[2][i], fma(l[1], c.B[1][i], fma(l[0], c.B[0][i], c.T[i])));
    return in;
}
// Nearest point of the cylinder (radius R, half height H, at the origin) to x, and whether x
// lies strictly inside it.
SSPP_HD bool cb_proj_cyl(const CylBox& c, double R, double H, const double* x, double* y) {
    const double z = dot3(c.a, x);
    const double r[3] = {x[0] - z * c.a[0], x[1] - z * c.a[1], x[2] - z * c.a[2]};
    const double rr = dot3(r, r);
    const bool in = rr < R * R && z < H && z > -H;
    const double zc = z > H ? H : (z < -H ? -H : z);
    const double f = rr > R * R ? R / sqrt(rr) : 1.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) y[i] = fma(zc, c.a[i], f * r[i]);
    return in;
}
// dist < thr (thr >= 0) proven by alternating projections: x on the cylinder strictly inside
// the box (interiors overlap), or x on the cylinder and y on the box closer than thr.
SSPP_HD bool cb_touch_witness(const CylBox& c, double thr) {
    double x[3], y[3] = {c.T[0], c.T[1], c.T[2]};
#pragma unroll 1
    for (int it = 0; it < 3; ++it) {
        cb_proj_cyl(c, c.R, c.H, y, x);
        if (cb_proj_box(c, c.e, x, y)) return true;
        const double d[3] = {x[0] - y[0], x[1] - y[1], x[2] - y[2]};
        if (thr > 0.0 && dot3(d, d) < thr * thr) return true;
    }
    return false;
}
// dist < -dl proven by a point of the cylinder shrunk by dl strictly inside the box, or of the
// box shrunk by dl strictly inside the cylinder: (A (-) ball) - B lies in (A - B) (-) ball.
SSPP_HD bool cb_deep_witness(const CylBox& c, double dl) {
    double x[3], y[3];
    if (c.R > dl && c.H > dl) {
        y[0] = c.T[0]; y[1] = c.T[1]; y[2] = c.T[2];
#pragma unroll 1
        for (int it = 0; it < 3; ++it) {
            cb_proj_cyl(c, c.R - dl, c.H - dl, y, x);
            if (cb_proj_box(c, c.e, x, y)) return true;
        }
    }
    if (c.e[0] > dl && c.e[1] > dl && c.e[2] > dl) {
        const double es[3] = {c.e[0] - dl, c.e[1] - dl, c.e[2] - dl};
        x[0] = 0.0; x[1] = 0.0; x[2] = 0.0;
#pragma unroll 1
        for (int it = 0; it < 3; ++it) {
            cb_proj_box(c, es, x, y);
            if (cb_proj_cyl(c, c.R, c.H, y, x)) return true;
        }
    }
    return false;
}

// The candidate-direction search in the box's frame (box axes = identity): the cylinder-box pair
// then travels as 12 doubles, which fit the argument registers of an out-of-line call.
SSPP_HD CylBox cb_box_frame(const CylBox& c) {
    CylBox b;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        b.T[k] = dot3(c.B[k], c.T);
        b.a[k] = dot3(c.B[k], c.a);
        b.e[k] = c.e[k];
#pragma unroll
        for (int i = 0; i < 3; ++i) b.B[k][i] = k == i ? 1.0 : 0.0;
    }
    b.R = c.R; b.H = c.H;
    return b;
}
// The candidate directions past the SAT axes and the witnesses, in the box's frame (box axes =
// identity), from 12 doubles (so it fits the argument registers of a call).
SSPP_HD bool cb_ext_overlap(double T0, double T1, double T2, double a0, double a1, double a2,
                            double e0, double e1, double e2, double R, double H, double thr) {
    CylBox b;
    b.T[0] = T0; b.T[1] = T1; b.T[2] = T2;
    b.a[0] = a0; b.a[1] = a1; b.a[2] = a2;
    b.e[0] = e0; b.e[1] = e1; b.e[2] = e2;
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int i = 0; i < 3; ++i) b.B[k][i] = k == i ? 1.0 : 0.0;
    b.R = R; b.H = H;
    SSPP_NP_STAT(12);
    return !cb_ext_sep(b, thr, thr < 0.0);
}
// Out of line, for kernels at their register budget (k_tsp): reached only by the pairs neither
// the SAT axes nor a witness decide (well under 0.1 % of the multi-goal bench's tests).
__host__ __device__ inline __attribute__((noinline)) bool cb_ext_overlap_call(
    double T0, double T1, double T2, double a0, double a1, double a2, double e0, double e1,
    double e2, double R, double H, double thr) {
    return cb_ext_overlap(T0, T1, T2, a0, a1, a2, e0, e1, e2, R, H, thr);
}

// Cylinder (A) vs box (B) when the cylinder's axis is vertical (ma[2] = ma[5] = 0) and the box
// is upright (mb[2] = mb[5] = mb[6] = mb[7] = 0): both are prisms along z, so their Minkowski
// difference is (box rectangle + disc of radius R) x [-(ez + H), ez + H] and the signed distance
// is that of the centre offset c (box frame) to it: d_xy = (signed distance of c_xy to the
// rectangle) - R, d_z = |c_z| - (H + ez); sd = sqrt(d_xy^2 + d_z^2) when both are positive, else
// max(d_xy, d_z).  Exact (the same decision as the candidate-direction search up to rounding);
// the oracle runs the same operations (oracle/sspp_oracle.c::cb_upright_sd), so both decide
// every pair identically.  A yaw-only TaskSpacePlanner mover keeps a vertical cylinder vertical.
SSPP_HD bool cyl_vertical(const double* m) { return m[2] == 0.0 && m[5] == 0.0; }
SSPP_HD double cb_upright_sd(const double* pa, const double* sz, const double* pb, const double* mb,
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

// cylinder (A) vs box (B): signed distance < thr (thr = margin >= 0, or kDeep for a deep
// contact).  The 7 SAT axes (world frame) separate most pairs; the rest runs in the box frame:
// witnesses prove most overlaps, the candidate directions (OUTLINE: as a call) decide the rest.
template <bool OUTLINE>
SSPP_HD bool cyl_box_overlap(const double* pa, const double* ma, const double* sz, const double* pb,
                             const double* mb, const double* eb, double thr) {
    const CylBox c = make_cylbox(pa, ma, sz, pb, mb, eb);
    SSPP_NP_STAT(10);
    if (cb_base_sep(c, thr)) return false;
    SSPP_NP_STAT(11);
    const CylBox b = cb_box_frame(c);
    if (thr < 0.0 ? cb_deep_witness(b, -thr) : cb_touch_witness(b, thr)) return true;
    if (OUTLINE)
        return cb_ext_overlap_call(b.T[0], b.T[1], b.T[2], b.a[0], b.a[1], b.a[2], b.e[0], b.e[1], b.e[2],
                                   b.R, b.H, thr);
    return cb_ext_overlap(b.T[0], b.T[1], b.T[2], b.a[0], b.a[1], b.a[2], b.e[0], b.e[1], b.e[2],
                          b.R, b.H, thr);
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
// CB = false compiles out the cylinder-box code (only for scenes without such pairs); OUTLINE
// calls the rare cylinder-box candidate search out of line.
// DEFER (feasibility only): a cylinder-box pair (already past the bounding-sphere test) returns
// -1, undecided, without any narrowphase; the caller settles it later with the exact test
// (k_sspp_c2f -> k_sspp_cbfix), so its pair loop carries none of that code.
// UP (deep counts only): every box-box pair is upright (box_box_deep_count_up; host-checked).
// CB: 0 no cylinder-box pairs (code compiled out), 1 the exact test (vertical-cylinder /
// upright-box pairs take cb_upright_sd), 2 every cylinder-box pair is vertical / upright
// (host-checked): cb_upright_sd only, the candidate search compiled out.
template <bool NEED_DEEP, int CB = 1, bool OUTLINE = false, bool DEFER = false, bool UP = false>
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
    if (t1 == 5) {  // cylinder-box: exact signed distance test, one contact (MuJoCo's convex collider)
        if (!CB) return 0;
        if (CB == 2 || (!DEFER && cyl_vertical(m1) && upright3(m2))) {
            const double sd = cb_upright_sd(p1, s1, p2, m2, s2);
            if (NEED_DEEP) {
                const int d = (margin >= deep_thr()) ? (sd < deep_thr()) : (sd < margin && sd < deep_thr());
                *nd = d;
                return d;
            }
            return sd < margin ? 1 : 0;
        }
        if (DEFER && !NEED_DEEP) return -1;
        if (NEED_DEEP) {
            int d = (margin >= deep_thr()) ? (int)cyl_box_overlap<OUTLINE>(p1, m1, s1, p2, m2, s2, deep_thr())
                                      : (int)(cyl_box_overlap<OUTLINE>(p1, m1, s1, p2, m2, s2, margin) &&
                                              cyl_box_overlap<OUTLINE>(p1, m1, s1, p2, m2, s2, deep_thr()));
            *nd = d;
            return d;
        }
        return cyl_box_overlap<OUTLINE>(p1, m1, s1, p2, m2, s2, margin) ? 1 : 0;
    }
    // box-box: SAT (exact for boxes) decides contact; deep contacts: one pass, SAT + manifold
    if (NEED_DEEP) {
        SSPP_NP_STAT(13);
        // UP: every box-box pair of the job is upright (a per-pair run-time dispatch for the
        // generic kernels measured neutral on multi-goal: 31.4-31.5 vs 31.8 M cand/s)
        if (UP)
            *nd = (margin >= deep_thr() || sat_box_box(p1, m1, s1, p2, m2, s2, margin))
                      ? box_box_deep_count_up(p1, m1, s1, p2, m2, s2) : 0;
        else
            *nd = (margin >= deep_thr() || sat_box_box(p1, m1, s1, p2, m2, s2, margin))
                      ? box_box_deep_count(p1, m1, s1, p2, m2, s2) : 0;
        if (*nd > 0) SSPP_NP_STAT(14);
        return *nd;
    }
    return sat_box_box(p1, m1, s1, p2, m2, s2, margin) ? 1 : 0;
}

// rounding allowance of the culls (pair_near, the hull masks): the spline evaluation's |error| ~ 1e-15
constexpr double kHullPad = 1e-9;

// Per-waypoint broadphase of one pair (exact: it only rejects pairs whose narrowphase cannot
// report dist < margin).  Two spheres: MuJoCo's bounding-sphere test.  Plane vs a bounded
// geom: every point of the geom lies within rbound of its centre, so a centre height over the
// plane above rbound + margin (+ kHullPad for rounding) rules out a contact — the plane-box
// corners satisfy t >= h - sum_j |n.a_j| e_j >= h - |e| = h - rbound (Cauchy-Schwarz).
// A box partner that passes the sphere test is tested once more against the moving geom's
// bounding sphere (centre in the box frame, distance to the box): a geom whose sphere stays
// farther than rbound + margin (+ kHullPad) from the box cannot touch it.  This rejects, for a
// few dozen flops, the near-but-apart pairs (a block above a large table) before the 15-axis SAT.
SSPP_HD bool pair_near(const DPair& pr, double rg, const double* gp,
                                          const double* op, const double* om) {
    const double ro = pr.orbound;
    if (rg > 0.0 && ro > 0.0) {
        const double dc[3] = {op[0] - gp[0], op[1] - gp[1], op[2] - gp[2]};
        const double thr = rg + ro + pr.margin;
        if (dot3(dc, dc) > thr * thr) return false;
        if (pr.otype == 6) {
            const double lx = fma(om[6], dc[2], fma(om[3], dc[1], om[0] * dc[0]));
            const double ly = fma(om[7], dc[2], fma(om[4], dc[1], om[1] * dc[0]));
            const double lz = fma(om[8], dc[2], fma(om[5], dc[1], om[2] * dc[0]));
            const double ex = fmax(fabs(lx) - pr.osize[0], 0.0), ey = fmax(fabs(ly) - pr.osize[1], 0.0),
                         ez = fmax(fabs(lz) - pr.osize[2], 0.0);
            const double lim = rg + pr.margin + in_sgpr(kHullPad);  // (the pad: see deep_thr)
            return !(fma(ez, ez, fma(ey, ey, ex * ex)) > lim * lim);
        }
        return true;
    }
    if (pr.otype == 0 && rg > 0.0) {
        const double h = (gp[0] - op[0]) * om[2] + (gp[1] - op[1]) * om[5] + (gp[2] - op[2]) * om[8];
        return !(h - rg > pr.margin + in_sgpr(kHullPad));
    }
    return true;
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
