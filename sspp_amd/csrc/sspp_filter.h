// sspp_filter.h — FP32-filtered contact decisions for the SamplingPathPlanner scan (gfx950).
//
// checkCollision (include/sspp.h:132-150) asks, per waypoint, whether ANY pair has a contact;
// the FP64 narrowphase (sspp_device.h) decides each pair in the oracle's operation order.  On
// gfx950 an FP32 VALU instruction issues in half the cycles of an FP64 one (SIMD-32: a wave64
// v_fma_f32 takes 2 cycles, v_fma_f64 4; MI355X_MICROARCH.md), its transcendentals are single
// instructions, and it needs half the registers.  So k_sspp_c2f first evaluates every pair of a
// waypoint in FP32 and keeps FP64 for what FP32 cannot decide with certainty — a static filter
// in the sense of Shewchuk's adaptive predicates:
//   * every quantity the FP64 code compares with a threshold (SAT separations, the corner
//     heights of plane-box, the bounding-sphere distances) is recomputed in FP32 from FP32
//     copies of the same inputs; with |FP32 - FP64| <= eps for all of them (DESIGN.md §5
//     derives the error budget: <= ~6e-5 m at robocrane's scale against eps = 2e-4 m), a value
//     >= thr + eps proves that the FP64 code sees it >= thr, and one < thr - eps that it sees
//     it < thr;
//   * a pair is HIT when FP32 proves every separation below the threshold (the FP64 SAT finds
//     no separating axis: contact), NO when it proves one separating axis (or a cull), and
//     AMBIGUOUS otherwise — a value within eps of its threshold, a near-parallel SAT edge axis
//     whose inclusion (FP64 skips |L|^2 < 1e-12) FP32 cannot decide, a short quaternion, a
//     position outside the certified range, or a pair type the filter does not handle
//     (spheres, cylinders): the lane then runs that pair in FP64 exactly as before.
// Every NaN comparison falls on the AMBIGUOUS side.  The feasibility flag is an OR over
// (waypoint, pair), so it equals the all-FP64 scan's — and the oracle's — bit for bit; FP32
// only settles what FP64 would settle the same way (tests/test_filter32.py checks the filter
// against the FP64 functions on random near-boundary configurations, and every GPU parity test
// runs with it).
//
// __host__ __device__: the host test build runs the same code (1/sqrtf stands in for v_rsq_f32).
#pragma once
#include "sspp_device.h"

namespace sspf {

using namespace sspd;

constexpr int kNo = 0, kHit = 1, kAmb = 2;
// FP64's degenerate-edge cut (sat_box_box: len2 < 1e-12 is skipped) is undecidable in FP32
// within kLenBand of it: FP32's |L| is within ~7e-6 of FP64's, so an edge axis is
// certainly evaluated by FP64 when |L|_32 >= 1e-6 + kLenBand, and otherwise uncertain
constexpr float kLenBand = 1e-5f;
constexpr float kLenEval2 = (1e-6f + 2.0f * kLenBand) * (1e-6f + 2.0f * kLenBand);
// quaternions shorter than this are left to FP64 (normalisation would amplify FP32's error)
constexpr float kMinQuat2 = 0.25f;

SSPP_HD float dot3f(const float* a, const float* b) { return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])); }
SSPP_HD void matvec3f(const float* m, const float* v, float* r) {
    r[0] = dot3f(m + 0, v);
    r[1] = dot3f(m + 3, v);
    r[2] = dot3f(m + 6, v);
}
SSPP_HD void matmul3f(const float* a, const float* b, float* r) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float c[3] = {b[j], b[3 + j], b[6 + j]};
            r[3 * i + j] = dot3f(a + 3 * i, c);
        }
}
#if defined(SSPF_HOST_RSQ_JITTER)
float rsq_jitter();  // host test: v_rsq_f32's 1-ulp error, emulated (tests/filter32/check_filter.cpp)
#endif
SSPP_HD float rsqf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rsqf(x);  // v_rsq_f32 (1 ulp)
#elif defined(SSPF_HOST_RSQ_JITTER)
    return (1.0f / sqrtf(x)) * rsq_jitter();
#else
    return 1.0f / sqrtf(x);
#endif
}

// Normalised rotation of a free joint's quaternion (w, x, y, z); false (FP64 decides) when
// |q|^2 < kMinQuat2 or not finite.  FP64's normalize4 leaves |q| within 1e-15 of 1 untouched;
// the difference is far inside eps.
SSPP_HD bool quat_rot32(const float* q, float* R) {
    float s = q[0] * q[0];
    s = fmaf(q[1], q[1], s);
    s = fmaf(q[2], q[2], s);
    s = fmaf(q[3], q[3], s);
    if (!(s >= kMinQuat2 && s < 1e30f)) return false;
    const float inv = rsqf(s);
    const float w = q[0] * inv, x = q[1] * inv, y = q[2] * inv, z = q[3] * inv;
    const float q00 = w * w, q01 = w * x, q02 = w * y, q03 = w * z;
    const float q11 = x * x, q12 = x * y, q13 = x * z, q22 = y * y, q23 = y * z, q33 = z * z;
    R[0] = q00 + q11 - q22 - q33;
    R[4] = q00 - q11 + q22 - q33;
    R[8] = q00 - q11 - q22 + q33;
    R[1] = 2.0f * (q12 - q03);
    R[2] = 2.0f * (q13 + q02);
    R[3] = 2.0f * (q12 + q03);
    R[5] = 2.0f * (q23 - q01);
    R[6] = 2.0f * (q13 - q02);
    R[7] = 2.0f * (q23 + q01);
    return true;
}

// The bounding-sphere culls of sspd::pair_near, certified: kNo when FP64 certainly culls the pair
// (then it reports no contact for it), kHit when FP64 certainly does not, kAmb within eps of a
// cull threshold.  Both sides matter: with a margin, the SAT's contact test (every axis
// separation < margin) can hold for boxes whose bounding spheres are farther apart than
// rg + ro + margin (corner to corner), so a certain contact needs a certain "not culled" too.
SSPP_HD int pair_near32(float ro, int otype, float margin, const float* osize, float rg, const float* gp,
                        const float* op, const float* om, float eps, float pad) {
    int r = kHit;
    if (rg > 0.0f && ro > 0.0f) {
        const float dc[3] = {op[0] - gp[0], op[1] - gp[1], op[2] - gp[2]};
        const float thr = rg + ro + margin;
        const float d2 = dot3f(dc, dc);
        if (d2 > (thr + eps) * (thr + eps)) return kNo;
        if (!(d2 < (thr - eps) * (thr - eps))) r = kAmb;
        if (otype == 6) {
            const float lx = fmaf(om[6], dc[2], fmaf(om[3], dc[1], om[0] * dc[0]));
            const float ly = fmaf(om[7], dc[2], fmaf(om[4], dc[1], om[1] * dc[0]));
            const float lz = fmaf(om[8], dc[2], fmaf(om[5], dc[1], om[2] * dc[0]));
            const float ex = fmaxf(fabsf(lx) - osize[0], 0.0f), ey = fmaxf(fabsf(ly) - osize[1], 0.0f),
                        ez = fmaxf(fabsf(lz) - osize[2], 0.0f);
            const float lim = rg + margin + pad;
            const float e2 = fmaf(ez, ez, fmaf(ey, ey, ex * ex));
            if (e2 > (lim + eps) * (lim + eps)) return kNo;
            if (!(e2 < (lim - eps) * (lim - eps))) r = kAmb;
        }
        return r;
    }
    if (otype == 0 && rg > 0.0f) {
        const float h = (gp[0] - op[0]) * om[2] + (gp[1] - op[1]) * om[5] + (gp[2] - op[2]) * om[8];
        const float x = h - rg;
        if (x > margin + pad + eps) return kNo;
        return x < margin + pad - eps ? kHit : kAmb;
    }
    return kHit;
}

SSPP_HD float sqrt_1ulp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);  // v_sqrt_f32 (1 ulp; far inside eps)
#else
    return sqrtf(x);
#endif
}

// sat_box_box (sspp_device.h) with certified margins: kHit when no axis can separate by thr,
// kNo when one certainly does, kAmb otherwise.  Early exit per axis like the FP64 code (a
// branch-free form kept every axis's intermediates live: 275 spilled VGPRs at 96), and the edge
// axes' dot products written without the exact-zero component of L = A_i x B_j.
SSPP_HD int sat_box_box32(const float* pa, const float* ma, const float* ea, const float* pb, const float* mb,
                          const float* eb, float thr, float eps) {
    const float T[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    const float hi = thr + eps, lo = thr - eps;
    float t[3], R[3][3], AR[3][3];
    bool amb = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        t[i] = fmaf(ma[6 + i], T[2], fmaf(ma[3 + i], T[1], ma[i] * T[0]));
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            R[i][j] = fmaf(ma[6 + i], mb[6 + j], fmaf(ma[3 + i], mb[3 + j], ma[i] * mb[j]));
            AR[i][j] = fabsf(R[i][j]);
        }
        const float rb = fmaf(eb[2], AR[i][2], fmaf(eb[1], AR[i][1], eb[0] * AR[i][0]));
        const float sep = fabsf(t[i]) - (ea[i] + rb);
        if (sep >= hi) return kNo;
        amb |= !(sep < lo);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float pr = fabsf(fmaf(t[2], R[2][j], fmaf(t[1], R[1][j], t[0] * R[0][j])));
        const float ra = fmaf(ea[2], AR[2][j], fmaf(ea[1], AR[1][j], ea[0] * AR[0][j]));
        const float sep = pr - (ra + eb[j]);
        if (sep >= hi) return kNo;
        amb |= !(sep < lo);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        // L = A_i x B_j in A's frame has L_i = 0: (a, b) are its other two components, on axes
        // (i1, i2) = the other two indices of A, so that L_i1 = a, L_i2 = b
        const int i1 = i == 0 ? 1 : 0, i2 = i == 2 ? 1 : 2;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            // i = 0: (0, -R2j, R1j); i = 1: (R2j, 0, -R0j); i = 2: (-R1j, R0j, 0)
            const float a = i == 0 ? -R[2][j] : (i == 1 ? R[2][j] : -R[1][j]);
            const float b = i == 0 ? R[1][j] : (i == 1 ? -R[0][j] : R[0][j]);
            const float len2 = fmaf(b, b, a * a);
            const bool eval = len2 >= kLenEval2;  // else FP64 may or may not include this axis
            const float pr = fabsf(fmaf(t[i2], b, t[i1] * a));
            const float ra = fmaf(ea[i2], fabsf(b), ea[i1] * fabsf(a));
            float rb = 0.0f;
#pragma unroll
            for (int k = 0; k < 3; ++k) rb = fmaf(eb[k], fabsf(fmaf(R[i2][k], b, R[i1][k] * a)), rb);
            // FP64 compares the unnormalised num with thr |L| (|L| <= 1: num's error <= eps too)
            const float num = (pr - (ra + rb)) - (thr == 0.0f ? 0.0f : thr * sqrt_1ulp(len2));
            if (eval && num >= eps) return kNo;
            amb |= !eval || !(num < -eps);
        }
    }
    return amb ? kAmb : kHit;
}

// col_plane_box's contact test (some corner with dist <= margin on the half facing the plane)
SSPP_HD int plane_box32(const float* pp, const float* pm, const float* bp, const float* bm, const float* e,
                        float margin, float eps) {
    const float n[3] = {pm[2], pm[5], pm[8]};
    const float d[3] = {bp[0] - pp[0], bp[1] - pp[1], bp[2] - pp[2]};
    const float d0 = dot3f(d, n);
    float a[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float ax[3] = {bm[j], bm[3 + j], bm[6 + j]};
        a[j] = dot3f(n, ax) * e[j];
    }
    bool amb = false, hit = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        float l = (k & 1) ? a[0] : -a[0];
        l = l + ((k & 2) ? a[1] : -a[1]);
        l = l + ((k & 4) ? a[2] : -a[2]);
        const float t = d0 + l;
        // FP64 counts the corner iff !(t > margin) && !(l > 0)
        hit |= t < margin - eps && l < -eps;
        amb |= !(t > margin + eps || l > eps);
    }
    return hit ? kHit : (amb ? kAmb : kNo);
}

// Narrowphase dispatch (types ordered as sspd::collide's): the contact test of the pairs the
// filter handles; everything else is left to FP64
SSPP_HD int collide32(int t1, const float* p1, const float* m1, const float* s1, int t2, const float* p2,
                      const float* m2, const float* s2, float margin, float eps) {
    if (t1 == 0 && t2 == 6) return plane_box32(p1, m1, p2, m2, s2, margin, eps);
    if (t1 == 6 && t2 == 6) return sat_box_box32(p1, m1, s1, p2, m2, s2, margin, eps);
    return kAmb;
}

}  // namespace sspf
