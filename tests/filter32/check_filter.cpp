// The FP32 filter (sspp_filter.h) against the FP64 narrowphase it stands in for (sspp_device.h):
// random box-box and plane-box configurations placed within 1e-8..1e-1 m of touching, with the
// kernel's input pipeline restated on both sides (a 4-term spline evaluation of the position and
// quaternion from control points — doubles for FP64, their float copies for FP32 — then the
// quaternion's normalisation and rotation).  Every certain FP32 decision (HIT / NO) must equal
// the FP64 decision in both argument orders; AMBIGUOUS is allowed.  v_rsq_f32's 1-ulp error is
// emulated (SSPF_HOST_RSQ_JITTER).  Built and run by tests/test_filter32.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#define SSPF_HOST_RSQ_JITTER
#include "sspp_filter.h"

static std::mt19937_64 g_rng(20261018);
static std::uniform_real_distribution<double> U01(0.0, 1.0);
float sspf::rsq_jitter() { return 1.0f + (float)((U01(g_rng) * 2.0 - 1.0) * 1.2e-7); }

static double U(double a, double b) { return a + (b - a) * U01(g_rng); }

// eval_split's operation order: acc = N0 c0, acc = fma(Nr, cr, acc)
static void spline4(const double N[4], const double c[4][7], int D, double* qd, float* q32) {
    for (int d = 0; d < D; ++d) {
        double a = N[0] * c[0][d];
        float f = (float)N[0] * (float)c[0][d];
        for (int r = 1; r < 4; ++r) {
            a = fma(N[r], c[r][d], a);
            f = fmaf((float)N[r], (float)c[r][d], f);
        }
        qd[d] = a;
        q32[d] = f;
    }
}

// the 15 SAT quantities FP64 and FP32 compare with the margin (sat_box_box's formulas, both
// precisions), for the error measurement: max |FP32 - FP64| over axes FP64 evaluates
template <class T>
static void sat_seps(const T* pa, const T* ma, const T* ea, const T* pb, const T* mb, const T* eb, T* out, bool* used) {
    const T Tv[3] = {pb[0] - pa[0], pb[1] - pa[1], pb[2] - pa[2]};
    T t[3], R[3][3];
    for (int i = 0; i < 3; ++i) {
        t[i] = ma[i] * Tv[0] + ma[3 + i] * Tv[1] + ma[6 + i] * Tv[2];
        for (int j = 0; j < 3; ++j) R[i][j] = ma[i] * mb[j] + ma[3 + i] * mb[3 + j] + ma[6 + i] * mb[6 + j];
    }
    int o = 0;
    for (int i = 0; i < 3; ++i) {
        out[o] = std::fabs(t[i]) - (ea[i] + eb[0] * std::fabs(R[i][0]) + eb[1] * std::fabs(R[i][1]) + eb[2] * std::fabs(R[i][2]));
        used[o++] = true;
    }
    for (int j = 0; j < 3; ++j) {
        out[o] = std::fabs(t[0] * R[0][j] + t[1] * R[1][j] + t[2] * R[2][j]) -
                 (ea[0] * std::fabs(R[0][j]) + ea[1] * std::fabs(R[1][j]) + ea[2] * std::fabs(R[2][j]) + eb[j]);
        used[o++] = true;
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            T L[3];
            if (i == 0) { L[0] = 0; L[1] = -R[2][j]; L[2] = R[1][j]; }
            else if (i == 1) { L[0] = R[2][j]; L[1] = 0; L[2] = -R[0][j]; }
            else { L[0] = -R[1][j]; L[1] = R[0][j]; L[2] = 0; }
            const T len2 = L[0] * L[0] + L[1] * L[1] + L[2] * L[2];
            T rb = 0;
            for (int k = 0; k < 3; ++k) rb += eb[k] * std::fabs(R[0][k] * L[0] + R[1][k] * L[1] + R[2][k] * L[2]);
            out[o] = std::fabs(t[0] * L[0] + t[1] * L[1] + t[2] * L[2]) -
                     (ea[0] * std::fabs(L[0]) + ea[1] * std::fabs(L[1]) + ea[2] * std::fabs(L[2]) + rb);
            used[o++] = len2 >= (T)1e-10;
        }
}

static void rand_quat(double* q) {
    double s = 0;
    for (int k = 0; k < 4; ++k) { q[k] = U(-1, 1); s += q[k] * q[k]; }
    s = std::sqrt(s);
    for (int k = 0; k < 4; ++k) q[k] /= s;
}

struct Cfg {
    double ea[3], eb[3], pb[3], mb[9], margin;
    double qbase[4];
    double qsig, psig;
    bool plane;
};

// one FP64 / FP32 evaluation at root position target + along dir * s
struct Eval {
    double pa[3], ma[9];
    float pa32[3], ma32[9];
    bool ok32;
};

static Eval make_eval(const Cfg& c, const double* target, const double N[4], const double dq[4][4],
                      const double dp[4][3]) {
    double ctrl[4][7];
    for (int r = 0; r < 4; ++r) {
        for (int k = 0; k < 3; ++k) ctrl[r][k] = target[k] + dp[r][k];
        for (int k = 0; k < 4; ++k) ctrl[r][3 + k] = c.qbase[k] + dq[r][k];
    }
    // remove the weighted offsets so that the FP64 evaluation lands on the target (up to rounding)
    double shift[7] = {0};
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 3; ++k) shift[k] += N[r] * dp[r][k];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 3; ++k) ctrl[r][k] -= shift[k];
    double qd[7];
    float q32[7];
    spline4(N, ctrl, 7, qd, q32);
    Eval e;
    double qq[4] = {qd[3], qd[4], qd[5], qd[6]};
    sspd::normalize4(qq);
    sspd::quat2mat(qq, e.ma);
    for (int k = 0; k < 3; ++k) { e.pa[k] = qd[k]; e.pa32[k] = q32[k]; }
    e.ok32 = sspf::quat_rot32(q32 + 3, e.ma32);
    return e;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 200000;
    long bad = 0, amb = 0, hit = 0, no = 0, tot = 0, notok = 0;
    double worst_certified = 1e300;  // smallest |FP64 boundary offset| of a certain decision
    double max_err = 0.0;            // largest |FP32 - FP64| SAT separation / eps's scale S
    const double margins[] = {0.0, 0.0, 0.001, 0.1};
    const double qsigs[] = {0.0, 1e-7, 1e-4, 0.02, 0.08, 0.5};
    for (long it = 0; it < n; ++it) {
        Cfg c{};
        c.plane = U01(g_rng) < 0.2;
        c.margin = margins[it % 4];
        for (int k = 0; k < 3; ++k) { c.ea[k] = U(0.005, 0.3); c.eb[k] = U(0.005, 0.6); c.pb[k] = U(-1.0, 1.0); }
        // partner rotation: identity, 90 deg about z, a yaw, or generic
        const int orient = (int)(U01(g_rng) * 4);
        double qb[4] = {1, 0, 0, 0};
        if (orient == 1) { qb[0] = std::sqrt(0.5); qb[3] = std::sqrt(0.5); }
        else if (orient == 2) { const double h = U(-M_PI, M_PI) / 2; qb[0] = std::cos(h); qb[3] = std::sin(h); }
        else if (orient == 3) rand_quat(qb);
        sspd::quat2mat(qb, c.mb);
        if (c.plane) { for (int k = 0; k < 9; ++k) c.mb[k] = (k % 4 == 0) ? 1.0 : 0.0; c.pb[2] = 0.0; }
        // moving box orientation: aligned with the partner's, or random, then perturbed
        if (U01(g_rng) < 0.5) for (int k = 0; k < 4; ++k) c.qbase[k] = qb[k];
        else rand_quat(c.qbase);
        c.qsig = qsigs[(it / 4) % 6];
        c.psig = U01(g_rng) < 0.5 ? 0.0 : 0.05;
        // spline weights: a partition of unity (sometimes a single control point, like u = 0)
        double N[4] = {1, 0, 0, 0};
        if (U01(g_rng) < 0.8) {
            double s = 0;
            for (int r = 0; r < 4; ++r) { N[r] = U(0, 1); s += N[r]; }
            for (int r = 0; r < 4; ++r) N[r] /= s;
        }
        double dq[4][4], dp[4][3];
        for (int r = 0; r < 4; ++r) {
            for (int k = 0; k < 4; ++k) dq[r][k] = c.qsig * U(-1, 1);
            for (int k = 0; k < 3; ++k) dp[r][k] = c.psig * U(-1, 1);
        }
        // direction from the partner, then the touching distance along it (FP64 bisection)
        double dir[3], dn = 0;
        for (int k = 0; k < 3; ++k) { dir[k] = U(-1, 1); dn += dir[k] * dir[k]; }
        dn = std::sqrt(dn);
        for (int k = 0; k < 3; ++k) dir[k] /= dn;
        if (c.plane && dir[2] < 0) dir[2] = -dir[2];
        const double ra = std::sqrt(c.ea[0] * c.ea[0] + c.ea[1] * c.ea[1] + c.ea[2] * c.ea[2]);
        const double rb = c.plane ? 0.0 : std::sqrt(c.eb[0] * c.eb[0] + c.eb[1] * c.eb[1] + c.eb[2] * c.eb[2]);
        // the kernel's FP64 decision: the pair_near culls, then the narrowphase
        sspd::DPair pr{};
        pr.otype = c.plane ? 0 : 6;
        pr.margin = c.margin;
        for (int k = 0; k < 3; ++k) { pr.opos[k] = c.pb[k]; pr.osize[k] = c.eb[k]; }
        for (int k = 0; k < 9; ++k) pr.omat[k] = c.mb[k];
        pr.orbound = c.plane ? 0.0 : std::sqrt(c.eb[0] * c.eb[0] + c.eb[1] * c.eb[1] + c.eb[2] * c.eb[2]);
        const double rgd = std::sqrt(c.ea[0] * c.ea[0] + c.ea[1] * c.ea[1] + c.ea[2] * c.ea[2]);
        auto contact64 = [&](const Eval& e, bool swap) -> bool {
            int nd = 0;
            if (!sspd::pair_near(pr, rgd, e.pa, c.pb, c.mb)) return false;
            if (c.plane) return sspd::col_plane_box(c.pb, c.mb, e.pa, e.ma, c.ea, c.margin, &nd) > 0;
            return swap ? sspd::sat_box_box(c.pb, c.mb, c.eb, e.pa, e.ma, c.ea, c.margin)
                        : sspd::sat_box_box(e.pa, e.ma, c.ea, c.pb, c.mb, c.eb, c.margin);
        };
        auto at = [&](double s) {
            double t[3];
            for (int k = 0; k < 3; ++k) t[k] = c.pb[k] + s * dir[k];
            return make_eval(c, t, N, dq, dp);
        };
        double lo = 0.0, hi = ra + rb + c.margin + 1.0;
        if (!contact64(at(lo), false) || contact64(at(hi), false)) continue;
        for (int k = 0; k < 60; ++k) {
            const double mid = 0.5 * (lo + hi);
            if (contact64(at(mid), false)) lo = mid; else hi = mid;
        }
        const double off = (U01(g_rng) < 0.5 ? -1 : 1) * std::pow(10.0, U(-8.0, -1.0));
        const Eval e = at(0.5 * (lo + hi) + off);
        if (!e.ok32) { ++notok; continue; }
        ++tot;
        const double S = std::max(1.0, ra + rb + c.margin);
        const float eps = (float)(2e-4 * S);
        float ea32[3], eb32[3], pb32[3], mb32[9];
        for (int k = 0; k < 3; ++k) { ea32[k] = (float)c.ea[k]; eb32[k] = (float)c.eb[k]; pb32[k] = (float)c.pb[k]; }
        for (int k = 0; k < 9; ++k) mb32[k] = (float)c.mb[k];
        // the kernel's FP32 decision (scan_pairs32): the certified culls, then the narrowphase
        const float ro32 = (float)pr.orbound, rg32 = (float)rgd;
        const int nr = sspf::pair_near32(ro32, pr.otype, (float)c.margin, eb32, rg32, e.pa32, pb32, mb32, eps, 1e-9f);
        int r32 = sspf::kNo;
        if (nr != sspf::kNo) {
            if (c.plane) r32 = sspf::collide32(0, pb32, mb32, eb32, 6, e.pa32, e.ma32, ea32, (float)c.margin, eps);
            else r32 = sspf::collide32(6, e.pa32, e.ma32, ea32, 6, pb32, mb32, eb32, (float)c.margin, eps);
            if (r32 == sspf::kHit && nr == sspf::kAmb) r32 = sspf::kAmb;
        }
        const bool c64a = contact64(e, false), c64b = c.plane ? c64a : contact64(e, true);
        if (!c.plane) {
            double s64[15], s32d[15];
            float s32[15];
            bool u64[15], u32[15];
            sat_seps<double>(e.pa, e.ma, c.ea, c.pb, c.mb, c.eb, s64, u64);
            sat_seps<float>(e.pa32, e.ma32, ea32, pb32, mb32, eb32, s32, u32);
            for (int a = 0; a < 15; ++a) {
                s32d[a] = s32[a];
                if (u64[a] && u32[a]) max_err = std::max(max_err, std::fabs(s32d[a] - s64[a]) / S);
            }
        }
        if (r32 == sspf::kAmb) { ++amb; continue; }
        if (r32 == sspf::kHit) ++hit; else ++no;
        const bool want = r32 == sspf::kHit;
        if (c64a != want || c64b != want) {
            ++bad;
            if (bad <= 10)
                printf("MISMATCH it %ld plane %d r32 %d fp64 %d/%d off %.3e margin %g qsig %g\n", it, c.plane, r32,
                       c64a, c64b, off, c.margin, c.qsig);
        } else {
            worst_certified = std::min(worst_certified, std::fabs(off));
        }
    }
    printf("tested %ld certain-hit %ld certain-no %ld ambiguous %ld (%.3f%%) short-quaternion %ld\n", tot, hit, no,
           amb, 100.0 * amb / (tot ? tot : 1), notok);
    printf("smallest boundary offset certified %.3e\n", worst_certified);
    printf("largest |FP32 - FP64| SAT separation per metre of scale %.3e (eps %.1e per metre)\n", max_err, 2e-4);
    printf("mismatches %ld\n", bad);
    return bad ? 1 : 0;
}
