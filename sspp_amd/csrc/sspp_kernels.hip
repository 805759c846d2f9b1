// sspp_kernels.hip — MI355X (gfx950) kernels for sampled-spline candidate scoring.
//
// Hot path (reference include/sspp.h:194-225 and include/sspp/tsp_planner.h:95-138):
//   candidate sampling -> B-spline evaluation -> free-joint FK -> collision -> cost -> argmin.
//
// Work decomposition:
//   * a candidate owns LPC = 64*ceil(items/64) lanes (capped at 256), one waypoint per lane;
//     a 256-thread workgroup holds CPB = 256/LPC candidates;
//   * the workgroup prologue builds the shared basis tables (span + N_0..N_p for every
//     waypoint parameter) and the candidates' control points in LDS (Philox + Box-Muller
//     in-kernel, or a coalesced copy of caller-supplied control points);
//   * each lane evaluates its waypoint(s): spline from LDS, FK of the moving body, pair
//     loop over the scene table (wave-uniform -> scalar loads), broadphase + narrowphase;
//   * per-candidate sums use the canonical order (lane partials, xor butterfly per wave,
//     waves in order) that oracle/sspp_oracle.c::or_canon_sum restates;
//   * one BlockBest per workgroup, then a one-block argmin kernel (lowest id on ties).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "model.h"
#ifdef SSPP_C2F_STATS  // profiling builds only (tools/build_variant.sh stats -DSSPP_C2F_STATS)
__device__ unsigned long long g_c2f_stats[16];
#define SSPP_CB_STAT(i) atomicAdd(&g_c2f_stats[i], 1ull)
#endif
#ifdef SSPP_WG_TIMING  // profiling builds only: per-workgroup (start, end, CU, survivors) of k_sspp_c2f
__device__ unsigned long long g_wg_t[1 << 18];
__device__ unsigned long long g_wg_ph[6 << 16];  // per workgroup: shader clock after each phase
#define WG_PH(k) do { if (threadIdx.x == 0 && blockIdx.x < (1 << 16)) g_wg_ph[6 * blockIdx.x + (k)] = clock64(); } while (0)
#else
#define WG_PH(k) do { } while (0)
#endif
#include "sspp_device.h"

using namespace sspd;

namespace {

constexpr int kBlock = 256;
#ifndef SSPP_SCORE_WAVES_PER_EU
#define SSPP_SCORE_WAVES_PER_EU 4  // min waves per SIMD (4 -> <=128 VGPRs; measured best on gfx950)
#endif
constexpr int kMaxMovers = 2;
constexpr int kMaxSteps = 64;  // steps per launch (k_sspp_c2f)

struct KScene {
    int npairs;
    int onegeom;        // every pair shares one moving geom: its pose is computed once
    int static_block;   // sspp: env-env contacts counted and present -> nothing feasible
    double static_cost; // tsp: Collision.h cost of env-env contacts, added per waypoint
    int cylbox;         // some moving pair is cylinder-box (selects the kernels that carry that code)
};

// Scene tables are passed as separate __restrict__ kernel arguments: the pair loop is
// wave-uniform and the tables are provably not written by the kernel, so the compiler
// reads them with scalar (s_load) instructions into SGPRs, once per wave.
struct SceneT {
    const DGeom* __restrict__ geoms;
    const DPair* __restrict__ pairs;
    const DMover* __restrict__ movers;
};

// Constant address space (4): loads through these are scalar (SMEM) whenever the address
// is wave-uniform, independent of the alias analysis of the surrounding kernel.
#if defined(__HIP_DEVICE_COMPILE__)
#define SSPP_CONST __attribute__((address_space(4)))
#else
#define SSPP_CONST
#endif
typedef const SSPP_CONST DGeom* cgeom_t;
typedef const SSPP_CONST DPair* cpair_t;
typedef const SSPP_CONST DMover* cmover_t;

__device__ __forceinline__ DGeom load_geom(cgeom_t p) {
    DGeom g;
#pragma unroll
    for (int k = 0; k < 3; ++k) g.pos[k] = p->pos[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) g.mat[k] = p->mat[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) g.size[k] = p->size[k];
    g.rbound = p->rbound;
    g.reach = p->reach;
    g.type = p->type;
    g.mover = p->mover;
    g.orig = p->orig;
    g.relrot = p->relrot;
    return g;
}
__device__ __forceinline__ DPair load_pair(cpair_t p) {
    DPair r;
    r.gm = p->gm;
    r.go = p->go;
    r.otype = p->otype;
    r.oorig = p->oorig;
    r.omover = p->omover;
    r.pad = 0;
    r.margin = p->margin;
#pragma unroll
    for (int k = 0; k < 3; ++k) r.opos[k] = p->opos[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) r.omat[k] = p->omat[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) r.osize[k] = p->osize[k];
    r.orbound = p->orbound;
    return r;
}

// ---------------------------------------------------------------- candidate-level broadphase
// A B-spline lies in the convex hull of its control points (non-negative basis, partition of
// unity), so every waypoint's mover position lies in the AABB [lo, hi] of the control points'
// position columns.  A pair whose partner cannot come within rbound + margin of that box
// (expanded by the moving geom's reach) for ANY waypoint is culled for the whole candidate:
// exactly the pairs the per-waypoint bounding-sphere test would reject at every waypoint.
// kHullPad absorbs the rounding of the spline evaluation (|error| ~ 1e-15).
constexpr double kHullPad = 1e-9;

__device__ __forceinline__ bool pair_may_touch(const DPair& pr, const DGeom& G, const double* lo,
                                               const double* hi) {
    if (pr.omover >= 0 || G.rbound <= 0.0) return true;
    const double slack = G.reach + G.rbound + pr.margin + kHullPad;
    if (pr.orbound > 0.0) {
        double d2 = 0.0;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const double c = pr.opos[d];
            const double e = c < lo[d] ? lo[d] - c : (c > hi[d] ? c - hi[d] : 0.0);
            d2 = fma(e, e, d2);
        }
        const double lim = pr.orbound + slack;
        return d2 <= lim * lim;
    }
    if (pr.otype == 0) {  // plane: lowest point of the box over the plane's normal
        const double n0 = pr.omat[2], n1 = pr.omat[5], n2 = pr.omat[8];
        const double m = (n0 >= 0 ? n0 * lo[0] : n0 * hi[0]) + (n1 >= 0 ? n1 * lo[1] : n1 * hi[1]) +
                         (n2 >= 0 ? n2 * lo[2] : n2 * hi[2]) -
                         (n0 * pr.opos[0] + n1 * pr.opos[1] + n2 * pr.opos[2]);
        return m - slack < 0.0;
    }
    return true;
}

// Bit k of the result: pair k can touch (pairs >= 64 are always evaluated).  One lane per
// pair, then a wave ballot -> the mask is wave-uniform (SGPRs).
template <int D, int NM, int MODE>
__device__ __forceinline__ unsigned long long hull_mask(const double* ctrl, int n, int npairs,
                                                        cpair_t pairs, cgeom_t geoms,
                                                        cmover_t movers) {
    const int lane = threadIdx.x & 63;
    bool act = false;
    if (lane < npairs) {
        const DPair pr = load_pair(pairs + lane);
        const DGeom G = load_geom(geoms + pr.gm);
        const int m = (NM > 1 && G.mover == 1) ? 1 : 0;
        double lo[3], hi[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int col = MODE == 1 ? d : 7 * m + d;
            if (col < D) {
                double a = ctrl[col], b = ctrl[col];
                for (int j = 1; j < n; ++j) {
                    const double v = ctrl[j * D + col];
                    a = v < a ? v : a;
                    b = v > b ? v : b;
                }
                lo[d] = a; hi[d] = b;
            } else {
                lo[d] = hi[d] = (double)movers[m].qpos0[d];
            }
        }
        act = pair_may_touch(pr, G, lo, hi);
    }
    unsigned long long mask = __ballot(act);
    if (npairs > 64) mask = ~0ull;
    return mask;
}

struct BlockBest {
    double cost;
    long long idx;
    long long count;
    long long pad;
};

struct SsppK {
    KScene sc;
    int has_scene;
    int ablate;    // profiling only (SSPP_ABLATE env): 1 no sampling, 2 no collision, 4 no arc
    int insample;  // draw the candidates inside the scoring kernel (else k_sample_sspp)
    int p, n, W;
    double sigma;
    unsigned long long seed;
    long long first_id, B;
    int lpc, cpb, shared_endpoints;
    int arc_all;
};

struct TspK {
    KScene sc;
    int n, K, cp;
    double start[4], end[4], lo[4], hi[4];
    double z_min;
    unsigned long long seed;
    long long first_id, B;
    double w_col, floor_z_min, floor_margin, floor_scale;
    int lpc, cpb;
    // CES slot mode (tsp_planner.h:78-93 seeds): launch candidate c is slot slot0 + c of the
    // iteration's list [mean set, forwarded best (if any), samples...].  Slots below *nfixed
    // copy fixed[slot]; slot s >= *nfixed is random sample s - *nfixed (Philox id first_id +
    // s - *nfixed); slots past *nfixed + samples are padding (status 0, cost +inf).
    int ces;
    const double* fixed;    // [2][K][4]
    const int* nfixed;
    long long slot0, samples;
};

// ---------------------------------------------------------------- Philox4x32-10 + Box-Muller
__device__ __forceinline__ void philox(unsigned c0, unsigned c1, unsigned c2, unsigned c3,
                                       unsigned k0, unsigned k1, unsigned o[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        unsigned hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        unsigned hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        unsigned n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3;
}
__device__ __forceinline__ void philox_words(unsigned long long seed, unsigned long long g,
                                             unsigned idx, unsigned stream, unsigned o[4]) {
    philox(idx, stream, (unsigned)g, (unsigned)(g >> 32), (unsigned)seed, (unsigned)(seed >> 32), o);
}
__device__ __forceinline__ void normal_pair(unsigned long long seed, unsigned long long g,
                                            unsigned idx, unsigned stream, double* z0, double* z1) {
    unsigned o[4];
    philox_words(seed, g, idx, stream, o);
    unsigned long long a = ((((unsigned long long)o[0]) << 32) | o[1]) >> 11;
    unsigned long long b = ((((unsigned long long)o[2]) << 32) | o[3]) >> 11;
    double u1 = (double)(a + 1) * 1.1102230246251565e-16;
    double u2 = (double)b * 1.1102230246251565e-16;
    double r = sqrt(-2.0 * log(u1));
    // angle 2*pi*u2 as sincospi(2 u2): one call, exact quarter-turn reduction (no Payne-Hanek);
    // oracle/sspp_oracle.c::or_sincospi restates it
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    *z0 = r * cs;
    *z1 = r * sn;
}
// SamplingPathPlanner normals (sampleWithNoise): one Philox4x32-10 call gives four 24-bit
// uniforms -> two Box-Muller pairs in FP32, with fmaf polynomials written out (ln u by the atanh
// series on the mantissa, sin / cos of 2 pi u after an exact quarter-turn reduction) and a
// correctly rounded sqrtf, so oracle/sspp_oracle.c::or_normal_quad reproduces it bit for bit.
// Four normals per Philox call and FP32 instead of FP64 log / sincospi: the FP64 sampler was
// the largest phase of k_sspp_c2f (24 of 62 kclk per workgroup, tools/wg_timing.py).
__device__ __forceinline__ float bm_log(float u) {  // ln u, u in [2^-24, 1]
    const unsigned bits = __float_as_uint(u);
    int e = (int)(bits >> 23) - 127;
    float m = __uint_as_float((bits & 0x7fffffu) | 0x3f800000u);  // [1, 2)
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    const float s = (m - 1.0f) / (m + 1.0f);                      // |s| <= 0.1716
    const float s2 = s * s;
    float p = fmaf(s2, 0.111111111f, 0.142857143f);
    p = fmaf(s2, p, 0.2f);
    p = fmaf(s2, p, 0.333333333f);
    p = fmaf(s2, p, 1.0f);
    return fmaf((float)e, 0.693147181f, (s + s) * p);
}
__device__ __forceinline__ void bm_sincos2pi(float u, float* sn, float* cs) {  // u in [0, 1)
    const float q = rintf(4.0f * u);
    const float r = fmaf(-0.25f, q, u);  // exact
    const float a = r * 6.28318531f;     // |a| <= pi / 4
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
__device__ __forceinline__ void normal_quad(unsigned long long seed, unsigned long long g,
                                            unsigned idx, unsigned stream, double z[4]) {
    unsigned o[4];
    philox_words(seed, g, idx, stream, o);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const float u1 = (float)((o[2 * h] >> 8) + 1u) * 5.96046448e-8f;  // (0, 1], exact
        const float u2 = (float)(o[2 * h + 1] >> 8) * 5.96046448e-8f;     // [0, 1), exact
        const float r = sqrtf(-2.0f * bm_log(u1));
        float sn, cs;
        bm_sincos2pi(u2, &sn, &cs);
        z[2 * h] = (double)(r * cs);
        z[2 * h + 1] = (double)(r * sn);
    }
}
__device__ __forceinline__ double uniform01(unsigned long long seed, unsigned long long g,
                                            unsigned idx, unsigned stream) {
    unsigned o[4];
    philox_words(seed, g, idx, stream, o);
    unsigned long long b = ((((unsigned long long)o[2]) << 32) | o[3]) >> 11;
    return (double)b * 1.1102230246251565e-16;
}

// ---------------------------------------------------------------- spline from basis rows
// N: p+1 basis values of one waypoint (host-precomputed table in global memory, L2 resident)
template <int D, int P>
__device__ __forceinline__ void eval_pt(const double* ctrl, const double* __restrict__ N,
                                        int span, double* q) {
    double Nr[P + 1];
#pragma unroll
    for (int r = 0; r <= P; ++r) Nr[r] = N[r];
    const double* c0 = ctrl + (span - P) * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        double acc = Nr[0] * c0[d];
#pragma unroll
        for (int r = 1; r <= P; ++r) acc = fma(Nr[r], c0[r * D + d], acc);
        q[d] = acc;
    }
}

template <int D>
__device__ __forceinline__ double dist_nd(const double* a, const double* b) {
    double d0 = b[0] - a[0];
    double s = d0 * d0;
#pragma unroll
    for (int d = 1; d < D; ++d) { double dd = b[d] - a[d]; s = fma(dd, dd, s); }
    return sqrt(s);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------- one waypoint vs the scene
// Mover root poses (position + rotation) for MODE 0 (q -> qpos[0:D] window, free joints at
// qpos[7m:7m+7]) or MODE 1 ((x, y, z, yaw) -> the bound free body, utility.h:149-206).
template <int D, int NM, int MODE>
__device__ __forceinline__ void mover_poses(const double* q, cmover_t movers,
                                            double (&mp)[NM][3], double (&mR)[NM][9]) {
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        double qp[7];
        if (MODE == 0) {
#pragma unroll
            for (int k = 0; k < 7; ++k)
                qp[k] = (7 * m + k < D) ? q[(7 * m + k < D) ? 7 * m + k : 0] : (double)movers[m].qpos0[k];
        } else {
#ifndef SSPP_YAW_GENERIC
            // yaw_to_quat (utility.h:198-206): q = (cos h, 0, 0, sin h) — a rotation about z.
            // normalize4 + quat2mat written out for x = y = +0: every entry equals the generic
            // formula's (sums with exact zeros), except the sign of the four zero entries,
            // which only ever enter products and sums with non-zero terms
            const double half = q[3] * 0.5;
            double w = cos(half), z = sin(half);
            const double nn = sqrt(fma(z, z, w * w));
            if (nn < kMinVal) { w = 1.0; z = 0.0; }
            else if (fabs(nn - 1.0) > kMinVal) { const double inv = 1.0 / nn; w *= inv; z *= inv; }
            const double q00 = w * w, q33 = z * z, q03 = w * z;
            double* R = mR[m];
            R[0] = q00 - q33; R[1] = 2.0 * (0.0 - q03); R[2] = 0.0;
            R[3] = 2.0 * (0.0 + q03); R[4] = q00 - q33; R[5] = 0.0;
            R[6] = 0.0; R[7] = 0.0; R[8] = q00 + q33;
            mp[m][0] = q[0]; mp[m][1] = q[1]; mp[m][2] = q[2];
            continue;
#else
            double half = q[3] * 0.5;
            qp[0] = q[0]; qp[1] = q[1]; qp[2] = q[2];
            qp[3] = cos(half); qp[4] = 0.0; qp[5] = 0.0; qp[6] = sin(half);
#endif
        }
        normalize4(qp + 3);
        quat2mat(qp + 3, mR[m]);
        mp[m][0] = qp[0]; mp[m][1] = qp[1]; mp[m][2] = qp[2];
    }
}

// Geom pose from its mover's pose.  With an identity relative rotation the geom frame IS the
// mover frame: copying R reproduces the oracle's quat2mat(mulquat(root, 1)) exactly.
__device__ __forceinline__ void geom_pose(const double* P, const double* R, const DGeom& G,
                                          double* gp, double* gm) {
    double t[3];
    matvec3(R, G.pos, t);
    gp[0] = P[0] + t[0]; gp[1] = P[1] + t[1]; gp[2] = P[2] + t[2];
    if (G.relrot) {
        matmul3(R, G.mat, gm);
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) gm[k] = R[k];
    }
}

__device__ __forceinline__ void geom_pos(const double* P, const double* R, const DGeom& G, double* gp) {
    double t[3];
    matvec3(R, G.pos, t);
    gp[0] = P[0] + t[0]; gp[1] = P[1] + t[1]; gp[2] = P[2] + t[2];
}
__device__ __forceinline__ void geom_rot(const double* R, const DGeom& G, double* gm) {
    if (G.relrot) {
        matmul3(R, G.mat, gm);
    } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) gm[k] = R[k];
    }
}

// Geom pose from a mover rotation about z (R[2] = R[5] = R[6] = R[7] = 0, MODE 1): the
// generic dot products with those zero terms dropped (each dropped term adds an exact zero).
template <bool ZR>
__device__ __forceinline__ void geom_pos_t(const double* P, const double* R, const DGeom& G, double* gp) {
    if (!ZR) { geom_pos(P, R, G, gp); return; }
    gp[0] = P[0] + fma(R[1], G.pos[1], R[0] * G.pos[0]);
    gp[1] = P[1] + fma(R[4], G.pos[1], R[3] * G.pos[0]);
    gp[2] = P[2] + R[8] * G.pos[2];
}
template <bool ZR>
__device__ __forceinline__ void geom_rot_t(const double* R, const DGeom& G, double* gm) {
    if (!ZR || !G.relrot) { geom_rot(R, G, gm); return; }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        gm[j] = fma(R[1], G.mat[3 + j], R[0] * G.mat[j]);
        gm[3 + j] = fma(R[4], G.mat[3 + j], R[3] * G.mat[j]);
        gm[6 + j] = R[8] * G.mat[6 + j];
    }
}

// Per-waypoint broadphase of one pair (exact: it only rejects pairs whose narrowphase cannot
// report dist < margin).  Two spheres: MuJoCo's bounding-sphere test.  Plane vs a bounded
// geom: every point of the geom lies within rbound of its centre, so a centre height over the
// plane above rbound + margin (+ kHullPad for rounding) rules out a contact — the plane-box
// corners satisfy t >= h - sum_j |n.a_j| e_j >= h - |e| = h - rbound (Cauchy-Schwarz).
__device__ __forceinline__ bool pair_near(const DPair& pr, double rg, const double* gp,
                                          const double* op, const double* om) {
    const double ro = pr.orbound;
    if (rg > 0.0 && ro > 0.0) {
        const double dc[3] = {op[0] - gp[0], op[1] - gp[1], op[2] - gp[2]};
        const double thr = rg + ro + pr.margin;
        return !(dot3(dc, dc) > thr * thr);
    }
    if (pr.otype == 0 && rg > 0.0) {
        const double h = (gp[0] - op[0]) * om[2] + (gp[1] - op[1]) * om[5] + (gp[2] - op[2]) * om[8];
        return !(h - rg > pr.margin + kHullPad);
    }
    return true;
}

// DEEP=false: checkCollision's ncon > 0 for one candidate.  Every active lane of the wave
//   must belong to that candidate: the scan stops for the whole wave at the first pair where
//   any lane finds a contact (returns 1 on every lane — the candidate is infeasible whatever
//   the other waypoints give), or when *stop (the candidate's LDS flag, cleared by another
//   wave of the same candidate) reads 0.  Returns 0 when no lane has a contact.
// DEEP=true : returns 0, *cost = sum over deep contacts of -1/(center_dist + 1e-4) + static.
template <int D, int NM, int MODE, bool DEEP, bool ONEGEOM, bool CB = true>
__device__ int point_collide(const double* q, const KScene& sc, const SceneT& T,
                             unsigned long long mask, double* cost, int* stop = nullptr) {
    static_assert(!ONEGEOM || NM == 1, "single moving geom implies a single mover");
    const cgeom_t geoms = (cgeom_t)T.geoms;
    const cpair_t pairs = (cpair_t)T.pairs;
    double mp[NM][3], mR[NM][9];
    mover_poses<D, NM, MODE>(q, (cmover_t)T.movers, mp, mR);
    double acc = 0.0;
    int cur = -1;
    double gp[3], gmat[9];
    bool have_rot = true;  // multi-geom movers: a geom's rotation is formed at its first near pair
    DGeom G;
    constexpr bool ZR = MODE == 1;  // yaw-only mover rotation
    if (ONEGEOM) {  // every pair shares one moving geom: pose once, mover pose dies here
        cur = pairs[0].gm;
        G = load_geom(geoms + cur);
        geom_pos_t<ZR>(mp[0], mR[0], G, gp);
        geom_rot_t<ZR>(mR[0], G, gmat);
    }
    const int np = sc.npairs;
    for (int k = 0; k < np; ++k) {
        if (k < 64) {
            // skip culled pairs with a scalar bit scan
            const unsigned long long rest = mask >> k;
            if (rest == 0ull) break;
            k += __builtin_ctzll(rest);
            if (k >= np) break;
        }
        const DPair pr = load_pair(pairs + k);
        if (!ONEGEOM && pr.gm != cur) {
            cur = pr.gm;
            G = load_geom(geoms + cur);
            const bool second = NM > 1 && G.mover == 1;
            geom_pos_t<ZR>(second ? mp[NM - 1] : mp[0], second ? mR[NM - 1] : mR[0], G, gp);
            have_rot = false;
        }
        double op_[3], om_[9];
        const double* op = pr.opos;
        const double* om = pr.omat;
        if (NM > 1 && pr.omover >= 0) {
            const bool second = pr.omover == 1;
            const double* R = second ? mR[NM - 1] : mR[0];
            const double* P = second ? mp[NM - 1] : mp[0];
            double t[3];
            matvec3(R, pr.opos, t);
            op_[0] = P[0] + t[0]; op_[1] = P[1] + t[1]; op_[2] = P[2] + t[2];
            matmul3(R, pr.omat, om_);
            op = op_; om = om_;
        }
        const bool near = pair_near(pr, G.rbound, gp, op, om);
        int nd = 0, nc = 0;
        if (near) {
            if (!ONEGEOM && !have_rot) {
                const bool second = NM > 1 && G.mover == 1;
                geom_rot_t<ZR>(second ? mR[NM - 1] : mR[0], G, gmat);
                have_rot = true;
            }
            const bool gfirst = (G.type < pr.otype) || (G.type == pr.otype && G.orig < pr.oorig);
            if (gfirst) nc = collide<DEEP, CB, DEEP>(G.type, gp, gmat, G.size, pr.otype, op, om, pr.osize, pr.margin, &nd);
            else nc = collide<DEEP, CB, DEEP>(pr.otype, op, om, pr.osize, G.type, gp, gmat, G.size, pr.margin, &nd);
        }
        if (!DEEP) {
            // the loop trip is wave-uniform, so every active lane reaches this vote
            if (__ballot(nc > 0) != 0ull) return 1;
            if (stop && __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                return 1;
        } else if (nd > 0) {
            const double dc[3] = {op[0] - gp[0], op[1] - gp[1], op[2] - gp[2]};
            const double cd = sqrt(dot3(dc, dc));
            const double term = -1.0 / (cd + 1e-4);
            for (int i = 0; i < nd; ++i) acc = acc + term;
        }
    }
    if (DEEP) *cost = acc + sc.static_cost;
    return 0;
}

// ---------------------------------------------------------------- batch argmin helpers
__device__ __forceinline__ bool better(double c1, long long i1, double c2, long long i2) {
    // lexicographic (cost, index); index -1 means "none"
    if (i2 < 0) return i1 >= 0;
    if (i1 < 0) return false;
    return (c1 < c2) || (c1 == c2 && i1 < i2);
}

// ---------------------------------------------------------------- fused batch argmin
// Each workgroup publishes one BlockBest; arrivals are counted on 8 sharded counters (one
// 64-byte line each, shard = block % 8) so no single word sees more than ~B/16 atomics.
// The last arriver of a shard reduces that shard and publishes a shard record; the last of
// the shards reduces the 8 shard records into *out and re-arms every counter.
// Hand-off (cdna_hip_programming.md Guideline 16, R1 with sc1 on both sides): records are
// written with 8-byte agent-scope relaxed atomic stores (global_store ... sc1, write-through),
// every storing lane drains with s_waitcnt vmcnt(0) before its relaxed agent atomic add, and
// consumers read records only with agent-scope relaxed atomic loads (sc1, bypass L1) after
// their add returned "last" and a workgroup barrier.  No release/acquire fences needed.
struct ArgminSync {
    unsigned int shard[8][16];  // arrival counters, one cache line each
    unsigned int top[16];
    BlockBest rec[8];           // shard results
};

__device__ __forceinline__ void st_rec(BlockBest* p, const BlockBest& b) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q + 0, (unsigned long long)__double_as_longlong(b.cost), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)b.idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 2, (unsigned long long)b.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ BlockBest ld_rec(BlockBest* p) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    BlockBest b;
    b.cost = __longlong_as_double((long long)__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    b.idx = (long long)__hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b.count = (long long)__hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b.pad = 0;
    return b;
}

// block-wide lexicographic reduction of records idx0 + stride*i, i < n (all NT threads call)
template <int NT = kBlock>
__device__ BlockBest reduce_recs(BlockBest* recs, int idx0, int stride, int n, double* scratch) {
    double bc = INFINITY;
    long long bi = -1, cnt = 0;
    for (int i = threadIdx.x; i < n; i += NT) {
        const BlockBest b = ld_rec(recs + idx0 + (long long)stride * i);
        cnt += b.count;
        if (better(b.cost, b.idx, bc, bi)) { bc = b.cost; bi = b.idx; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double oc = __shfl_xor(bc, off, 64);
        const long long oi = __shfl_xor(bi, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
        if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
    }
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        scratch[3 * w] = bc;
        scratch[3 * w + 1] = __longlong_as_double(bi);
        scratch[3 * w + 2] = __longlong_as_double(cnt);
    }
    __syncthreads();
    BlockBest r;
    r.cost = scratch[0];
    r.idx = __double_as_longlong(scratch[1]);
    r.count = __double_as_longlong(scratch[2]);
    r.pad = 0;
    for (int k = 1; k < NT / 64; ++k) {
        const double oc = scratch[3 * k];
        const long long oi = __double_as_longlong(scratch[3 * k + 1]);
        r.count += __double_as_longlong(scratch[3 * k + 2]);
        if (better(oc, oi, r.cost, r.idx)) { r.cost = oc; r.idx = oi; }
    }
    return r;
}

// All NT threads of the workgroup call this after thread 0 filled `bb`.
template <int NT = kBlock>
__device__ void finish_batch(const BlockBest& bb, BlockBest* __restrict__ part, ArgminSync* sync,
                             sspp_best* out, int nblk = -1, int b = -1) {
    __shared__ double scratch[16];
    if (nblk < 0) { nblk = gridDim.x; b = blockIdx.x; }
    const int sh = b & 7;
    const int nsh = nblk < 8 ? nblk : 8;
    int* flag = reinterpret_cast<int*>(scratch + 14);
    if (!out) {
        if (threadIdx.x == 0) part[b] = bb;
        return;
    }
    if (threadIdx.x == 0) {
        st_rec(part + b, bb);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned shard_n = (unsigned)((nblk - sh + 7) >> 3);
        const unsigned prev = __hip_atomic_fetch_add(&sync->shard[sh][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = prev == shard_n - 1;
    }
    __syncthreads();
    if (!*flag) return;
    const BlockBest shard_best = reduce_recs<NT>(part, sh, 8, (nblk - sh + 7) >> 3, scratch);
    if (threadIdx.x == 0) {
        st_rec(sync->rec + sh, shard_best);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(&sync->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = prev == (unsigned)nsh - 1;
    }
    __syncthreads();
    if (!*flag) return;
    const BlockBest r = reduce_recs<NT>(sync->rec, 0, 1, nsh, scratch);
    if (threadIdx.x == 0) {
        out->cost = r.idx < 0 ? INFINITY : r.cost;
        out->index = r.idx;
        out->count = r.count;
        out->reserved = 0;
        for (int k = 0; k < 8; ++k) __hip_atomic_store(&sync->shard[k][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sync->top[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------- candidate sampler
// sampleWithNoise (include/sspp.h:114-130) for `steps` batches of B candidates, step s covering
// ids first_id + s * step_stride + [0, B): one thread per (step, candidate, Box-Muller pair) over
// the whole chip; writes the perturbed control-point columns j in [p, n-p) as
// pert[steps][B][npert] with npert = (n-2p)*D, value = init + (sigma * z) * limits[d].
// A separate launch at full occupancy (26 VGPRs, 8 waves/SIMD): the FP64 log/sqrt/sincospi
// chains are latency-bound, and in the scoring kernel (3 waves/SIMD) they were 40% of its time.
__global__ __launch_bounds__(kBlock) void k_sample_sspp(
    unsigned long long seed, long long first_id, long long step_stride, long long B, int steps,
    int D, int p, int npert, double sigma, const double* __restrict__ init_ctrl,
    const double* __restrict__ limits, double* __restrict__ pert) {
    const int nq = (npert + 3) >> 2;
    const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (t >= (long long)steps * B * nq) return;
    const long long sb = t / nq;
    const int m = (int)(t - sb * nq);
    const long long s = sb / B, b = sb - s * B;
    double z[4];
    normal_quad(seed, (unsigned long long)(first_id + s * step_stride + b), (unsigned)m, 0u, z);
    const double* base = init_ctrl + p * D;
    double* out = pert + sb * npert;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int k = 4 * m + h;
        if (k < npert) out[k] = base[k] + (sigma * z[h]) * limits[k % D];
    }
}

// ---------------------------------------------------------------- SamplingPathPlanner kernel
// tab: host-precomputed basis rows, (W+1) collision rows u = i/W then W arc rows v = i/(W-1),
// P+1 doubles each; span: matching knot spans.
template <int D, int NM, int P, bool ONEGEOM>
__global__ __launch_bounds__(kBlock, SSPP_SCORE_WAVES_PER_EU) void k_sspp(
    SsppK a, SceneT T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ init_ctrl, const double* __restrict__ limits,
    const double* __restrict__ ctrl_in, const double* __restrict__ pert,
    double* __restrict__ ctrl_out, double* __restrict__ arc, unsigned char* __restrict__ feasible,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int P1 = P + 1;
    const int tid = threadIdx.x, lpc = a.lpc, cpb = a.cpb, n = a.n, W = a.W;
    const int ndof = n * D;
    const int slot = tid / lpc, lane = tid - slot * lpc;
    const long long cand0 = (long long)blockIdx.x * cpb;
    double* s_ctrl = smem;                        // [cpb][n][D]
    double* s_wsum = s_ctrl + cpb * ndof;         // [4]
    double* s_arc = s_wsum + kBlock / 64;         // [4]
    int* s_flag = (int*)(s_arc + 4);              // [cpb] + shared endpoints
    const double* tcol = tab;
    const double* tarc = tab + (W + 1) * P1;
    const int* scol = span;
    const int* sarc = span + (W + 1);

    if (tid <= cpb) s_flag[tid] = 1;
    const long long nvalid = min((long long)cpb, a.B - cand0);
    // prefetch this lane's basis rows (global, L2-resident) while the control points stage
    double Ncol[P1];
    int sc0 = P;
    {
        const int i = lane + 1 < W ? lane + 1 : W - 1;
#pragma unroll
        for (int r = 0; r < P1; ++r) Ncol[r] = tcol[i * P1 + r];
        sc0 = scol[i];
    }
    if (ctrl_in) {
        const double* src = ctrl_in + cand0 * ndof;
        for (int e = tid; e < nvalid * ndof; e += kBlock) s_ctrl[e] = src[e];
    } else {
        // init control points + perturbed columns j in [p, n-p): from the sampler kernel, or
        // (insample) drawn here by the workgroup itself
        const int npert = (n - 2 * P) * D;
        const bool from_pert = !a.insample && !(a.ablate & 1);
        for (int e = tid; e < cpb * ndof; e += kBlock) {
            const int sl = e / ndof, r = e - sl * ndof;
            const int k = r - P * D;
            s_ctrl[e] = (from_pert && k >= 0 && k < npert && sl < nvalid)
                            ? pert[(cand0 + sl) * npert + k]
                            : init_ctrl[r];
        }
        if (a.insample) {
            __syncthreads();
            const int nq = (npert + 3) >> 2;
            for (int e = tid; e < cpb * nq; e += kBlock) {
                const int sl = e / nq, m = e - sl * nq;
                if (sl >= nvalid) continue;
                double z[4];
                normal_quad(a.seed, (unsigned long long)(a.first_id + cand0 + sl), (unsigned)m, 0u, z);
                double* c = s_ctrl + sl * ndof + P * D;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const int k = 4 * m + h;
                    if (k < npert) c[k] = c[k] + (a.sigma * z[h]) * limits[k % D];
                }
            }
        }
    }
    __syncthreads();
    if (ctrl_out) {
        double* dst = ctrl_out + cand0 * ndof;
        for (int e = tid; e < nvalid * ndof; e += kBlock) dst[e] = s_ctrl[e];
    }

    const bool valid = slot < nvalid;
    const double* myc = s_ctrl + slot * ndof;
    double q[D], q2[D];
    const unsigned long long mask =
        a.has_scene ? hull_mask<D, NM, 0>(myc, n, a.sc.npairs, (cpair_t)T.pairs, (cgeom_t)T.geoms,
                                          (cmover_t)T.movers)
                    : 0ull;

    // checkCollision: interior points i = 1..W-1 one per lane; endpoints i = 0, W on a spare lane
    // Flags are plain LDS stores (every writer stores 0; read after the barrier below):
    // no volatile/atomic access, so the scene tables stay on the scalar-load path.
    if (a.has_scene && valid && !(a.ablate & 2)) {
        int* vflag = s_flag;
        if (a.sc.static_block) vflag[slot] = 0;
        for (int j = lane; j < W - 1; j += lpc) {
            const int i = j + 1;
            if (j == lane) eval_pt<D, P>(myc, Ncol, sc0, q);
            else eval_pt<D, P>(myc, tcol + i * P1, scol[i], q);
            if (point_collide<D, NM, 0, false, ONEGEOM>(q, a.sc, T, mask, nullptr, vflag + slot)) {
                __hip_atomic_store(vflag + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                break;
            }
        }
        const int spare = (W - 1) % lpc == 0 ? 0 : lpc - 1;
        bool duty0 = false, dutyW = false;
        int fidx = slot;
        if (a.shared_endpoints) {
            fidx = cpb;
            if (lane == spare) {
                if (nvalid == 1) { duty0 = dutyW = slot == 0; }
                else { duty0 = slot == 0; dutyW = slot == 1; }
            }
        } else if (lane == spare) {
            duty0 = dutyW = true;
        }
        if (duty0) {
            eval_pt<D, P>(myc, tcol, scol[0], q);
            if (point_collide<D, NM, 0, false, ONEGEOM>(q, a.sc, T, mask, nullptr)) vflag[fidx] = 0;
        }
        if (dutyW) {
            eval_pt<D, P>(myc, tcol + W * P1, scol[W], q);
            if (point_collide<D, NM, 0, false, ONEGEOM>(q, a.sc, T, mask, nullptr)) vflag[fidx] = 0;
        }
    }

    // computeArcLength: chords between v_{i-1} and v_i, i = 1..W-1
    double acc = 0.0;
    if (valid && !(a.ablate & 4)) {
        for (int j = lane; j < W - 1; j += lpc) {
            const int i = j + 1;
            eval_pt<D, P>(myc, tarc + (i - 1) * P1, sarc[i - 1], q);
            eval_pt<D, P>(myc, tarc + i * P1, sarc[i], q2);
            acc = acc + dist_nd<D>(q, q2);
        }
    }
    acc = wave_sum(acc);
    if ((tid & 63) == 0) s_wsum[tid >> 6] = acc;
    __syncthreads();
    if (lane == 0 && valid) {
        const int w0 = (slot * lpc) >> 6, nw = lpc >> 6;
        double t = s_wsum[w0];
        for (int w = 1; w < nw; ++w) t = t + s_wsum[w0 + w];
        const long long c = cand0 + slot;
        const int f = s_flag[slot] & s_flag[cpb];
        arc[c] = (f || a.arc_all) ? t : INFINITY;
        feasible[c] = (unsigned char)f;
        s_arc[slot] = f ? t : INFINITY;
    }
    __syncthreads();
    BlockBest bb;
    if (tid == 0) {
        bb.cost = INFINITY; bb.idx = -1; bb.count = 0; bb.pad = 0;
        for (int s = 0; s < nvalid; ++s) {
            if (!(s_flag[s] & s_flag[cpb])) continue;
            bb.count++;
            if (s_arc[s] < bb.cost) { bb.cost = s_arc[s]; bb.idx = a.first_id + cand0 + s; }
        }
    }
    finish_batch(bb, part, sync, best);
}

// ================================================================ coarse-to-fine feasibility
// k_sspp_c2f: SamplingPathPlanner scoring, workgroup = CPB candidates (CPB = 256 / G1).
//
// checkCollision (include/sspp.h:132-150) stops at the first waypoint in contact, so the result
// is an OR over waypoints and pairs; the order in which they are examined cannot change it.
// An infeasible candidate is typically in contact over a long stretch of its path (robocrane,
// config 2: ~55 of 129 waypoints), so a handful of well-spread waypoints finds almost all of
// them.  The host orders the W+1 collision waypoints breadth-first by interval bisection
// (ord table); then per workgroup:
//   phase 1  G1 lanes per candidate test the first G1 waypoints of that order; a candidate's
//            lanes leave the pair loop together at the first pair any of them touches
//            (ballot over the candidate's lane group);
//   phase 2  the survivors (few: the feasible ones plus the rare misses) are compacted in LDS
//            and their remaining waypoints spread over all 256 lanes; a lane group that finds
//            a contact clears the candidate's LDS flag, which stops its other lanes;
//   phase 3  arc length for every candidate, in passes of 256/LPC candidates that keep the
//            canonical reduction order of oracle/sspp_oracle.c::or_canon_sum;
//   phase 4  block argmin + the fused batch argmin (finish_batch).
// Sampling (sampleWithNoise, include/sspp.h:114-130) runs in the prologue: one Box-Muller pair
// per thread.
struct SsppC2F {
    KScene sc;
    int has_scene;
    int ablate;
    int insample;
    int p, n, W;
    double sigma;
    unsigned long long seed;
    long long first_id, B;
    int g1, cpb;   // phase-1 lanes per candidate (divides 64), candidates per workgroup
    int npts, n1;  // collision waypoints per candidate (W+1), phase-1 waypoints (<= g1)
    int lpc;       // canonical lanes of the arc-length sum (or_lanes_for(W-1))
    // several independent steps (batches) per launch: workgroup b belongs to step b / nblk_step;
    // step s scores ids first_id + s * step_stride + [0, B) into arc/feasible + s * B, its own
    // argmin records / counters (part + s * nblk_step, sync + s) and best[s]
    int nblk_step;
    long long step_stride;
    int arc_all;   // 0: arc length only for collision-free candidates (+inf otherwise)
    int hull;      // candidate hull broadphase: 0 off, 1 all candidates, 2 phase-1 survivors
    unsigned* dfr; // [0]: candidates of this launch left undecided (cylinder-box), [1]: k_sspp_cbfix arrivals
};

#ifdef SSPP_C2F_STATS
#define C2F_STAT(i, v) do { const unsigned long long v_ = (v); if ((threadIdx.x & 63) == 0 && v_) atomicAdd(&g_c2f_stats[i], v_); } while (0)
#else
#define C2F_STAT(i, v) do { } while (0)
#endif

// Pair loop of one waypoint per lane.  All 64 lanes run the (wave-uniform) loop; `live` lanes
// test the pairs of their own mask.  gbits = the lanes of this lane's candidate within the
// wave: when any of them touches, all of them stop (returns true for the group).  flag: the
// candidate's LDS feasibility flag (phase 2), polled so lanes in other waves stop too.
// A cylinder-box pair that passes the bounding-sphere test sets dfr (undecided) and counts as
// no contact here (collide<..., DEFER>); k_sspp_cbfix settles it with the exact test.
template <int D, int NM, bool ONEGEOM>
__device__ __forceinline__ bool scan_pairs(const double* q, bool live, unsigned long long mymask,
                                           unsigned long long umask, unsigned long long gbits,
                                           int* flag, const KScene& sc, const SceneT& T, bool& dfr) {
    const cgeom_t geoms = (cgeom_t)T.geoms;
    const cpair_t pairs = (cpair_t)T.pairs;
    double mp[NM][3], mR[NM][9];
    mover_poses<D, NM, 0>(q, (cmover_t)T.movers, mp, mR);
    int cur = -1;
    double gp[3], gmat[9];
    bool have_rot = true;
    DGeom G;
    if (ONEGEOM) {
        cur = pairs[0].gm;
        G = load_geom(geoms + cur);
        geom_pose(mp[0], mR[0], G, gp, gmat);
    }
    bool ghit = false;
    const int np = sc.npairs;
    for (int k = 0; k < np; ++k) {
        if (k < 64) {
            const unsigned long long rest = umask >> k;
            if (rest == 0ull) break;
            k += __builtin_ctzll(rest);
            if (k >= np) break;
        }
        const DPair pr = load_pair(pairs + k);
        if (!ONEGEOM && pr.gm != cur) {
            cur = pr.gm;
            G = load_geom(geoms + cur);
            const bool second = NM > 1 && G.mover == 1;
            geom_pos(second ? mp[NM - 1] : mp[0], second ? mR[NM - 1] : mR[0], G, gp);
            have_rot = false;
        }
        int nc = 0;
        if (live && (k >= 64 || ((mymask >> k) & 1ull))) {
            double op_[3], om_[9];
            const double* op = pr.opos;
            const double* om = pr.omat;
            if (NM > 1 && pr.omover >= 0) {
                const bool second = pr.omover == 1;
                const double* R = second ? mR[NM - 1] : mR[0];
                const double* P = second ? mp[NM - 1] : mp[0];
                double t[3];
                matvec3(R, pr.opos, t);
                op_[0] = P[0] + t[0]; op_[1] = P[1] + t[1]; op_[2] = P[2] + t[2];
                matmul3(R, pr.omat, om_);
                op = op_; om = om_;
            }
            const bool nr = pair_near(pr, G.rbound, gp, op, om);
            C2F_STAT(2, __popcll(__ballot(nr)));
            if (nr) {
                if (!ONEGEOM && !have_rot) {
                    const bool second = NM > 1 && G.mover == 1;
                    geom_rot(second ? mR[NM - 1] : mR[0], G, gmat);
                    have_rot = true;
                }
                int nd = 0;
                const bool gfirst = (G.type < pr.otype) || (G.type == pr.otype && G.orig < pr.oorig);
                if (gfirst) nc = collide<false, true, false, true>(G.type, gp, gmat, G.size, pr.otype, op, om, pr.osize, pr.margin, &nd);
                else nc = collide<false, true, false, true>(pr.otype, op, om, pr.osize, G.type, gp, gmat, G.size, pr.margin, &nd);
                if (nc < 0) { dfr = true; nc = 0; }
            }
        }
        C2F_STAT(flag ? 4 : 0, 1);                          // wave pair iterations (phase 2 / 1)
        C2F_STAT(flag ? 5 : 1, __popcll(__ballot(live && (k >= 64 || ((mymask >> k) & 1ull)))));
        if (__ballot(nc > 0) & gbits) { ghit = true; live = false; }
        if (flag && live && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
            live = false;
        if (__ballot(live) == 0ull) break;
    }
    return ghit;
}

// The exact cylinder-box test (witnesses + candidate search, sspd::cyl_box_overlap) of one
// waypoint over the pairs of `mask` (k_sspp_cbfix).
template <int D, int NM, int P, bool ONEGEOM>
__device__ __forceinline__ bool cb_point_exact(const double* ctrl, const double* row, int span,
                                               unsigned long long mask, int np, SceneT T) {
    double q[D];
    eval_pt<D, P>(ctrl, row, span, q);
    const cgeom_t geoms = (cgeom_t)T.geoms;
    const cpair_t pairs = (cpair_t)T.pairs;
    double mp[NM][3], mR[NM][9];
    mover_poses<D, NM, 0>(q, (cmover_t)T.movers, mp, mR);
    for (int k = 0; k < np; ++k) {
        if (k < 64 && !((mask >> k) & 1ull)) continue;
        const DPair pr = load_pair(pairs + k);
        const DGeom G = load_geom(geoms + pr.gm);
        if (!((G.type == 5 && pr.otype == 6) || (G.type == 6 && pr.otype == 5))) continue;
        const bool second = NM > 1 && G.mover == 1;
        double gp[3], gmat[9], op_[3], om_[9];
        geom_pose(second ? mp[NM - 1] : mp[0], second ? mR[NM - 1] : mR[0], G, gp, gmat);
        const double* op = pr.opos;
        const double* om = pr.omat;
        if (NM > 1 && pr.omover >= 0) {
            const bool osecond = pr.omover == 1;
            const double* R = osecond ? mR[NM - 1] : mR[0];
            const double* Pp = osecond ? mp[NM - 1] : mp[0];
            double t[3];
            matvec3(R, pr.opos, t);
            op_[0] = Pp[0] + t[0]; op_[1] = Pp[1] + t[1]; op_[2] = Pp[2] + t[2];
            matmul3(R, pr.omat, om_);
            op = op_; om = om_;
        }
        if (!pair_near(pr, G.rbound, gp, op, om)) continue;
        int nd = 0;
        const bool gfirst = (G.type < pr.otype) || (G.type == pr.otype && G.orig < pr.oorig);
        const int nc = gfirst ? collide<false>(G.type, gp, gmat, G.size, pr.otype, op, om, pr.osize, pr.margin, &nd)
                              : collide<false>(pr.otype, op, om, pr.osize, G.type, gp, gmat, G.size, pr.margin, &nd);
        if (nc > 0) return true;
    }
    return false;
}

#ifndef SSPP_C2F_WAVES_PER_EU
#define SSPP_C2F_WAVES_PER_EU 4  // measured: 3 -> 1280, 4 -> 1396, 5 -> 1237, 6 -> 697 M cand/s (robocrane)
#endif
template <int D, int NM, int P, bool ONEGEOM, int NT>
__global__ __launch_bounds__(NT, SSPP_C2F_WAVES_PER_EU) void k_sspp_c2f(
    SsppC2F a, SceneT T, const double* __restrict__ otab, const int* __restrict__ ospan,
    const double* __restrict__ atab, const int* __restrict__ aspan,
    const double* __restrict__ init_ctrl, const double* __restrict__ limits,
    const double* __restrict__ ctrl_in, const double* __restrict__ pert,
    double* __restrict__ ctrl_out, double* __restrict__ arc, unsigned char* __restrict__ feasible,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int P1 = P + 1;
    constexpr int NB = 3 * NM;  // AABB extents per candidate (x, y, z per mover)
    const int tid = threadIdx.x, cpb = a.cpb, n = a.n, W = a.W, g1 = a.g1;
    const int lg1 = __builtin_ctz(g1);
    const int ndof = n * D, nch = W - 1;
    const int step = blockIdx.x / a.nblk_step, blk = blockIdx.x - step * a.nblk_step;
    const long long cand0 = (long long)blk * cpb;
    const int nvalid = (int)min((long long)cpb, a.B - cand0);
    const long long first_id = a.first_id + step * a.step_stride;
    if (a.ablate & 64) return;  // profiling: launch + dispatch cost only
#ifdef SSPP_WG_TIMING
    const unsigned long long wg_t0 = wall_clock64();
    int wg_ns = -1;
#endif
    WG_PH(0);
    if (step) {
        arc += step * a.B;
        feasible += step * a.B;
        if (pert) pert += step * a.B * ((n - 2 * P) * D);
        if (ctrl_out) ctrl_out += step * a.B * ndof;
        part += step * a.nblk_step;
        sync += step;
        if (best) best += step;
    }
    double* s_ctrl = smem;                                    // [cpb][n][D]
    // s_box is dead once phase 2's hull masks are built (a barrier follows), so phase 3's
    // s_vsum / s_arc reuse its space: 384 B less per 16-candidate workgroup, which lets LDS
    // hold 16 workgroups per CU instead of 14
    const int nvw3 = a.lpc >> 6, rbox = 2 * NB > nvw3 + 1 ? 2 * NB : nvw3 + 1;
    double* s_box = s_ctrl + cpb * ndof;                      // [cpb][2][NB] (hull)
    double* s_vsum = s_box;                                   // [cpb][lpc/64] (phase 3)
    double* s_arc = s_box + cpb * nvw3;                       // [cpb] (phase 3, outputs)
    unsigned long long* s_mask = (unsigned long long*)(s_box + cpb * rbox);  // [cpb]
    int* s_feas = (int*)(s_mask + cpb);                       // [cpb]
    int* s_surv = s_feas + cpb;                               // [cpb + 1] (last = count)
    int* s_defer = s_surv + cpb + 1;                          // [cpb] undecided cylinder-box pair

    // ---- prologue: control points (+ sampleWithNoise) in LDS.
    {
        if (ctrl_in) {  // element e = sl * ndof + r walked with add-with-carry
            const int dsl = NT / ndof, dr = NT - dsl * ndof;
            int sl = tid / ndof, r = tid - sl * ndof;
            const double* src = ctrl_in + cand0 * ndof;
            for (; sl < nvalid; sl += dsl) {
                s_ctrl[sl * ndof + r] = src[sl * ndof + r];
                r += dr;
                if (r >= ndof) { r -= ndof; ++sl; }
            }
        } else {
            // lane-owned columns: the initial spline's value is loaded once per column and
            // stored for every candidate (LDS stores only, no load latency per element)
            const int npert = (n - 2 * P) * D;
            const bool from_pert = !a.insample && !(a.ablate & 1);
            for (int rr = tid; rr < ndof; rr += NT) {
                const double v0 = init_ctrl[rr];
                const int k = rr - P * D;
                const bool pr = from_pert && k >= 0 && k < npert;
                for (int s2 = 0; s2 < cpb; ++s2)
                    s_ctrl[s2 * ndof + rr] = (pr && s2 < nvalid) ? pert[(cand0 + s2) * npert + k] : v0;
            }
        }
    }
    if (tid < cpb) s_mask[tid] = 0ull;
    __syncthreads();
    if (!ctrl_in && a.insample && !(a.ablate & 1)) {
        // sampleWithNoise: item t = (candidate sl, Philox quad m: normals 4m .. 4m+3).  kUnr
        // items per lane are drawn in straight-line code (ids past the end clamped, results
        // dropped), so the scheduler interleaves their independent chains
        constexpr int kUnr = 2;
        const int npert = (n - 2 * P) * D;
        const int nq = (npert + 3) >> 2;
        const int total = nvalid * nq;
        const int dsl = NT / nq, dm = NT - dsl * nq;
        int sl = tid / nq, m = tid - sl * nq;
        for (int base = 0; base < total; base += kUnr * NT) {  // workgroup-uniform
            double z[kUnr][4];
            int usl[kUnr], um[kUnr];
#pragma unroll
            for (int u = 0; u < kUnr; ++u) {
                usl[u] = sl; um[u] = m;
                const int csl = sl < nvalid ? sl : 0;
                normal_quad(a.seed, (unsigned long long)(first_id + cand0 + csl), (unsigned)m, 0u, z[u]);
                m += dm; sl += dsl;
                if (m >= nq) { m -= nq; ++sl; }
            }
#pragma unroll
            for (int u = 0; u < kUnr; ++u) {
                if (base + u * NT + tid >= total) continue;
                double* c = s_ctrl + usl[u] * ndof + P * D;
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const int k = 4 * um[u] + h;
                    if (k < npert) c[k] = c[k] + (a.sigma * z[u][h]) * limits[k % D];
                }
            }
        }
        __syncthreads();
    }
    if (ctrl_out) {
        double* dst = ctrl_out + cand0 * ndof;
        for (int e = tid; e < nvalid * ndof; e += NT) dst[e] = s_ctrl[e];
    }
    WG_PH(1);

    const SceneT TT = T;
    const bool collide_on = a.has_scene && !(a.ablate & 2);
    const int np = a.sc.npairs;
    // ---- candidate-level broadphase (convex hull of the control points, see pair_may_touch):
    // AABB per (candidate, mover, axis), then one (candidate, pair) test per thread; the mask
    // bits are OR-ed into LDS.
    // hull = 1: every candidate before phase 1; hull = 2 (default): only phase 1's survivors,
    // before phase 2 — phase 1 stops at the first touching pair anyway, and on robocrane the
    // all-candidate hull cost more than it saved (measured: 1.11 vs 1.22 G cand/s without it)
    const int hull = (a.ablate & 32) ? 0 : a.hull;
    if (collide_on && hull == 1) {
        for (int e = tid; e < cpb * NB; e += NT) {
            const int sl = e / NB, md = e - sl * NB, m = md / 3, d = md - m * 3;
            const int col = 7 * m + d;
            double lo, hi;
            if (col < D) {
                const double* c = s_ctrl + sl * ndof + col;
                lo = hi = c[0];
                for (int j = 1; j < n; ++j) {
                    const double v = c[j * D];
                    lo = v < lo ? v : lo;
                    hi = v > hi ? v : hi;
                }
            } else {
                lo = hi = (double)((cmover_t)TT.movers)[m].qpos0[d];
            }
            s_box[sl * 2 * NB + md] = lo;
            s_box[sl * 2 * NB + NB + md] = hi;
        }
        __syncthreads();
        if (np > 64) {
            if (tid < cpb) s_mask[tid] = ~0ull;
        } else {
            for (int e = tid; e < cpb * np; e += NT) {
                const int sl = e / np, k = e - sl * np;
                const DPair pr = load_pair((cpair_t)TT.pairs + k);
                const DGeom G = load_geom((cgeom_t)TT.geoms + pr.gm);
                const int m = (NM > 1 && G.mover == 1) ? 1 : 0;
                const double* bx = s_box + sl * 2 * NB;
                if (pair_may_touch(pr, G, bx + 3 * m, bx + NB + 3 * m))
                    atomicOr(s_mask + sl, 1ull << k);
            }
        }
        __syncthreads();
    } else if (collide_on) {
        if (tid < cpb) s_mask[tid] = ~0ull;
        __syncthreads();
    }
    // ---- phase 1: G1 lanes per candidate, first n1 waypoints of the coarse-to-fine order
    {
        const int g = tid >> lg1, l = tid & (g1 - 1), wg = (tid & 63) >> lg1;
        const unsigned long long low = g1 == 64 ? ~0ull : ((1ull << g1) - 1ull);
        const unsigned long long gbits = low << (wg * g1);
        const bool valid = g < nvalid;
        bool ghit = false, dfr = false;
        if (collide_on) {
            const unsigned long long mymask = s_mask[g];
            unsigned long long umask = 0ull;  // union over the wave's groups (wave-uniform)
            const int g0 = (tid & ~63) >> lg1;
            for (int w = 0; w < (64 >> lg1); ++w) umask |= s_mask[g0 + w];
            const bool live = valid && l < a.n1 && !a.sc.static_block && !(a.ablate & 16);
            double q[D];
            const int row = l < a.npts ? l : 0;
            eval_pt<D, P>(s_ctrl + (valid ? g : 0) * ndof, otab + row * P1, ospan[row], q);
            ghit = scan_pairs<D, NM, ONEGEOM>(q, live, mymask, umask, gbits, nullptr, a.sc, TT, dfr);
        }
        const bool gdef = (__ballot(dfr) & gbits) != 0ull;
        if (l == 0) {
            s_feas[g] = valid && !ghit && !(collide_on && a.sc.static_block);
            s_defer[g] = gdef;
        }
    }
    __syncthreads();
    WG_PH(2);
    // ---- phase 2: survivors' remaining waypoints over the whole workgroup
    const int R = a.npts - a.n1;
    if (collide_on && R > 0 && !(a.ablate & 8)) {
        if (tid < 64) {  // survivors compacted by one wave ballot (cpb <= 64), in candidate order
            const bool f = tid < nvalid && s_feas[tid] != 0;
            const unsigned long long m = __ballot(f);
            if (f) s_surv[__popcll(m & ((1ull << tid) - 1ull))] = tid;
            if (tid == 0) s_surv[cpb] = __popcll(m);
        }
        __syncthreads();
        const int ns = s_surv[cpb];
        if (tid == 0) C2F_STAT(6, ns);
#ifdef SSPP_WG_TIMING
        wg_ns = ns;
#endif
        if (hull == 2 && ns > 0 && np <= 64) {  // the survivors' hull masks (see above)
            for (int e = tid; e < ns * NB; e += NT) {
                const int si = e / NB, md = e - si * NB, m = md / 3, d = md - m * 3;
                const int sl = s_surv[si], col = 7 * m + d;
                double lo, hi;
                if (col < D) {
                    const double* c = s_ctrl + sl * ndof + col;
                    lo = hi = c[0];
                    for (int j = 1; j < n; ++j) {
                        const double v = c[j * D];
                        lo = v < lo ? v : lo;
                        hi = v > hi ? v : hi;
                    }
                } else {
                    lo = hi = (double)((cmover_t)TT.movers)[m].qpos0[d];
                }
                s_box[sl * 2 * NB + md] = lo;
                s_box[sl * 2 * NB + NB + md] = hi;
            }
            if (tid < ns) s_mask[s_surv[tid]] = 0ull;
            __syncthreads();
            for (int e = tid; e < ns * np; e += NT) {
                const int si = e / np, k = e - si * np, sl = s_surv[si];
                const DPair pr = load_pair((cpair_t)TT.pairs + k);
                const DGeom G = load_geom((cgeom_t)TT.geoms + pr.gm);
                const int m = (NM > 1 && G.mover == 1) ? 1 : 0;
                const double* bx = s_box + sl * 2 * NB;
                if (pair_may_touch(pr, G, bx + 3 * m, bx + NB + 3 * m))
                    atomicOr(s_mask + sl, 1ull << k);
            }
            __syncthreads();
        }
        unsigned long long umask = 0ull;
        for (int i = 0; i < ns; ++i) umask |= s_mask[s_surv[i]];
        const int items = ns * R;
        for (int base = 0; base < items; base += NT) {  // workgroup-uniform trip count
            const int it = base + tid;
            bool live = it < items;
            const int si = live ? it / R : 0;
            const int s = s_surv[si];
            const int j = a.n1 + (live ? it - si * R : 0);
            live = live && __hip_atomic_load(s_feas + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
            // lanes of this wave that work on the same survivor
            const int wave_it0 = base + (tid & ~63);
            int lo = si * R - wave_it0, hi = (si + 1) * R - wave_it0;
            lo = lo < 0 ? 0 : lo;
            hi = hi > 64 ? 64 : hi;
            unsigned long long gb = 0ull;
            if (it < items && hi > lo) gb = (hi - lo >= 64) ? ~0ull : (((1ull << (hi - lo)) - 1ull) << lo);
            double q[D];
            eval_pt<D, P>(s_ctrl + s * ndof, otab + j * P1, ospan[j], q);
            bool dfr = false;
            const bool h = scan_pairs<D, NM, ONEGEOM>(q, live, s_mask[s], umask, gb, s_feas + s, a.sc, TT, dfr);
            if (h) __hip_atomic_store(s_feas + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (dfr) __hip_atomic_store(s_defer + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    WG_PH(3);
    // ---- phase 3: arc length (computeArcLength, include/sspp.h:152-169) of the listed
    // candidates: the collision-free ones (findBestPath scores only successful paths), or all
    // of them with arc_all.  Chords v_j -> v_{j+1} (v_i = s(i/(W-1))) go to LDS, then each
    // candidate's chords are summed in the canonical order of oracle/sspp_oracle.c::or_canon_sum:
    // lpc lane partials (chords vl, vl+lpc, ...), an xor butterfly per 64 lanes, 64-lane groups
    // in order.
    if (tid < cpb) s_arc[tid] = INFINITY;
    if (!(a.ablate & 4)) {
        __syncthreads();
        int* s_list = s_surv;  // phase 2 is done with it
        if (tid < 64) {  // one wave ballot, candidate order
            const bool f = tid < nvalid && (a.arc_all || s_feas[tid] != 0);
            const unsigned long long m = __ballot(f);
            if (f) s_list[__popcll(m & ((1ull << tid) - 1ull))] = tid;
            if (tid == 0) s_list[cpb] = __popcll(m);
        }
        __syncthreads();
        const int nl = s_list[cpb];
        // one wave per (listed candidate, 64-lane group v of the lpc canonical lanes): lane l
        // accumulates chords j = 64 v + l, + lpc, ... (the lane partials of or_canon_sum), then
        // the xor butterfly gives the group's sum.  A chord's first point is the previous lane's
        // second point (same candidate, same pass), taken by shuffle: bit-identical to
        // evaluating it again.  No chord array: the workgroup's LDS holds only control points.
        const int lpc = a.lpc, nvw = lpc >> 6, lane = tid & 63;
        for (int vw = tid >> 6; vw < nl * nvw; vw += NT / 64) {  // wave-uniform
            const int si = vw / nvw, v = vw - si * nvw;
            const double* myc = s_ctrl + s_list[si] * ndof;
            double acc = 0.0;
            for (int base = v * 64; base < nch; base += lpc) {  // wave-uniform trip count
                const int j = base + lane, jj = j < nch ? j : nch - 1;
                double qa[D], qb[D];
                eval_pt<D, P>(myc, atab + (jj + 1) * P1, aspan[jj + 1], qb);
#pragma unroll
                for (int d = 0; d < D; ++d) qa[d] = __shfl_up(qb[d], 1, 64);
                if (lane == 0) eval_pt<D, P>(myc, atab + jj * P1, aspan[jj], qa);
                if (j < nch) acc = acc + dist_nd<D>(qa, qb);
            }
            acc = wave_sum(acc);
            if (lane == 0) s_vsum[vw] = acc;
        }
        __syncthreads();
        if (tid < nl) {
            double t = s_vsum[tid * nvw];
            for (int w = 1; w < nvw; ++w) t = t + s_vsum[tid * nvw + w];
            s_arc[s_list[tid]] = t;
        }
    }
    __syncthreads();
    WG_PH(4);
    if (tid == 0) C2F_STAT(7, nvalid);
    if (tid < nvalid) {
        const long long c = cand0 + tid;
        if (s_feas[tid]) C2F_STAT(8, 0);
        arc[c] = s_arc[tid];
        // 2: no contact except cylinder-box pairs left undecided; k_sspp_cbfix writes 0 or 1
        feasible[c] = (unsigned char)(s_feas[tid] == 0 ? 0 : (s_defer[tid] ? 2 : 1));
    }
    // block argmin over the workgroup's feasible candidates: one wave, lexicographic (cost, id)
    // xor butterfly (exact, order independent: the lowest id wins ties like the serial scan).
    // Undecided candidates stay out; k_sspp_cbfix merges the ones it clears.
    BlockBest bb;
    if (tid < 64) {
        const bool und = tid < nvalid && s_feas[tid] != 0 && s_defer[tid] != 0;
        const unsigned long long um = __ballot(und);
        if (tid == 0 && um != 0ull)
            __hip_atomic_fetch_add(a.dfr, (unsigned)__popcll(um), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool f = tid < nvalid && s_feas[tid] != 0 && !und;
        double bc = f ? s_arc[tid] : INFINITY;
        long long bi = f ? first_id + cand0 + tid : -1;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double oc = __shfl_xor(bc, off, 64);
            const long long oi = __shfl_xor(bi, off, 64);
            if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
        }
        bb.cost = bi < 0 ? INFINITY : bc; bb.idx = bi; bb.count = __popcll(__ballot(f)); bb.pad = 0;
    }
    finish_batch<NT>(bb, part, sync, best, a.nblk_step, blk);
    WG_PH(5);
#ifdef SSPP_WG_TIMING
    if (tid == 0 && blockIdx.x < (1 << 16)) {
        g_wg_t[4 * blockIdx.x] = wg_t0;
        g_wg_t[4 * blockIdx.x + 1] = wall_clock64();
        g_wg_t[4 * blockIdx.x + 2] = __smid();
        g_wg_t[4 * blockIdx.x + 3] = (unsigned long long)(long long)wg_ns;
    }
#endif
}

// ---------------------------------------------------------------- undecided cylinder-box pairs
// k_sspp_c2f leaves a cylinder-box pair that passes the bounding-sphere test undecided (the
// exact test's registers would spill its whole pair loop).  A candidate with no other contact is
// written as feasible = 2, kept out of the argmin and counted in dfr[0].  This kernel, queued
// right after it on the same stream, gives each such candidate the exact test at every
// collision waypoint: a contact makes it infeasible (arc +inf unless arc_all), otherwise it is
// feasible and is merged into its step's records (block record and fused result, lexicographic
// (cost, id) under the step's lock, count + 1), so the outputs equal a kernel that ran the exact
// test inline.  With dfr[0] == 0 (every scene without such pairs near a path) each workgroup
// returns after one scalar load.  The last workgroup to finish re-arms dfr.
constexpr int kFixThreads = 256;
constexpr int kFixBlocks = 64;
template <int D, int NM, int P, bool ONEGEOM>
__global__ __launch_bounds__(kFixThreads) void k_sspp_cbfix(
    SsppC2F a, SceneT T, int steps, const double* __restrict__ otab, const int* __restrict__ ospan,
    const double* __restrict__ init_ctrl, const double* __restrict__ limits,
    const double* __restrict__ ctrl_in, const double* __restrict__ pert, double* __restrict__ arc,
    unsigned char* __restrict__ feasible, BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    if (__hip_atomic_load(a.dfr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) return;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int P1 = P + 1;
    __shared__ int s_list[kFixThreads + 1];
    __shared__ int s_hit;
    const int tid = threadIdx.x, n = a.n, ndof = n * D;
    double* s_ctrl = smem;  // [n][D]
    const long long total = (long long)steps * a.B;
    for (long long base = (long long)blockIdx.x * kFixThreads; base < total; base += (long long)gridDim.x * kFixThreads) {
        const long long c0 = base + tid;
        if (tid == 0) s_list[kFixThreads] = 0;
        __syncthreads();
        if (c0 < total && feasible[c0] == 2) s_list[atomicAdd(&s_list[kFixThreads], 1)] = tid;
        __syncthreads();
        const int nl = s_list[kFixThreads];
        for (int i = 0; i < nl; ++i) {  // workgroup-uniform
            const long long c = base + s_list[i];
            const int step = (int)(c / a.B);
            const long long cand = c - (long long)step * a.B;
            const long long first_id = a.first_id + step * a.step_stride;
            // the candidate's control points, exactly as k_sspp_c2f's prologue made them
            const int npert = (n - 2 * P) * D;
            for (int r = tid; r < ndof; r += kFixThreads) {
                const int k = r - P * D;
                double v = init_ctrl[r];
                if (ctrl_in) v = ctrl_in[cand * ndof + r];
                else if (pert && !a.insample && !(a.ablate & 1) && k >= 0 && k < npert)
                    v = pert[((long long)step * a.B + cand) * npert + k];
                s_ctrl[r] = v;
            }
            if (tid == 0) s_hit = 0;
            __syncthreads();
            if (!ctrl_in && a.insample && !(a.ablate & 1)) {
                const int nq = (npert + 3) >> 2;
                for (int m = tid; m < nq; m += kFixThreads) {
                    double z[4];
                    normal_quad(a.seed, (unsigned long long)(first_id + cand), (unsigned)m, 0u, z);
                    double* cc = s_ctrl + P * D;
                    for (int h = 0; h < 4; ++h) {
                        const int k = 4 * m + h;
                        if (k < npert) cc[k] = cc[k] + (a.sigma * z[h]) * limits[k % D];
                    }
                }
                __syncthreads();
            }
            for (int j = tid; j < a.npts; j += kFixThreads) {
                if (__hip_atomic_load(&s_hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
                if (cb_point_exact<D, NM, P, ONEGEOM>(s_ctrl, otab + j * P1, ospan[j], ~0ull, a.sc.npairs, T))
                    __hip_atomic_store(&s_hit, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __syncthreads();
            if (tid == 0) {
                if (s_hit) {
                    feasible[c] = 0;
                    if (!a.arc_all) arc[c] = INFINITY;
                } else {
                    feasible[c] = 1;
                    const double cost = arc[c];
                    const long long id = first_id + cand;
                    unsigned* lock = &sync[step].top[1];
                    while (atomicCAS(lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(2);
                    __threadfence();
                    BlockBest* pb = part + (long long)step * a.nblk_step + cand / a.cpb;
                    BlockBest r = ld_rec(pb);
                    if (better(cost, id, r.cost, r.idx)) { r.cost = cost; r.idx = id; }
                    r.count += 1;
                    st_rec(pb, r);
                    if (best) {
                        volatile sspp_best* o = best + step;
                        if (better(cost, id, o->cost, o->index)) { o->cost = cost; o->index = id; }
                        o->count = o->count + 1;
                    }
                    __threadfence();
                    atomicExch(lock, 0u);
                }
            }
            __syncthreads();
        }
    }
    // the last workgroup re-arms the counters for the next launch on this job
    if (tid == 0) {
        __threadfence();
        const unsigned prev = __hip_atomic_fetch_add(a.dfr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(a.dfr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.dfr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// ---------------------------------------------------------------- TaskSpacePlanner kernel
// tab: (cp+1) rows of 3 basis values at u = i * (1/cp); Minv: collocation inverse (n x n).
#ifndef SSPP_TSP_WAVES_PER_EU
#define SSPP_TSP_WAVES_PER_EU 3
#endif
#ifndef SSPP_TSP_WAVES_PER_EU_CB  // with the exact cylinder-box test (its live state doubles)
#define SSPP_TSP_WAVES_PER_EU_CB 2
#endif
// CB: the scene has cylinder-box pairs (without them the exact cylinder-box code is compiled
// out: it costs registers even when it never runs)
template <int NM, bool ONEGEOM, bool CB>
__global__ __launch_bounds__(kBlock, CB ? SSPP_TSP_WAVES_PER_EU_CB : SSPP_TSP_WAVES_PER_EU) void k_tsp(
    TspK a, SceneT T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ Minv, const double* __restrict__ mean,
    const double* __restrict__ sigma, const double* __restrict__ vias_in,
    double* __restrict__ vias_out, double* __restrict__ oL, double* __restrict__ oCnf,
    double* __restrict__ oCwf, double* __restrict__ ocost, unsigned char* __restrict__ ostatus,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int D = 4, P = 2, P1 = 3;
    const int tid = threadIdx.x, lpc = a.lpc, cpb = a.cpb, n = a.n, K = a.K, cp = a.cp;
    const int slot = tid / lpc, lane = tid - slot * lpc;
    const long long cand0 = (long long)blockIdx.x * cpb;
    const int ndof = n * D;
    double* s_V = smem;                      // [cpb][n][4]
    double* s_ctrl = s_V + cpb * ndof;       // [cpb][n][4]
    double* s_wsum = s_ctrl + cpb * ndof;    // [3][4]
    double* s_best = s_wsum + 3 * (kBlock / 64);
    int* s_stat = (int*)(s_best + 4);        // [cpb]

    const long long nvalid = min((long long)cpb, a.B - cand0);
    const long long nfx = a.ces ? (long long)*a.nfixed : 0;  // uniform: scalar load
    for (int e = tid; e < cpb * 2 * D; e += kBlock) {
        const int s = e / (2 * D), r = e - s * 2 * D;
        if (r < D) s_V[s * ndof + r] = a.start[r];
        else s_V[s * ndof + (n - 1) * D + (r - D)] = a.end[r - D];
    }
    if (vias_in) {
        for (int e = tid; e < nvalid * K * D; e += kBlock) {
            const int s = e / (K * D), r = e - s * K * D;
            s_V[s * ndof + D + r] = vias_in[(cand0 + s) * K * D + r];
        }
    } else {
        // Sampler::sample_set (tsp_sampler.h:12-51) with Philox streams per (candidate, via, dim)
        for (int e = tid; e < cpb * K * D; e += kBlock) {
            const int s = e / (K * D), r = e - s * K * D;
            if (s >= nvalid) continue;
            const int v = r / D, i = r - v * D;
            long long gi = cand0 + s;
            if (a.ces) {
                const long long slot = a.slot0 + cand0 + s;
                if (slot < nfx) {  // mean set / forwarded best: no sampling
                    s_V[s * ndof + D + r] = a.fixed[(slot * K + v) * D + i];
                    continue;
                }
                gi = slot - nfx;
                if (gi >= a.samples) {  // padding slot
                    s_V[s * ndof + D + r] = mean[v * D + i];
                    continue;
                }
            }
            const unsigned long long g = (unsigned long long)(a.first_id + gi);
            const double m = mean[v * D + i], sg = sigma[v * D + i];
            double val;
            if (i < 3) {
                bool ok = false;
                val = 0.0;
                for (int t = 0; t < 99; ++t) {
                    double z0, z1;
                    normal_pair(a.seed, g, (unsigned)(((v * 4 + i) << 7) | t), 1u, &z0, &z1);
                    val = z0 * sg;
                    val = val + m;
                    if (!(val < a.lo[i] || val > a.hi[i])) { ok = true; break; }
                }
                if (!ok) {
                    double u = uniform01(a.seed, g, (unsigned)(((v * 4 + i) << 7) | 127), 1u);
                    val = u * (a.hi[i] - a.lo[i]);
                    val = val + a.lo[i];
                }
                if (i == 2 && val < a.z_min) val = a.z_min;
            } else if (a.lo[3] != a.hi[3]) {
                double z0, z1;
                normal_pair(a.seed, g, (unsigned)((v * 4 + 3) << 7), 1u, &z0, &z1);
                val = z0 * sg;
                val = val + m;
                const double range = a.hi[3] - a.lo[3];
                while (val < a.lo[3]) val += range;
                while (val > a.hi[3]) val -= range;
            } else {
                val = m;
            }
            s_V[s * ndof + D + r] = val;
        }
    }
    __syncthreads();
    if (vias_out) {
        for (int e = tid; e < nvalid * K * D; e += kBlock) {
            const int s = e / (K * D), r = e - s * K * D;
            vias_out[(cand0 + s) * K * D + r] = s_V[s * ndof + D + r];
        }
    }
    // PathModel::fromVias: ctrl = A^-1 V (collocation inverse precomputed on the host)
    for (int e = tid; e < cpb * ndof; e += kBlock) {
        const int s = e / ndof, r = e - s * ndof, j = r / D, d = r - j * D;
        const double* Vs = s_V + s * ndof;
        double acc = Minv[j * n] * Vs[d];
        for (int i = 1; i < n; ++i) acc = fma(Minv[j * n + i], Vs[i * D + d], acc);
        s_ctrl[e] = acc;
    }
    __syncthreads();

    // Evaluator::eval_one_pass (tsp_evaluator.h:18-32), waypoint i = 1..cp per lane
    const bool valid = slot < nvalid;
    const double* myc = s_ctrl + slot * ndof;
    const unsigned long long mask = hull_mask<D, NM, 1>(myc, n, a.sc.npairs, (cpair_t)T.pairs,
                                                        (cgeom_t)T.geoms, (cmover_t)T.movers);
    double aL = 0.0, aC = 0.0, aW = 0.0;
    // cp <= lpc: one waypoint per lane, so s((i-1)du) is the previous lane's s(i du); take it
    // by shuffle (bit-identical: same eval_pt inputs) except on a wave's first lane
    const bool one_pass = cp <= lpc;
    if (valid) {
        for (int j = lane; j < cp; j += lpc) {
            const int i = j + 1;
            double pv[4], pc[4];
            eval_pt<D, P>(myc, tab + i * P1, span[i], pc);
            if (one_pass) {
#pragma unroll
                for (int d = 0; d < D; ++d) pv[d] = __shfl_up(pc[d], 1, 64);
                if ((tid & 63) == 0) eval_pt<D, P>(myc, tab + (i - 1) * P1, span[i - 1], pv);
            } else {
                eval_pt<D, P>(myc, tab + (i - 1) * P1, span[i - 1], pv);
            }
            aL = aL + dist_nd<D>(pv, pc);
            double c = 0.0;
#ifndef SSPP_PROF_NOCOLL  // profiling variant only
            point_collide<D, NM, 1, true, ONEGEOM, CB>(pc, a.sc, T, mask, &c);
#endif
            const double deficit = (a.floor_z_min + a.floor_margin) - pc[2];
            const double fp = deficit > 0.0 ? (a.floor_scale * deficit) * deficit : 0.0;
            aC = aC + c;
            aW = aW + (c + fp);
        }
    }
    aL = wave_sum(aL);
    aC = wave_sum(aC);
    aW = wave_sum(aW);
    constexpr int NW = kBlock / 64;
    if ((tid & 63) == 0) {
        s_wsum[tid >> 6] = aL;
        s_wsum[NW + (tid >> 6)] = aC;
        s_wsum[2 * NW + (tid >> 6)] = aW;
    }
    __syncthreads();
    if (lane == 0 && valid) {
        const int w0 = (slot * lpc) >> 6, nw = lpc >> 6;
        double L = s_wsum[w0], Cn = s_wsum[NW + w0], Cw = s_wsum[2 * NW + w0];
        for (int w = 1; w < nw; ++w) {
            L = L + s_wsum[w0 + w];
            Cn = Cn + s_wsum[NW + w0 + w];
            Cw = Cw + s_wsum[2 * NW + w0 + w];
        }
        const long long c = cand0 + slot;
        int st = Cn == 0.0;
        double cost = L + a.w_col * Cw;
        if (a.ces && a.slot0 + c >= nfx + a.samples) {  // padding slot
            st = 0; cost = INFINITY; L = 0.0; Cn = 0.0; Cw = 0.0;
        }
        oL[c] = L; oCnf[c] = Cn; oCwf[c] = Cw; ocost[c] = cost;
        ostatus[c] = (unsigned char)st;
        s_stat[slot] = st;
        s_best[slot] = cost;
    }
    __syncthreads();
    BlockBest bb;
    if (tid == 0) {
        bb.cost = INFINITY; bb.idx = -1; bb.count = 0; bb.pad = 0;
        for (int s = 0; s < nvalid; ++s) {
            if (!s_stat[s]) continue;
            bb.count++;
            if (s_best[s] < bb.cost) { bb.cost = s_best[s]; bb.idx = a.first_id + cand0 + s; }
        }
    }
    finish_batch(bb, part, sync, best);
}

// ---------------------------------------------------------------- argmin over block results

constexpr int kArgminThreads = 1024;
__global__ __launch_bounds__(kArgminThreads) void k_argmin(const BlockBest* __restrict__ part,
                                                           int nparts, sspp_best* out) {
    __shared__ double sc[kArgminThreads / 64];
    __shared__ long long si[kArgminThreads / 64], sn[kArgminThreads / 64];
    double bc = INFINITY;
    long long bi = -1, cnt = 0;
    for (int i = threadIdx.x; i < nparts; i += kArgminThreads) {
        const BlockBest b = part[i];
        cnt += b.count;
        if (better(b.cost, b.idx, bc, bi)) { bc = b.cost; bi = b.idx; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double oc = __shfl_xor(bc, off, 64);
        const long long oi = __shfl_xor(bi, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
        if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sc[w] = bc; si[w] = bi; sn[w] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double c = sc[0];
        long long i = si[0], n = sn[0];
        for (int k = 1; k < kArgminThreads / 64; ++k) {
            n += sn[k];
            if (better(sc[k], si[k], c, i)) { c = sc[k]; i = si[k]; }
        }
        out->cost = i < 0 ? INFINITY : c;
        out->index = i;
        out->count = n;
        out->reserved = 0;
    }
}

int lanes_for(int items) {
    int l = ((items + 63) / 64) * 64;
    return std::min(std::max(l, 64), kBlock);
}

}  // namespace

// =============================================================== host side: scene + jobs
struct sspp_scene {
    int mode, arg, dof;
    int count_static;
    std::vector<DGeom> geoms;
    std::vector<DPair> pairs;
    std::vector<DMover> movers;
    int n_moving_geoms = 0, n_static_geoms = 0, n_static_pairs = 0, static_contacts = 0;
    double static_cost = 0.0;
    DGeom* d_geoms = nullptr;
    DPair* d_pairs = nullptr;
    DMover* d_movers = nullptr;
    int device = 0;
};

struct sspp_job {
    int kind = 0;  // 0 sspp, 1 tsp
    const sspp_scene* scene = nullptr;
    int D = 0, p = 0, n = 0, W = 0, nknots = 0, K = 0, cp = 0;
    int lpc = 0, cpb = 0, nm = 1, shared_endpoints = 0;
    size_t lds = 0;
    int64_t max_batch = 0;
    double sigma = 0.0;
    uint64_t seed = 0;
    double* d_knots = nullptr;
    double* d_tab = nullptr;   // basis rows (host-precomputed, P+1 doubles per waypoint)
    int* d_span = nullptr;     // knot span per waypoint
    double* d_init = nullptr;
    double* d_limits = nullptr;
    double* d_Minv = nullptr;
    double* d_mean = nullptr;
    double* d_sigma = nullptr;
    BlockBest* d_part = nullptr;
    double* d_pert = nullptr;  // sampler output: perturbed columns [pert_steps][max_batch][(n-2p)*D]
    int npert = 0;
    int pert_steps = 1;        // steps per launch the sampler buffer holds
    int insample = 0;          // sample inside the scoring kernel (SSPP_INSAMPLE=1)
    // coarse-to-fine kernel (k_sspp_c2f; SSPP_KERNEL=0 selects the one-waypoint-per-lane k_sspp)
    int c2f = 1, g1 = 16, cpb2 = 16, n1 = 16, nt2 = 256;
    int arc_all = 0;           // arc length for every candidate (else collision-free only)
    int hull = 2;              // c2f hull broadphase (SSPP_HULL: 0 off, 1 all, 2 survivors)
    size_t lds2 = 0;
    double* d_otab = nullptr;  // collision rows in coarse-to-fine order
    int* d_ospan = nullptr;
    DPair* d_pairs = nullptr;  // this job's pair table (closest-to-the-mean-path first)
    ArgminSync* d_sync = nullptr;  // sharded arrival counters of the fused argmin [kMaxSteps]
    unsigned* d_dfr = nullptr;     // k_sspp_c2f -> k_sspp_cbfix counters (SsppC2F::dfr)
    int has_cb = 0;                // the pair table has cylinder-box pairs (k_sspp_cbfix runs)
    std::vector<double> h_knots;   // host copies: the knot vector, and the staging of
    std::vector<double> h_stage;   // sspp_job_update_sspp's asynchronous uploads (init | limits)
    std::vector<DPair> h_pairs;
    double start[4], end[4], lo[4], hi[4];
    double z_min = 0, w_col = 1, floor_z_min = 0, floor_margin = 0.01, floor_scale = 10;
};

namespace {

int hip_fail(hipError_t e, const char* what) {
    return sspp::set_error(SSPP_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIPCHK(x)                                   \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return hip_fail(e_, #x); \
    } while (0)

template <class T>
int upload(T** dst, const T* src, size_t count) {
    if (count == 0) { *dst = nullptr; return SSPP_OK; }
    HIPCHK(hipMalloc((void**)dst, sizeof(T) * count));
    HIPCHK(hipMemcpy(*dst, src, sizeof(T) * count, hipMemcpyHostToDevice));
    return SSPP_OK;
}

// MuJoCo-like kinematics on the host (same operation order as oracle/sspp_oracle.c::fk)
void host_fk(const sspp_model& m, const std::vector<double>& qpos, std::vector<double>& xpos,
             std::vector<double>& xquat, std::vector<double>& xmat, std::vector<double>& gxpos,
             std::vector<double>& gxmat) {
    int nb = m.nbody(), ng = m.ngeom();
    xpos.assign(3 * nb, 0.0); xquat.assign(4 * nb, 0.0); xmat.assign(9 * nb, 0.0);
    gxpos.assign(3 * ng, 0.0); gxmat.assign(9 * ng, 0.0);
    xquat[0] = 1.0;
    quat2mat(&xquat[0], &xmat[0]);
    for (int b = 1; b < nb; ++b) {
        double* p = &xpos[3 * b];
        double* q = &xquat[4 * b];
        if (m.body_jnt_type[b] == 0) {
            const double* qp = &qpos[m.body_qpos_adr[b]];
            p[0] = qp[0]; p[1] = qp[1]; p[2] = qp[2];
            q[0] = qp[3]; q[1] = qp[4]; q[2] = qp[5]; q[3] = qp[6];
        } else {
            int pa = m.body_parent[b];
            double t[3];
            matvec3(&xmat[9 * pa], &m.body_pos[3 * b], t);
            p[0] = xpos[3 * pa] + t[0]; p[1] = xpos[3 * pa + 1] + t[1]; p[2] = xpos[3 * pa + 2] + t[2];
            mulquat(&xquat[4 * pa], &m.body_quat[4 * b], q);
        }
        normalize4(q);
        quat2mat(q, &xmat[9 * b]);
    }
    for (int g = 0; g < ng; ++g) {
        int b = m.geom_body[g];
        double t[3], gq[4];
        matvec3(&xmat[9 * b], &m.geom_pos[3 * g], t);
        gxpos[3 * g] = xpos[3 * b] + t[0];
        gxpos[3 * g + 1] = xpos[3 * b + 1] + t[1];
        gxpos[3 * g + 2] = xpos[3 * b + 2] + t[2];
        mulquat(&xquat[4 * b], &m.geom_quat[4 * g], gq);
        normalize4(gq);
        quat2mat(gq, &gxmat[9 * g]);
    }
}

}  // namespace

extern "C" {

int sspp_scene_create(const sspp_model* m, int mode, int arg, int count_static, sspp_scene** out) {
    sspp::clear_error();
    if (!m || !out) return sspp::set_error(SSPP_E_INVAL, "sspp_scene_create: null argument");
    const int nb = m->nbody(), ng = m->ngeom();
    std::vector<int> weld(nb, 0), moving(nb, 0);
    for (int b = 1; b < nb; ++b)
        weld[b] = (m->body_jnt_type[b] != -1) ? b : weld[m->body_parent[b]];
    std::vector<int> mover_of(nb, -1);
    std::vector<int> mover_bodies;
    if (mode == SSPP_MODE_QPOS) {
        if (arg < 1 || arg > 16) return sspp::set_error(SSPP_E_INVAL, "dof must be in [1, 16]");
        if (arg > (int)m->qpos0.size())
            return sspp::set_error(SSPP_E_SCENE, "model has nq=" + std::to_string(m->qpos0.size()) +
                                                     " < dof=" + std::to_string(arg));
        for (int b = 1; b < nb; ++b)
            if (m->body_jnt_type[b] == 0 && m->body_qpos_adr[b] < arg) {
                moving[b] = 1;
                mover_of[b] = (int)mover_bodies.size();
                mover_bodies.push_back(b);
            }
    } else if (mode == SSPP_MODE_BODY) {
        if (arg <= 0 || arg >= nb || m->body_jnt_type[arg] != 0)
            return sspp::set_error(SSPP_E_SCENE, "collision body must have a free joint");
        moving[arg] = 1;
        mover_of[arg] = 0;
        mover_bodies.push_back(arg);
    } else {
        return sspp::set_error(SSPP_E_INVAL, "unknown scene mode");
    }
    if ((int)mover_bodies.size() > kMaxMovers)
        return sspp::set_error(SSPP_E_UNSUPPORTED, "more than 2 moving free bodies");
    for (size_t i = 0; i < mover_bodies.size(); ++i)
        if (mode == SSPP_MODE_QPOS && m->body_qpos_adr[mover_bodies[i]] != 7 * (int)i)
            return sspp::set_error(SSPP_E_UNSUPPORTED, "free joints must occupy qpos[7k:7k+7]");

    auto* s = new sspp_scene();
    s->mode = mode; s->arg = arg; s->dof = mode == SSPP_MODE_QPOS ? arg : 4;
    s->count_static = count_static;
    (void)hipGetDevice(&s->device);

    // kinematics at qpos0: world poses of static geoms
    std::vector<double> xpos, xquat, xmat, gxpos, gxmat;
    host_fk(*m, m->qpos0, xpos, xquat, xmat, gxpos, gxmat);
    // moving geoms relative to their mover root: same FK with every mover at the identity
    std::vector<double> qrel = m->qpos0;
    for (int b : mover_bodies) {
        int adr = m->body_qpos_adr[b];
        double id[7] = {0, 0, 0, 1, 0, 0, 0};
        for (int k = 0; k < 7; ++k) qrel[adr + k] = id[k];
    }
    std::vector<double> rxpos, rxquat, rxmat, rgxpos, rgxmat;
    host_fk(*m, qrel, rxpos, rxquat, rxmat, rgxpos, rgxmat);

    std::vector<int> table_index(ng, -1);
    for (int g = 0; g < ng; ++g) {
        int b = m->geom_body[g];
        int w = weld[b];
        bool mv = moving[w];
        DGeom dg{};
        dg.type = m->geom_type[g];
        dg.mover = mv ? mover_of[w] : -1;
        dg.orig = g;
        const std::vector<double>& P = mv ? rgxpos : gxpos;
        const std::vector<double>& M = mv ? rgxmat : gxmat;
        for (int k = 0; k < 3; ++k) dg.pos[k] = P[3 * g + k];
        for (int k = 0; k < 9; ++k) dg.mat[k] = M[9 * g + k];
        for (int k = 0; k < 3; ++k) dg.size[k] = m->geom_size[3 * g + k];
        dg.rbound = geom_rbound(dg.type, dg.size);
        dg.relrot = 0;
        for (int k = 0; k < 9; ++k) dg.relrot |= dg.mat[k] != ((k % 4 == 0) ? 1.0 : 0.0);
        dg.reach = mv ? std::sqrt(dg.pos[0] * dg.pos[0] + dg.pos[1] * dg.pos[1] + dg.pos[2] * dg.pos[2]) * (1.0 + 1e-12)
                      : 0.0;
        table_index[g] = (int)s->geoms.size();
        s->geoms.push_back(dg);
        if (m->geom_contype[g] || m->geom_conaffinity[g]) {
            if (mv) s->n_moving_geoms++; else s->n_static_geoms++;
        }
    }
    // mj_collision pair filter, (g1 < g2) order
    struct P2 { int g1, g2; double margin; bool stat; };
    std::vector<P2> all;
    for (int g1 = 0; g1 < ng; ++g1) {
        for (int g2 = g1 + 1; g2 < ng; ++g2) {
            int b1 = m->geom_body[g1], b2 = m->geom_body[g2];
            int w1 = weld[b1], w2 = weld[b2];
            if (w1 == w2) continue;
            int ct1 = m->geom_contype[g1], ca1 = m->geom_conaffinity[g1];
            int ct2 = m->geom_contype[g2], ca2 = m->geom_conaffinity[g2];
            if (!((ct1 & ca2) || (ct2 & ca1))) continue;
            if (w1 != 0 && w2 != 0 &&
                (w1 == weld[m->body_parent[w2]] || w2 == weld[m->body_parent[w1]]))
                continue;
            bool excl = false;
            for (size_t e = 0; e + 1 < m->exclude.size(); e += 2) {
                int e1 = m->exclude[e], e2 = m->exclude[e + 1];
                if ((e1 == b1 && e2 == b2) || (e1 == b2 && e2 == b1)) { excl = true; break; }
            }
            if (excl) continue;
            if (!pair_supported(m->geom_type[g1], m->geom_type[g2])) {
                delete s;
                return sspp::set_error(SSPP_E_UNSUPPORTED,
                                       "unsupported collision pair: geom '" + m->geom_names[g1] +
                                           "' (type " + std::to_string(m->geom_type[g1]) + ") vs '" +
                                           m->geom_names[g2] + "' (type " +
                                           std::to_string(m->geom_type[g2]) + ")");
            }
            double mg = std::max(m->geom_margin[g1], m->geom_margin[g2]);
            all.push_back({g1, g2, mg, !(moving[w1] || moving[w2])});
        }
    }
    // env-env pairs: constant over waypoints -> evaluated once here (same device math)
    for (auto& pr : all) {
        if (!pr.stat) continue;
        s->n_static_pairs++;
        const DGeom& A = s->geoms[table_index[pr.g1]];
        const DGeom& B = s->geoms[table_index[pr.g2]];
        double dc[3] = {B.pos[0] - A.pos[0], B.pos[1] - A.pos[1], B.pos[2] - A.pos[2]};
        if (A.rbound > 0.0 && B.rbound > 0.0) {
            double thr = A.rbound + B.rbound + pr.margin;
            if (dot3(dc, dc) > thr * thr) continue;
        }
        bool afirst = A.type <= B.type;
        const DGeom& F = afirst ? A : B;
        const DGeom& S = afirst ? B : A;
        int nd = 0;
        int nc = collide<false>(F.type, F.pos, F.mat, F.size, S.type, S.pos, S.mat, S.size, pr.margin, &nd);
        collide<true>(F.type, F.pos, F.mat, F.size, S.type, S.pos, S.mat, S.size, pr.margin, &nd);
        s->static_contacts += nc;
        if (nd > 0) {
            double term = -1.0 / (sqrt(dot3(dc, dc)) + 1e-4);
            for (int i = 0; i < nd; ++i) s->static_cost = s->static_cost + term;
        }
    }
    // moving pairs: sspp mode groups by moving geom (pose computed once per group);
    // tsp mode keeps the oracle's (g1, g2) order so per-waypoint cost sums match bit for bit.
    std::vector<P2> mov;
    for (auto& pr : all)
        if (!pr.stat) mov.push_back(pr);
    auto moving_geom = [&](const P2& pr) {
        int w1 = weld[m->geom_body[pr.g1]];
        return moving[w1] ? pr.g1 : pr.g2;
    };
    if (mode == SSPP_MODE_QPOS) {
        std::stable_sort(mov.begin(), mov.end(), [&](const P2& x, const P2& y) {
            return moving_geom(x) < moving_geom(y);
        });
    }
    for (auto& pr : mov) {
        int gm = moving_geom(pr);
        int go = gm == pr.g1 ? pr.g2 : pr.g1;
        DPair dp{};
        dp.gm = table_index[gm];
        dp.go = table_index[go];
        const DGeom& O = s->geoms[dp.go];
        dp.otype = O.type;
        dp.oorig = O.orig;
        dp.omover = O.mover;
        dp.margin = pr.margin;
        for (int k = 0; k < 3; ++k) dp.opos[k] = O.pos[k];
        for (int k = 0; k < 9; ++k) dp.omat[k] = O.mat[k];
        for (int k = 0; k < 3; ++k) dp.osize[k] = O.size[k];
        dp.orbound = O.rbound;
        s->pairs.push_back(dp);
    }
    for (size_t i = 0; i < mover_bodies.size(); ++i) {
        DMover mv{};
        mv.qpos_adr = m->body_qpos_adr[mover_bodies[i]];
        for (int k = 0; k < 7; ++k) mv.qpos0[k] = m->qpos0[mv.qpos_adr + k];
        s->movers.push_back(mv);
    }
    int rc;
    if ((rc = upload(&s->d_geoms, s->geoms.data(), s->geoms.size())) ||
        (rc = upload(&s->d_pairs, s->pairs.data(), s->pairs.size())) ||
        (rc = upload(&s->d_movers, s->movers.data(), s->movers.size()))) {
        sspp_scene_free(s);
        return rc;
    }
    *out = s;
    return SSPP_OK;
}

int sspp_scene_get_info(const sspp_scene* s, sspp_scene_info* out) {
    if (!s || !out) return sspp::set_error(SSPP_E_INVAL, "null argument");
    out->n_moving_geoms = s->n_moving_geoms;
    out->n_static_geoms = s->n_static_geoms;
    out->n_pairs = (int)s->pairs.size();
    out->n_static_pairs = s->n_static_pairs;
    out->static_contacts = s->static_contacts;
    out->n_movers = (int)s->movers.size();
    out->static_cost = s->static_cost;
    return SSPP_OK;
}

void sspp_scene_free(sspp_scene* s) {
    if (!s) return;
    if (s->d_geoms) (void)hipFree(s->d_geoms);
    if (s->d_pairs) (void)hipFree(s->d_pairs);
    if (s->d_movers) (void)hipFree(s->d_movers);
    delete s;
}

}  // extern "C"

static KScene kscene(const sspp_scene* s, bool tsp) {
    KScene k{};
    if (!s) return k;
    k.npairs = (int)s->pairs.size();
    k.onegeom = 1;
    for (const DPair& p : s->pairs) k.onegeom &= (p.gm == s->pairs[0].gm);
    k.static_block = (!tsp && s->count_static && s->static_contacts > 0) ? 1 : 0;
    k.static_cost = tsp ? s->static_cost : 0.0;
    for (const DPair& p : s->pairs) {
        const int tg = s->geoms[p.gm].type;
        k.cylbox |= (tg == 5 && p.otype == 6) || (tg == 6 && p.otype == 5);
    }
    return k;
}

static SceneT scene_t(const sspp_scene* s) {
    SceneT t{};
    if (!s) return t;
    t.geoms = s->d_geoms;
    t.pairs = s->d_pairs;
    t.movers = s->d_movers;
    return t;
}

// Pair order for the feasibility scan of one job.  checkCollision's answer is an OR over pairs,
// so the order is free; the scan stops at the first pair in contact, so the pairs the sampled
// paths most often touch should come first.  Heuristic: the smallest bounding-sphere gap
// (planes: height of the geom centre minus its radius) between the moving geom and the partner
// along the mean path (the init spline, 33 points), ascending; ties keep the scene order.
static std::vector<DPair> pairs_for_job(const sspp_scene* sc, const double* knots, int nknots, int p,
                                        const double* ctrl, int D) {
    std::vector<DPair> out = sc->pairs;
    const int np = (int)out.size();
    if (np < 2) return out;
    std::vector<double> gap(np, 1e300);
    const int nm = (int)sc->movers.size();
    const int n = nknots - p - 1;
    for (int t = 0; t <= 32; ++t) {
        const double u = t / 32.0;
        const int sp = span_of(u, p, knots, nknots);
        double N[kMaxP + 1];
        basis_funcs(u, p, sp, knots, N);
        double q[16] = {0};
        for (int d = 0; d < D && d < 16; ++d) {
            double acc = 0.0;
            for (int r = 0; r <= p; ++r) {
                const int j = sp - p + r;
                if (j >= 0 && j < n) acc += N[r] * ctrl[j * D + d];
            }
            q[d] = acc;
        }
        double mp[kMaxMovers][3], mR[kMaxMovers][9];
        for (int m = 0; m < nm && m < kMaxMovers; ++m) {
            double qp[7];
            for (int k = 0; k < 7; ++k) qp[k] = (7 * m + k < D) ? q[7 * m + k] : sc->movers[m].qpos0[k];
            normalize4(qp + 3);
            quat2mat(qp + 3, mR[m]);
            for (int k = 0; k < 3; ++k) mp[m][k] = qp[k];
        }
        for (int k = 0; k < np; ++k) {
            const DPair& pr = out[k];
            const DGeom& G = sc->geoms[pr.gm];
            const int m = G.mover > 0 ? G.mover : 0;
            double t3[3], gp[3], op[3];
            matvec3(mR[m], G.pos, t3);
            for (int d = 0; d < 3; ++d) gp[d] = mp[m][d] + t3[d];
            if (pr.omover >= 0) {
                matvec3(mR[pr.omover], pr.opos, t3);
                for (int d = 0; d < 3; ++d) op[d] = mp[pr.omover][d] + t3[d];
            } else {
                for (int d = 0; d < 3; ++d) op[d] = pr.opos[d];
            }
            double g;
            if (pr.otype == 0) {
                const double nz[3] = {pr.omat[2], pr.omat[5], pr.omat[8]};
                g = (gp[0] - op[0]) * nz[0] + (gp[1] - op[1]) * nz[1] + (gp[2] - op[2]) * nz[2] - G.rbound;
            } else if (G.rbound > 0.0 && pr.orbound > 0.0) {
                const double dx = gp[0] - op[0], dy = gp[1] - op[1], dz = gp[2] - op[2];
                g = std::sqrt(dx * dx + dy * dy + dz * dz) - G.rbound - pr.orbound;
            } else {
                g = 0.0;
            }
            gap[k] = std::min(gap[k], g);
        }
    }
    std::vector<int> idx(np);
    for (int k = 0; k < np; ++k) idx[k] = k;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return gap[a] < gap[b]; });
    std::vector<DPair> sorted(np);
    for (int k = 0; k < np; ++k) sorted[k] = out[idx[k]];
    return sorted;
}

// Coarse-to-fine order of the collision waypoints 0..W: breadth-first interval bisection, so
// every prefix is spread evenly over the path (k_sspp_c2f phase 1 tests a prefix).
static std::vector<int> c2f_order(int W) {
    std::vector<int> ord;
    std::vector<std::pair<int, int>> cur{{0, W}}, next;
    while (!cur.empty()) {
        next.clear();
        for (auto [lo, hi] : cur) {
            if (lo > hi) continue;
            const int mid = lo + (hi - lo) / 2;
            ord.push_back(mid);
            next.push_back({lo, mid - 1});
            next.push_back({mid + 1, hi});
        }
        cur.swap(next);
    }
    return ord;
}

// Basis rows for a list of parameters (same A2.1/A2.2 code as the device header).
static int upload_basis(const std::vector<double>& us, int p, const double* knots, int nknots,
                        double** d_tab, int** d_span) {
    std::vector<double> tab(us.size() * (p + 1));
    std::vector<int> sp(us.size());
    for (size_t i = 0; i < us.size(); ++i) {
        sp[i] = span_of(us[i], p, knots, nknots);
        basis_funcs(us[i], p, sp[i], knots, &tab[i * (p + 1)]);
    }
    int rc = upload(d_tab, tab.data(), tab.size());
    if (rc) return rc;
    return upload(d_span, sp.data(), sp.size());
}

extern "C" int sspp_job_create_sspp(const sspp_scene* scene, const sspp_sspp_args* a, int64_t max_batch,
                         sspp_job** out) {
    sspp::clear_error();
    if (!a || !out || !a->knots || !a->init_ctrl || !a->limits)
        return sspp::set_error(SSPP_E_INVAL, "sspp_job_create_sspp: null argument");
    const int D = a->dof, p = a->degree, n = a->n_ctrl, W = a->check_points;
    if (!(D == 1 || D == 2 || D == 3 || D == 4 || D == 6 || D == 7 || D == 9))
        return sspp::set_error(SSPP_E_UNSUPPORTED, "dof must be one of 1,2,3,4,6,7,9");
    if (p < 2 || p > 3) return sspp::set_error(SSPP_E_UNSUPPORTED, "GPU scorer supports spline degree 2 or 3");
    if (n < p + 1) return sspp::set_error(SSPP_E_INVAL, "need at least degree + 1 control points");
    // W = 1 is checkCollision(num_samples = 1): u = 0 and 1 (include/sspp.h:134-137); its arc
    // grid is the single point u = 0 (no chord, arc length 0)
    if (W < 1 || W > 1 << 20) return sspp::set_error(SSPP_E_INVAL, "check_points must be >= 1");
    if (max_batch < 1) return sspp::set_error(SSPP_E_INVAL, "max_batch must be >= 1");
    if (scene && (scene->mode != SSPP_MODE_QPOS || scene->dof != D))
        return sspp::set_error(SSPP_E_INVAL, "scene was not bound for this dof");
    auto* j = new sspp_job();
    j->kind = 0; j->scene = scene; j->D = D; j->p = p; j->n = n; j->W = W;
    j->nknots = n + p + 1; j->sigma = a->sigma; j->seed = a->seed; j->max_batch = max_batch;
    j->arc_all = a->arc_all ? 1 : 0;
    j->h_knots.assign(a->knots, a->knots + j->nknots);
    j->nm = scene ? (int)scene->movers.size() : 1;
    if (j->nm < 1) j->nm = 1;
    j->lpc = lanes_for(W - 1);
    j->cpb = kBlock / j->lpc;
    // endpoints are candidate-independent when the knot vector is clamped (sampled mode)
    bool clamped = true;
    for (int i = 0; i <= p; ++i) clamped = clamped && a->knots[i] == a->knots[0] && a->knots[n + i] == a->knots[n + p];
    j->shared_endpoints = clamped ? 1 : 0;
    j->lds = sizeof(double) * ((size_t)j->cpb * n * D + kBlock / 64 + 4) + sizeof(int) * (j->cpb + 1);
    if (j->lds > 160 * 1024) { delete j; return sspp::set_error(SSPP_E_UNSUPPORTED, "problem too large for LDS"); }
    int rc;
    const int64_t nblk = (max_batch + j->cpb - 1) / j->cpb;
    std::vector<double> us;
    for (int i = 0; i <= W; ++i) us.push_back((double)i / W);            // collision grid
    for (int i = 0; i < W; ++i) us.push_back(W > 1 ? (double)i / (W - 1) : 0.0);  // arc-length grid
    if ((rc = upload(&j->d_knots, a->knots, (size_t)j->nknots)) ||
        (rc = upload_basis(us, p, a->knots, j->nknots, &j->d_tab, &j->d_span)) ||
        (rc = upload(&j->d_init, a->init_ctrl, (size_t)n * D)) ||
        (rc = upload(&j->d_limits, a->limits, (size_t)D))) {
        sspp_job_free(j);
        return rc;
    }
    j->npert = (n - 2 * p) * D;
    if (j->npert < 0) j->npert = 0;
    { const char* e = getenv("SSPP_KERNEL"); j->c2f = e ? atoi(e) != 0 : 1; }
    // default: c2f draws inside the scoring kernel (SSPP_INSAMPLE=0: chip-wide k_sample_sspp; measured slower)
    { const char* e = getenv("SSPP_INSAMPLE"); j->insample = e ? atoi(e) : (j->c2f ? 1 : 0); }
    { const char* e = getenv("SSPP_HULL"); j->hull = e ? atoi(e) : 2; }
    {
        // defaults measured on MI355X (robocrane, 32 steps/launch, 4 streams):
        // one-wave workgroups of 16 candidates x 4 phase-1 lanes — 1.84 G cand/s against 1.56 G
        // for 8 x 8 and 1.40 G for 256 x 8 (the kernel is VALU-issue bound: fewer lanes per
        // candidate waste fewer pair-loop iterations on lanes that have already hit)
        const char* e = getenv("SSPP_G1");
        int g1 = e ? atoi(e) : 4;
        if (g1 != 4 && g1 != 8 && g1 != 16 && g1 != 32 && g1 != 64) g1 = 8;
        const char* t = getenv("SSPP_NT");
        int nt = t ? atoi(t) : 64;
        if (nt != 64 && nt != 128 && nt != 256) nt = 64;
        j->g1 = g1;
        j->nt2 = nt;
        j->cpb2 = nt / g1;
        j->n1 = std::min(g1, W + 1);
        std::vector<int> ord = c2f_order(W);
        std::vector<double> uo;
        for (int i : ord) uo.push_back((double)i / W);
        if ((rc = upload_basis(uo, p, a->knots, j->nknots, &j->d_otab, &j->d_ospan))) {
            sspp_job_free(j);
            return rc;
        }
        if (scene && !scene->pairs.empty()) {
            const char* po = getenv("SSPP_PAIR_ORDER");  // 0 = scene order (profiling)
            std::vector<DPair> jp = (po && atoi(po) == 0)
                                        ? scene->pairs
                                        : pairs_for_job(scene, a->knots, j->nknots, p, a->init_ctrl, D);
            if ((rc = upload(&j->d_pairs, jp.data(), jp.size()))) {
                sspp_job_free(j);
                return rc;
            }
        }
        const int nm = j->nm < 1 ? 1 : j->nm;
        const int rbox = std::max(6 * nm, lanes_for(W - 1) / 64 + 1);  // k_sspp_c2f: s_box / s_vsum + s_arc
        j->lds2 = sizeof(double) * ((size_t)j->cpb2 * (n * D + rbox)) +
                  sizeof(unsigned long long) * j->cpb2 + sizeof(int) * (3 * j->cpb2 + 1);
        if (j->lds2 > 64 * 1024) j->c2f = 0;
    }
    if (j->npert > 0 && !j->insample && j->c2f) {  // room for kMaxSteps steps, capped at 256 MiB
        const size_t per_step = sizeof(double) * (size_t)max_batch * j->npert;
        j->pert_steps = (int)std::max<size_t>(1, std::min<size_t>(kMaxSteps, ((size_t)256 << 20) / per_step));
    }
    if (j->npert > 0 && hipMalloc((void**)&j->d_pert, sizeof(double) * (size_t)max_batch * j->npert * j->pert_steps) != hipSuccess) {
        sspp_job_free(j);
        return sspp::set_error(SSPP_E_NOMEM, "hipMalloc sampler buffer");
    }
    // one record per workgroup: at most max_batch workgroups per step whatever the layout
    // one record per workgroup and step: k_sspp has nblk workgroups per batch (one step per
    // launch), k_sspp_c2f ceil(max_batch / cpb2) per step and up to kMaxSteps steps per launch
    const int64_t nrec = std::max<int64_t>(nblk, ((max_batch + j->cpb2 - 1) / j->cpb2) * kMaxSteps);
    if (scene)
        for (const DPair& pr : scene->pairs) {
            const int t1 = scene->geoms[pr.gm].type, t2 = pr.otype;
            if ((t1 == 5 && t2 == 6) || (t1 == 6 && t2 == 5)) j->has_cb = 1;
        }
    if (hipMalloc((void**)&j->d_part, sizeof(BlockBest) * nrec) != hipSuccess ||
        hipMalloc((void**)&j->d_sync, sizeof(ArgminSync) * kMaxSteps) != hipSuccess ||
        hipMemset(j->d_sync, 0, sizeof(ArgminSync) * kMaxSteps) != hipSuccess ||
        hipMalloc((void**)&j->d_dfr, sizeof(unsigned) * 2) != hipSuccess ||
        hipMemset(j->d_dfr, 0, sizeof(unsigned) * 2) != hipSuccess) {
        sspp_job_free(j);
        return sspp::set_error(SSPP_E_NOMEM, "hipMalloc block partials");
    }
    *out = j;
    return SSPP_OK;
}

struct SsppPtrs {
    const double* ctrl_in;
    double* ctrl_out;
    double* arc;
    unsigned char* feasible;
    sspp_best* best;
};

template <int D, int NM, int P>
static hipError_t launch_sspp(const SsppK& k, const sspp_job* j, const SsppPtrs& o, int nblk,
                              hipStream_t st) {
    if (NM == 1 && k.sc.onegeom && k.sc.npairs > 0) {
        hipLaunchKernelGGL((k_sspp<D, 1, P, true>), dim3(nblk), dim3(kBlock), j->lds, st, k,
                           scene_t(j->scene), j->d_tab, j->d_span, j->d_init, j->d_limits, o.ctrl_in,
                           j->d_pert, o.ctrl_out, o.arc, o.feasible, j->d_part, j->d_sync, o.best);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((k_sspp<D, NM, P, false>), dim3(nblk), dim3(kBlock), j->lds, st, k,
                       scene_t(j->scene), j->d_tab, j->d_span, j->d_init, j->d_limits, o.ctrl_in,
                       j->d_pert, o.ctrl_out, o.arc, o.feasible, j->d_part, j->d_sync, o.best);
    return hipGetLastError();
}

static SceneT scene_t_job(const sspp_job* j) {
    SceneT t = scene_t(j->scene);
    if (j->d_pairs) t.pairs = j->d_pairs;
    return t;
}

// k_sspp_cbfix after the scoring launch, only when the job's pairs include cylinder-box ones
template <int D, int NM, int P, bool OG>
static hipError_t launch_cbfix(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk,
                               hipStream_t st) {
    if (!j->has_cb || !k.has_scene) return hipSuccess;
    hipLaunchKernelGGL((k_sspp_cbfix<D, NM, P, OG>), dim3(kFixBlocks), dim3(kFixThreads),
                       sizeof(double) * j->n * D, st, k, scene_t_job(j), nblk / k.nblk_step, j->d_otab,
                       j->d_ospan, j->d_init, j->d_limits, o.ctrl_in, j->d_pert, o.arc, o.feasible,
                       j->d_part, j->d_sync, o.best);
    return hipGetLastError();
}

template <int D, int NM, int P, int NT>
static hipError_t launch_c2f_nt(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk,
                                hipStream_t st) {
    const double* atab = j->d_tab + (size_t)(j->W + 1) * (P + 1);
    const int* aspan = j->d_span + (j->W + 1);
    if (NM == 1 && k.sc.onegeom && k.sc.npairs > 0) {
        hipLaunchKernelGGL((k_sspp_c2f<D, 1, P, true, NT>), dim3(nblk), dim3(NT), j->lds2, st, k,
                           scene_t_job(j), j->d_otab, j->d_ospan, atab, aspan, j->d_init, j->d_limits,
                           o.ctrl_in, j->d_pert, o.ctrl_out, o.arc, o.feasible, j->d_part, j->d_sync, o.best);
        const hipError_t e = hipGetLastError();
        return e != hipSuccess ? e : launch_cbfix<D, 1, P, true>(k, j, o, nblk, st);
    }
    hipLaunchKernelGGL((k_sspp_c2f<D, NM, P, false, NT>), dim3(nblk), dim3(NT), j->lds2, st, k,
                       scene_t_job(j), j->d_otab, j->d_ospan, atab, aspan, j->d_init, j->d_limits,
                       o.ctrl_in, j->d_pert, o.ctrl_out, o.arc, o.feasible, j->d_part, j->d_sync, o.best);
    const hipError_t e = hipGetLastError();
    return e != hipSuccess ? e : launch_cbfix<D, NM, P, false>(k, j, o, nblk, st);
}

template <int D, int NM, int P>
static hipError_t launch_c2f(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk,
                             hipStream_t st) {
    if (j->nt2 == 64) return launch_c2f_nt<D, NM, P, 64>(k, j, o, nblk, st);
#ifdef SSPP_DEV_ONLY  // variant builds for experiments: robocrane shape only (fast compile)
    return hipErrorInvalidValue;
#else
    if (j->nt2 == 128) return launch_c2f_nt<D, NM, P, 128>(k, j, o, nblk, st);
    return launch_c2f_nt<D, NM, P, 256>(k, j, o, nblk, st);
#endif
}

template <int P>
static hipError_t dispatch_c2f_p(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk,
                                 hipStream_t st) {
#ifdef SSPP_DEV_ONLY
    if (P == 3 && j->nm == 1 && j->D == 7) return launch_c2f<7, 1, P>(k, j, o, nblk, st);
    return hipErrorInvalidValue;
#else
    if (j->nm == 2) {
        if (j->D == 9) return launch_c2f<9, 2, P>(k, j, o, nblk, st);
        return hipErrorInvalidValue;
    }
    switch (j->D) {
        case 1: return launch_c2f<1, 1, P>(k, j, o, nblk, st);
        case 2: return launch_c2f<2, 1, P>(k, j, o, nblk, st);
        case 3: return launch_c2f<3, 1, P>(k, j, o, nblk, st);
        case 4: return launch_c2f<4, 1, P>(k, j, o, nblk, st);
        case 6: return launch_c2f<6, 1, P>(k, j, o, nblk, st);
        case 7: return launch_c2f<7, 1, P>(k, j, o, nblk, st);
        case 9: return launch_c2f<9, 1, P>(k, j, o, nblk, st);
    }
    return hipErrorInvalidValue;
#endif
}

template <int P>
static hipError_t dispatch_sspp_p(const SsppK& k, const sspp_job* j, const SsppPtrs& o, int nblk,
                                  hipStream_t st) {
#ifdef SSPP_DEV_ONLY
    return hipErrorInvalidValue;
#else
    if (j->nm == 2) {
        if (j->D == 9) return launch_sspp<9, 2, P>(k, j, o, nblk, st);
        return hipErrorInvalidValue;
    }
    switch (j->D) {
        case 1: return launch_sspp<1, 1, P>(k, j, o, nblk, st);
        case 2: return launch_sspp<2, 1, P>(k, j, o, nblk, st);
        case 3: return launch_sspp<3, 1, P>(k, j, o, nblk, st);
        case 4: return launch_sspp<4, 1, P>(k, j, o, nblk, st);
        case 6: return launch_sspp<6, 1, P>(k, j, o, nblk, st);
        case 7: return launch_sspp<7, 1, P>(k, j, o, nblk, st);
        case 9: return launch_sspp<9, 1, P>(k, j, o, nblk, st);
    }
    return hipErrorInvalidValue;
#endif
}

static int run_sspp(sspp_job* j, const double* d_ctrl, int64_t first_id, int64_t B, double* d_arc,
                    uint8_t* d_feasible, double* d_ctrl_out, sspp_best* d_best, void* stream,
                    int steps = 1, int64_t step_stride = 0) {
    sspp::clear_error();
    if (!j || j->kind != 0) return sspp::set_error(SSPP_E_INVAL, "not a SamplingPathPlanner job");
    if (B < 1 || B > j->max_batch) return sspp::set_error(SSPP_E_INVAL, "batch size out of range");
    if (!d_arc || !d_feasible) return sspp::set_error(SSPP_E_INVAL, "null output");
    SsppK k{};
    k.sc = kscene(j->scene, false);
    k.has_scene = j->scene != nullptr;
    k.p = j->p; k.n = j->n; k.W = j->W;
    k.sigma = j->sigma; k.seed = j->seed;
    k.first_id = first_id; k.B = B;
    k.lpc = j->lpc; k.cpb = j->cpb; k.shared_endpoints = (d_ctrl == nullptr) ? j->shared_endpoints : 0;
    static const int ablate = [] { const char* e = getenv("SSPP_ABLATE"); return e ? atoi(e) : 0; }();
    k.ablate = ablate;
    k.insample = j->insample;
    k.arc_all = j->arc_all;
    SsppPtrs o{d_ctrl, d_ctrl_out, d_arc, d_feasible, d_best};
    if (steps < 1 || steps > kMaxSteps || (steps > 1 && (!j->c2f || d_ctrl || (j->npert > 0 && !j->insample && steps > j->pert_steps))))
        return sspp::set_error(SSPP_E_INVAL, "steps per launch: 1..64 (coarse-to-fine kernel, sampled candidates)");
    const int cpb = j->c2f ? j->cpb2 : j->cpb;
    const int nblk = (int)((B + cpb - 1) / cpb);
    hipStream_t st = (hipStream_t)stream;
    if (!d_ctrl && j->npert > 0 && !j->insample) {  // sampleWithNoise over the whole chip
        const long long work = (long long)steps * B * (long long)((j->npert + 3) / 4);
        hipLaunchKernelGGL(k_sample_sspp, dim3((unsigned)((work + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           (unsigned long long)j->seed, (long long)first_id, (long long)step_stride,
                           (long long)B, steps, j->D, j->p, j->npert, j->sigma, j->d_init, j->d_limits,
                           j->d_pert);
        hipError_t es = hipGetLastError();
        if (es != hipSuccess) return hip_fail(es, "k_sample_sspp launch");
    }
    hipError_t e;
    if (j->c2f) {
        SsppC2F c{};
        c.sc = k.sc; c.has_scene = k.has_scene; c.ablate = k.ablate; c.insample = j->insample;
        c.p = j->p; c.n = j->n; c.W = j->W; c.sigma = j->sigma; c.seed = j->seed;
        c.first_id = first_id; c.B = B;
        c.g1 = j->g1; c.cpb = j->cpb2; c.npts = j->W + 1; c.n1 = j->n1;
        c.lpc = lanes_for(j->W - 1);
        c.nblk_step = nblk;
        c.step_stride = step_stride;
        c.arc_all = j->arc_all;
        c.hull = j->hull;
        c.dfr = j->d_dfr;
        e = j->p == 3 ? dispatch_c2f_p<3>(c, j, o, nblk * steps, st) : dispatch_c2f_p<2>(c, j, o, nblk * steps, st);
    } else {
        e = j->p == 3 ? dispatch_sspp_p<3>(k, j, o, nblk, st) : dispatch_sspp_p<2>(k, j, o, nblk, st);
    }
    if (e != hipSuccess) return hip_fail(e, "k_sspp launch");
    return SSPP_OK;
}

extern "C" int sspp_job_sample_score(sspp_job* j, int64_t first_id, int64_t B, double* d_arc,
                          uint8_t* d_feasible, double* d_ctrl_out, sspp_best* d_best, void* stream) {
    return run_sspp(j, nullptr, first_id, B, d_arc, d_feasible, d_ctrl_out, d_best, stream);
}

// Re-target a SamplingPathPlanner job to another plan() call with the same knots, dof and
// check_points (the drop-in planner caches one job per shape): the initial control points,
// sigma, limits and seed change; the per-job pair order is recomputed for the new mean path.
// Uploads are asynchronous on `stream` from job-owned host copies (valid until the next update).
extern "C" int sspp_job_update_sspp(sspp_job* j, const double* init_ctrl, double sigma,
                                    const double* limits, uint64_t seed, void* stream) {
    sspp::clear_error();
    if (!j || j->kind != 0 || !init_ctrl || !limits) return sspp::set_error(SSPP_E_INVAL, "sspp_job_update_sspp: bad argument");
    const size_t nd = (size_t)j->n * j->D;
    hipStream_t st = (hipStream_t)stream;
    j->h_stage.assign(init_ctrl, init_ctrl + nd);
    j->h_stage.insert(j->h_stage.end(), limits, limits + j->D);
    j->sigma = sigma;
    j->seed = seed;
    HIPCHK(hipMemcpyAsync(j->d_init, j->h_stage.data(), sizeof(double) * nd, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(j->d_limits, j->h_stage.data() + nd, sizeof(double) * j->D, hipMemcpyHostToDevice, st));
    if (j->d_pairs && j->scene && !j->h_knots.empty()) {
        const char* po = getenv("SSPP_PAIR_ORDER");
        j->h_pairs = (po && atoi(po) == 0) ? j->scene->pairs
                                           : pairs_for_job(j->scene, j->h_knots.data(), j->nknots, j->p, init_ctrl, j->D);
        HIPCHK(hipMemcpyAsync(j->d_pairs, j->h_pairs.data(), sizeof(DPair) * j->h_pairs.size(),
                              hipMemcpyHostToDevice, st));
    }
    return SSPP_OK;
}

extern "C" int sspp_job_score_ctrl(sspp_job* j, const double* d_ctrl, int64_t first_id, int64_t B,
                        double* d_arc, uint8_t* d_feasible, sspp_best* d_best, void* stream) {
    if (!d_ctrl) return sspp::set_error(SSPP_E_INVAL, "null control points");
    return run_sspp(j, d_ctrl, first_id, B, d_arc, d_feasible, nullptr, d_best, stream);
}

extern "C" int sspp_job_create_tsp(const sspp_scene* scene, const sspp_tsp_args* a, int64_t max_batch,
                        sspp_job** out) {
    sspp::clear_error();
    if (!scene || !a || !out || !a->start || !a->end || !a->lo || !a->hi)
        return sspp::set_error(SSPP_E_INVAL, "sspp_job_create_tsp: null argument");
    if (scene->mode != SSPP_MODE_BODY) return sspp::set_error(SSPP_E_INVAL, "scene must be bound to a body");
    const int K = a->n_vias, cp = a->check_points, n = K + 2;
    if (K < 0 || K > 60) return sspp::set_error(SSPP_E_INVAL, "n_vias out of range");
    if (K > 0 && (!a->mean || !a->sigma)) return sspp::set_error(SSPP_E_INVAL, "null mean/sigma");
    if (cp < 1 || cp > 1 << 20) return sspp::set_error(SSPP_E_INVAL, "check_points must be >= 1");
    if (max_batch < 1) return sspp::set_error(SSPP_E_INVAL, "max_batch must be >= 1");
    if (n < 3) return sspp::set_error(SSPP_E_INVAL, "degree-2 interpolation needs >= 3 points");
    auto* j = new sspp_job();
    j->kind = 1; j->scene = scene; j->D = 4; j->p = 2; j->n = n; j->K = K; j->cp = cp;
    j->nknots = n + 3; j->seed = a->seed; j->max_batch = max_batch; j->nm = 1;
    for (int i = 0; i < 4; ++i) { j->start[i] = a->start[i]; j->end[i] = a->end[i]; j->lo[i] = a->lo[i]; j->hi[i] = a->hi[i]; }
    j->z_min = a->z_min; j->w_col = a->w_collision;
    j->floor_z_min = a->floor_z_min; j->floor_margin = a->floor_margin; j->floor_scale = a->floor_scale;
    j->lpc = lanes_for(cp);
    j->cpb = kBlock / j->lpc;
    j->lds = sizeof(double) * ((size_t)2 * j->cpb * n * 4 + 3 * (kBlock / 64) + 4) + sizeof(int) * j->cpb;
    if (j->lds > 160 * 1024) { delete j; return sspp::set_error(SSPP_E_UNSUPPORTED, "problem too large for LDS"); }
    std::vector<double> u(n), knots(n + 3), Minv((size_t)n * n);
    for (int i = 0; i < n; ++i) u[i] = (double)i / (n - 1);
    if (sspp::collocation_inverse(u.data(), n, 2, knots.data(), Minv.data()) != 0) {
        delete j;
        return sspp::set_error(SSPP_E_INVAL, "singular collocation matrix");
    }
    std::vector<double> zero(4, 0.0);
    int rc;
    const int64_t nblk = (max_batch + j->cpb - 1) / j->cpb;
    std::vector<double> us;
    const double du = 1.0 / cp;
    for (int i = 0; i <= cp; ++i) us.push_back((double)i * du);  // eval_one_pass: s(i * du)
    if ((rc = upload(&j->d_knots, knots.data(), knots.size())) ||
        (rc = upload_basis(us, 2, knots.data(), (int)knots.size(), &j->d_tab, &j->d_span)) ||
        (rc = upload(&j->d_Minv, Minv.data(), Minv.size())) ||
        (rc = upload(&j->d_mean, K ? a->mean : zero.data(), K ? (size_t)K * 4 : 4)) ||
        (rc = upload(&j->d_sigma, K ? a->sigma : zero.data(), K ? (size_t)K * 4 : 4))) {
        sspp_job_free(j);
        return rc;
    }
    if (hipMalloc((void**)&j->d_part, sizeof(BlockBest) * nblk) != hipSuccess ||
        hipMalloc((void**)&j->d_sync, sizeof(ArgminSync)) != hipSuccess ||
        hipMemset(j->d_sync, 0, sizeof(ArgminSync)) != hipSuccess) {
        sspp_job_free(j);
        return sspp::set_error(SSPP_E_NOMEM, "hipMalloc block partials");
    }
    *out = j;
    return SSPP_OK;
}

static int run_tsp(sspp_job* j, const double* d_vias, int64_t first_id, int64_t B, double* d_L,
                   double* d_Cnf, double* d_Cwf, uint8_t* d_status, double* d_cost,
                   double* d_vias_out, sspp_best* d_best, void* stream,
                   const sspp::TspCesEval* ces = nullptr) {
    sspp::clear_error();
    if (!j || j->kind != 1) return sspp::set_error(SSPP_E_INVAL, "not a TaskSpacePlanner job");
    if (B < 1 || B > j->max_batch) return sspp::set_error(SSPP_E_INVAL, "batch size out of range");
    if (!d_L || !d_Cnf || !d_Cwf || !d_status || !d_cost)
        return sspp::set_error(SSPP_E_INVAL, "null output");
    TspK k{};
    k.sc = kscene(j->scene, true);
    k.n = j->n; k.K = j->K; k.cp = j->cp;
    for (int i = 0; i < 4; ++i) { k.start[i] = j->start[i]; k.end[i] = j->end[i]; k.lo[i] = j->lo[i]; k.hi[i] = j->hi[i]; }
    k.z_min = j->z_min; k.seed = j->seed; k.first_id = first_id; k.B = B;
    k.w_col = j->w_col; k.floor_z_min = j->floor_z_min; k.floor_margin = j->floor_margin;
    k.floor_scale = j->floor_scale;
    k.lpc = j->lpc; k.cpb = j->cpb;
    const double* mean = j->d_mean;
    const double* sigma = j->d_sigma;
    if (ces) {
        if (d_vias) return sspp::set_error(SSPP_E_INVAL, "CES slot mode samples its own via sets");
        k.ces = 1; k.fixed = ces->fixed; k.nfixed = ces->nfixed;
        k.slot0 = ces->slot0; k.samples = ces->samples;
        mean = ces->mean; sigma = ces->sigma;
        for (int i = 0; i < 4; ++i) { k.start[i] = ces->start[i]; k.end[i] = ces->end[i]; }
    }
    const int nblk = (int)((B + j->cpb - 1) / j->cpb);
    hipStream_t st = (hipStream_t)stream;
    const SceneT tt = scene_t(j->scene);
#define SSPP_LAUNCH_TSP(OG, CBV)                                                                   \
    hipLaunchKernelGGL((k_tsp<1, OG, CBV>), dim3(nblk), dim3(kBlock), j->lds, st, k, tt, j->d_tab, \
                       j->d_span, j->d_Minv, mean, sigma, d_vias, d_vias_out, d_L, d_Cnf, d_Cwf, d_cost, \
                       d_status, j->d_part, j->d_sync, d_best)
    const bool og = k.sc.onegeom && k.sc.npairs > 0;
    if (og && k.sc.cylbox) SSPP_LAUNCH_TSP(true, true);
    else if (og) SSPP_LAUNCH_TSP(true, false);
    else if (k.sc.cylbox) SSPP_LAUNCH_TSP(false, true);
    else SSPP_LAUNCH_TSP(false, false);
#undef SSPP_LAUNCH_TSP
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_tsp launch");
    return SSPP_OK;
}

// CES slot-mode evaluation (ces.hip, tsp::Planner::plan eval loop): slots [slot0, slot0 + n)
int sspp::tsp_eval_ces(sspp_job* j, const TspCesEval* e, int64_t n, double* d_L, double* d_Cnf,
                       double* d_Cwf, uint8_t* d_status, double* d_cost, double* d_vias_out,
                       void* stream) {
    if (!e || !e->fixed || !e->nfixed || !e->mean || !e->sigma || !d_vias_out)
        return sspp::set_error(SSPP_E_INVAL, "tsp_eval_ces: null argument");
    return run_tsp(j, nullptr, e->first_id, n, d_L, d_Cnf, d_Cwf, d_status, d_cost, d_vias_out,
                   nullptr, stream, e);
}

extern "C" int sspp_job_tsp_sample_score(sspp_job* j, int64_t first_id, int64_t B, double* d_L, double* d_Cnf,
                              double* d_Cwf, uint8_t* d_status, double* d_cost, double* d_vias_out,
                              sspp_best* d_best, void* stream) {
    return run_tsp(j, nullptr, first_id, B, d_L, d_Cnf, d_Cwf, d_status, d_cost, d_vias_out, d_best, stream);
}

extern "C" int sspp_job_tsp_score_vias(sspp_job* j, const double* d_vias, int64_t first_id, int64_t B,
                            double* d_L, double* d_Cnf, double* d_Cwf, uint8_t* d_status,
                            double* d_cost, sspp_best* d_best, void* stream) {
    if (!d_vias && j && j->K > 0) return sspp::set_error(SSPP_E_INVAL, "null via points");
    return run_tsp(j, d_vias ? d_vias : nullptr, first_id, B, d_L, d_Cnf, d_Cwf, d_status, d_cost,
                   nullptr, d_best, stream);
}

extern "C" int sspp_job_info(const sspp_job* j, int* lpc, int* cpb, int* threads, size_t* lds) {
    if (!j) return sspp::set_error(SSPP_E_INVAL, "null job");
    if (lpc) *lpc = j->lpc;
    if (cpb) *cpb = j->cpb;
    if (threads) *threads = kBlock;
    if (lds) *lds = j->lds;
    return SSPP_OK;
}

extern "C" void sspp_job_free(sspp_job* j) {
    if (!j) return;
    for (double* p : {j->d_knots, j->d_tab, j->d_init, j->d_limits, j->d_Minv, j->d_mean, j->d_sigma})
        if (p) (void)hipFree(p);
    if (j->d_span) (void)hipFree(j->d_span);
    if (j->d_otab) (void)hipFree(j->d_otab);
    if (j->d_pairs) (void)hipFree(j->d_pairs);
    if (j->d_ospan) (void)hipFree(j->d_ospan);
    if (j->d_part) (void)hipFree(j->d_part);
    if (j->d_pert) (void)hipFree(j->d_pert);
    if (j->d_sync) (void)hipFree(j->d_sync);
    if (j->d_dfr) (void)hipFree(j->d_dfr);
    delete j;
}

extern "C" int sspp_best_reduce_device(const sspp_best* d_parts, int n, sspp_best* d_out,
                                       void* stream) {
    sspp::clear_error();
    if (!d_parts || !d_out || n < 1) return sspp::set_error(SSPP_E_INVAL, "sspp_best_reduce_device: bad argument");
    static_assert(sizeof(BlockBest) == sizeof(sspp_best), "layout");
    hipLaunchKernelGGL(k_argmin, dim3(1), dim3(kArgminThreads), 0, (hipStream_t)stream,
                       reinterpret_cast<const BlockBest*>(d_parts), n, d_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_argmin launch");
    return SSPP_OK;
}

// ---------------------------------------------------------------- step enqueue (host executor)
// A planning loop issues one small batch after another (4096 candidates = a few microseconds
// of GPU work).  Steps are independent, so they are spread round robin over several HIP
// streams and overlap on the chip; the host side of a step is one kernel launch issued from
// this C++ loop (no per-step Python).  Measured on MI355X: hipGraph replays of the same steps
// ran 1.5-4x slower than this (graph kernel nodes did not overlap), so there is no graph path.
namespace {
__global__ __launch_bounds__(64) void k_argmin_steps(const BlockBest* __restrict__ parts, int R,
                                                     int G, sspp_best* out) {
    // block g: lexicographic (cost, id) reduction of parts[r * G + g], r < R (one wave)
    const int g = blockIdx.x;
    double bc = INFINITY;
    long long bi = -1, cnt = 0;
    for (int r = threadIdx.x; r < R; r += 64) {
        const BlockBest b = parts[(long long)r * G + g];
        cnt += b.count;
        if (better(b.cost, b.idx, bc, bi)) { bc = b.cost; bi = b.idx; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double oc = __shfl_xor(bc, off, 64);
        const long long oi = __shfl_xor(bi, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
        if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
    }
    if (threadIdx.x == 0) {
        out[g].cost = bi < 0 ? INFINITY : bc;
        out[g].index = bi;
        out[g].count = cnt;
        out[g].reserved = 0;
    }
}
}  // namespace

extern "C" int sspp_steps_enqueue_sspp(sspp_job* const* jobs, int nbranch, void* const* streams,
                                       int64_t B, int nsteps, int steps_per_launch, int64_t first_id,
                                       int64_t step_stride, double* const* d_arc,
                                       uint8_t* const* d_feasible, sspp_best* d_best) {
    sspp::clear_error();
    if (!jobs || !streams || !d_arc || !d_feasible || nbranch < 1 || nsteps < 0 || B < 1)
        return sspp::set_error(SSPP_E_INVAL, "sspp_steps_enqueue_sspp: bad argument");
    for (int b = 0; b < nbranch; ++b) {
        if (!jobs[b] || jobs[b]->kind != 0 || !d_arc[b] || !d_feasible[b])
            return sspp::set_error(SSPP_E_INVAL, "sspp_steps_enqueue_sspp: bad branch");
        for (int c = 0; c < b; ++c)
            if (jobs[c] == jobs[b]) return sspp::set_error(SSPP_E_INVAL, "branches need distinct jobs");
    }
    const int S = steps_per_launch;
    if (S < 1 || S > kMaxSteps) return sspp::set_error(SSPP_E_INVAL, "steps_per_launch must be in [1, 64]");
    for (int i = 0, l = 0; i < nsteps; i += S, ++l) {
        const int b = l % nbranch, s = std::min(S, nsteps - i);
        const int rc = run_sspp(jobs[b], nullptr, first_id + (int64_t)i * step_stride, B, d_arc[b],
                                d_feasible[b], nullptr, d_best ? d_best + i : nullptr, streams[b],
                                s, step_stride);
        if (rc != SSPP_OK) return rc;
    }
    return SSPP_OK;
}

extern "C" int sspp_best_reduce_steps(const sspp_best* d_parts, int R, int G, sspp_best* d_out,
                                      void* stream) {
    sspp::clear_error();
    if (!d_parts || !d_out || R < 1 || G < 1) return sspp::set_error(SSPP_E_INVAL, "sspp_best_reduce_steps: bad argument");
    hipLaunchKernelGGL(k_argmin_steps, dim3(G), dim3(64), 0, (hipStream_t)stream,
                       reinterpret_cast<const BlockBest*>(d_parts), R, G, d_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_argmin_steps launch");
    return SSPP_OK;
}

#ifdef SSPP_C2F_STATS
extern "C" int sspp_debug_c2f_stats(unsigned long long* out, int reset) {
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c2f_stats), sizeof(unsigned long long) * 16);
    if (reset) {
        unsigned long long z[16] = {0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_c2f_stats), z, sizeof z);
    }
    return 0;
}
#endif

#ifdef SSPP_WG_TIMING
extern "C" int sspp_debug_wg_times(unsigned long long* out, int n) {
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_t), sizeof(unsigned long long) * (size_t)n);
    return 0;
}
extern "C" int sspp_debug_wg_phases(unsigned long long* out, int n) {
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_ph), sizeof(unsigned long long) * (size_t)n);
    return 0;
}
#endif

extern "C" int sspp_device_count(int* n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (n) *n = (e == hipSuccess) ? c : 0;
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    return SSPP_OK;
}


