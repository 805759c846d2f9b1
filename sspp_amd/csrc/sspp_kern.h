// sspp_kern.h — the MI355X (gfx950) candidate-scoring kernels and their launch templates.
//
// Included by sspp_kernels.hip (host side: scenes, jobs, the C ABI) and by sspp_inst.hip,
// which the Makefile compiles once per dof (-DSSPK_D=1,2,3,4,6,7,9) and once for the
// TaskSpacePlanner kernels (-DSSPK_D=0), each explicitly instantiating its entry points, so the
// kernel instantiations compile in parallel.  Variant builds (tools/build_variant.sh, profiling
// and ablation only) define SSPP_SINGLE_TU and instantiate everything in sspp_kernels.hip.
//
// Hot path (reference include/sspp.h:194-225 and include/sspp/tsp_planner.h:95-138):
//   candidate sampling -> B-spline evaluation -> free-joint FK -> collision -> cost -> argmin.
//
//   * k_sspp_c2f (SamplingPathPlanner): a workgroup holds CPB candidates; control points in
//     LDS (Philox + Box-Muller in-kernel, or a coalesced copy of caller-supplied splines), a
//     coarse-to-fine waypoint order with G1 lanes per candidate first, then the survivors'
//     remaining waypoints over the whole workgroup;
//   * k_tsp / k_tsp_pp / k_tsp_pp2 (TaskSpacePlanner): one waypoint per lane, the scene's pairs
//     in a wave-uniform loop (scalar loads), deep-contact costs;
//   * per-candidate sums use the canonical order (lane partials, xor butterfly per wave,
//     waves in order) that oracle/sspp_oracle.c::or_canon_sum restates;
//   * one BlockBest per workgroup, reduced by the last workgroup to arrive (lowest id on ties).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "model.h"
// k_tsp forms (bit f = form f) that run several sub-batches per workgroup (SSPP_OPT_TSP_REP)
#ifndef SSPP_TSP_REP_FORMS
#define SSPP_TSP_REP_FORMS (1 << 3)
#endif
#ifdef SSPP_TSP_STATS  // profiling builds only: point_collide's pair work (tools/tsp_stats.py)
__device__ unsigned long long g_tsp_stats[16];
#define TSP_STAT(i, c) do { const unsigned long long m_ = __ballot(c), a_ = __ballot(1);                  \
        if (__lane_id() == __builtin_ctzll(a_) && m_) atomicAdd(&g_tsp_stats[i], (unsigned long long)__popcll(m_)); } while (0)
#else
#define TSP_STAT(i, c) do { } while (0)
#endif
#ifdef SSPP_C2F_STATS  // profiling builds only (tools/build_variant.sh stats -DSSPP_C2F_STATS)
__device__ unsigned long long g_c2f_stats[16];
#define SSPP_CB_STAT(i) atomicAdd(&g_c2f_stats[i], 1ull)
#endif
#ifdef SSPP_WG_TIMING  // profiling builds only: per-workgroup (start, end, CU, survivors) of k_sspp_c2f
__device__ unsigned long long g_wg_t[1 << 18];
__device__ unsigned long long g_wg_ph[8 << 16];  // per workgroup: shader clock after each phase
#define WG_PH(k) do { if (threadIdx.x == 0 && blockIdx.x < (1 << 16)) g_wg_ph[8 * blockIdx.x + (k)] = clock64(); } while (0)
__device__ unsigned long long g_p2_t[8 << 12];  // split launch: [4095] the last arriver's epilogue (start, end, grid)
__device__ unsigned long long g_p2_w[8 << 13];  // split launch per queue slot: start, end (wall), passes, FP64 passes, feasible, p2/p3 clocks, wave
#else
#define WG_PH(k) do { } while (0)
#endif
#include "sspp_device.h"
#include "sspp_filter.h"
#include "sspp_logtab.h"

using namespace sspd;

namespace sspk {

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
    int upright;        // tsp: every box-box pair is upright for a yaw-only mover (k_tsp<..., UP>)
    int cbup;           // tsp: every cylinder-box pair is vertical / upright (collide<..., CB = 2>)
};

// Scene tables are passed as separate __restrict__ kernel arguments: the pair loop is
// wave-uniform and the tables are provably not written by the kernel, so the compiler
// reads them with scalar (s_load) instructions into SGPRs, once per wave.
struct SceneT {
    const DGeom* __restrict__ geoms;
    const DPair* __restrict__ pairs;
    const DMover* __restrict__ movers;
    // the scene's pairs (<= 64) in an order grouped by moving geom, for the pair loops whose
    // order does not enter a sum (point_collide REC 4: per-pair records, summed in pair order
    // afterwards), so a geom's pose is formed once per group instead of at every geom change of
    // the reference's (g1, g2) order
    // (a copy of the pairs in that order, each record's `pad` holding its index in `pairs`)
    const DPair* __restrict__ visit;
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
    r.pad = p->pad;
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
// kHullPad (sspp_device.h) absorbs the rounding of the spline evaluation (|error| ~ 1e-15).

__host__ __device__ __forceinline__ bool pair_may_touch(const DPair& pr, const DGeom& G, const double* lo,
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
                                                        cmover_t movers,
                                                        const DPair* visit = nullptr) {
    const int lane = threadIdx.x & 63;
    bool act = false;
    if (lane < npairs) {  // bit v: the visit order's pair v (the identity without a visit order)
        const DPair pr = load_pair(visit ? (cpair_t)visit + lane : pairs + lane);
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
    // k_tsp_pp2 (several workgroups per candidate): per-candidate deep-pair records and
    // arrival counters
    unsigned* rec_nd;       // [B][64 waypoints][64 pairs]
    double* rec_term;       // [B][64][64]
    unsigned* arrive;       // [B], zero between launches (the last arriver re-arms it)
    int npg;                // workgroups per candidate
    int rep;                // k_tsp: sub-batches of cpb candidates per workgroup (tsp_rep)
};

// ---------------------------------------------------------------- Philox4x32-10 + Box-Muller
__device__ __forceinline__ void philox(unsigned c0, unsigned c1, unsigned c2, unsigned c3,
                                       unsigned k0, unsigned k1, unsigned o[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        // one 32 x 32 -> 64-bit multiply per product (v_mad_u64_u32): hi and lo together
        const unsigned long long p0 = (unsigned long long)c0 * 0xD2511F53u;
        const unsigned long long p1 = (unsigned long long)c2 * 0xCD9E8D57u;
        const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (unsigned)p1; c2 = n2; c3 = (unsigned)p0;
    }
    o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3;
}
__device__ __forceinline__ void philox_words(unsigned long long seed, unsigned long long g,
                                             unsigned idx, unsigned stream, unsigned o[4]) {
    philox(idx, stream, (unsigned)g, (unsigned)(g >> 32), (unsigned)seed, (unsigned)(seed >> 32), o);
}
// FP64 Box-Muller (the default sampler of both planners; std::normal_distribution<double> in the
// reference, include/sspp.h:116,125 and include/sspp/tsp_sampler.h:17): one Philox4x32-10 call
// gives two 53-bit uniforms u1 in (0, 1], u2 in [0, 1) -> z0 = r cos(2 pi u2), z1 = r sin(2 pi u2),
// r = sqrt(-2 ln u1), |z| <= 8.57.  ln and sincos are written out as FP64 polynomials with
// explicit fma (sin / cos: Taylor on |a| <= pi/4 to a^17 / a^16), an IEEE sqrt, and no division:
// ln u = e ln 2 + ln m with m = k/64 (1 + t), k = round(64 m) — a 64-entry table (sspp_logtab.h,
// tools/gen_log_table.py) holds r = RN(64/k) and -ln r as hi + lo, t = fma(m, r, -1) is one
// rounding with |t| <= 2^-7, and ln(1 + t) is its series to t^8 (remainder < 2e-20).  m near 2
// takes the next exponent's entry k = 64 (r = 1, t = m/2 - 1 exact), so ln u keeps its relative
// precision as u -> 1.  (Round 5 computed ln m by the atanh series of s = (m-1)/(m+1), an IEEE
// FP64 division: v_div_scale x2, v_rcp_f64, four fma, v_div_fmas / fixup per pair.)
// oracle/sspp_oracle.c::or_normal_pair reproduces every normal bit for bit.
__device__ __forceinline__ double bm_log64(double u) {  // ln u, u in [2^-53, 1]
    static const double tab[64][4] = {SSPP_LOGTAB_ENTRIES};
    const unsigned long long bits = (unsigned long long)__double_as_longlong(u);
    const unsigned long long mb = bits & 0x000fffffffffffffull;
    int e = (int)(bits >> 52) - 1023;
    int k = (int)((mb + (1ull << 45)) >> 46);  // round(64 m) - 64, 0..64
    double m = __longlong_as_double((long long)(mb | 0x3ff0000000000000ull));
    if (k == 64) { k = 0; e += 1; m = m * 0.5; }  // m in [2 - 2^-7, 2): its half, next to 1
    const double t = fma(m, tab[k][0], -1.0);     // m r - 1
    const double t2 = t * t;
    double p = -0.125;                             // -1/8
    p = fma(t, p, 0x1.2492492492492p-3);           // 1/7
    p = fma(t, p, -0x1.5555555555555p-3);          // -1/6
    p = fma(t, p, 0x1.999999999999ap-3);           // 1/5
    p = fma(t, p, -0.25);                          // -1/4
    p = fma(t, p, 0x1.5555555555555p-2);           // 1/3
    p = fma(t, p, -0.5);                           // -1/2
    const double l1 = fma(t2, p, t);               // ln(1 + t)
    const double de = (double)e;                   // ln 2 = hi + lo (hi: 42 bits, e hi exact)
    const double hi = fma(de, 0x1.62e42fefa3800p-1, tab[k][1]);
    const double lo = fma(de, 0x1.ef35793c76730p-45, tab[k][2]) + l1;
    return hi + lo;
}
__device__ __forceinline__ void bm_sincos2pi64(double u, double* sn, double* cs) {  // u in [0, 1)
    const double q = rint(4.0 * u);
    const double r = fma(-0.25, q, u);         // exact, |r| <= 1/8
    const double a = r * 0x1.921fb54442d18p+2; // 2 pi r, |a| <= pi/4
    const double a2 = a * a;
    double sp = 0x1.952c77030ad4ap-49;         // 1/17!
    sp = fma(a2, sp, -0x1.ae7f3e733b81fp-41);
    sp = fma(a2, sp, 0x1.6124613a86d09p-33);
    sp = fma(a2, sp, -0x1.ae64567f544e4p-26);
    sp = fma(a2, sp, 0x1.71de3a556c734p-19);
    sp = fma(a2, sp, -0x1.a01a01a01a01ap-13);
    sp = fma(a2, sp, 0x1.1111111111111p-7);
    sp = fma(a2, sp, -0x1.5555555555555p-3);   // -1/3!
    const double sa = fma(a * a2, sp, a);
    double cp = 0x1.ae7f3e733b81fp-45;         // 1/16! (the a^18 term: < 2.1e-18 on |a| <= pi/4)
    cp = fma(a2, cp, -0x1.93974a8c07c9dp-37);
    cp = fma(a2, cp, 0x1.1eed8eff8d898p-29);
    cp = fma(a2, cp, -0x1.27e4fb7789f5cp-22);
    cp = fma(a2, cp, 0x1.a01a01a01a01ap-16);
    cp = fma(a2, cp, -0x1.6c16c16c16c17p-10);
    cp = fma(a2, cp, 0x1.5555555555555p-5);
    cp = fma(a2, cp, -0x1.0000000000000p-1);   // -1/2!
    const double ca = fma(a2, cp, 1.0);
    const int qi = (int)q & 3;
    *sn = qi == 0 ? sa : (qi == 1 ? ca : (qi == 2 ? -sa : -ca));
    *cs = qi == 0 ? ca : (qi == 1 ? -sa : (qi == 2 ? -ca : sa));
}
__device__ __forceinline__ void normal_pair(unsigned long long seed, unsigned long long g,
                                            unsigned idx, unsigned stream, double* z0, double* z1) {
    unsigned o[4];
    philox_words(seed, g, idx, stream, o);
    const unsigned long long a = ((((unsigned long long)o[0]) << 32) | o[1]) >> 11;
    const unsigned long long b = ((((unsigned long long)o[2]) << 32) | o[3]) >> 11;
    const double u1 = (double)(a + 1) * 0x1p-53;  // (0, 1], exact
    const double u2 = (double)b * 0x1p-53;        // [0, 1), exact
    const double r = sqrt(-2.0 * bm_log64(u1));
    double sn, cs;
    bm_sincos2pi64(u2, &sn, &cs);
    *z0 = r * cs;
    *z1 = r * sn;
}
// Opt-in FP32 SamplingPathPlanner normals (sspp_sspp_args::sampler = 1, the round-2 default): one
// Philox4x32-10 call gives four 24-bit uniforms -> two Box-Muller pairs in FP32, with fmaf
// polynomials written out (ln u by the atanh series on the mantissa, sin / cos of 2 pi u after an
// exact quarter-turn reduction) and a correctly rounded sqrtf, so
// oracle/sspp_oracle.c::or_normal_quad reproduces it bit for bit.  |z| <= 5.77 (u1 >= 2^-24):
// narrower than the reference's std::normal_distribution<double>, hence not the default.
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

// sampleWithNoise (include/sspp.h:114-130) in work items: item m of a candidate draws normals
// 2m, 2m+1 (sampler 0: FP64 pair, Philox idx m) or 4m .. 4m+3 (sampler 1: FP32 quad) and adds
// (sigma z) limits(d) to the initial spline's perturbed control-point block `base` (row-major
// (j - p) * D + d), writing the candidate's block c: c[k] = base[k] + (sigma z_k) limits[k % D].
__device__ __forceinline__ int sample_items(int sampler, int npert) {
    return sampler ? (npert + 3) >> 2 : (npert + 1) >> 1;
}
// c32 (optional): the FP32 copy of the same values (k_sspp_c2f's filtered scan)
__device__ __forceinline__ void sample_item_to(int sampler, unsigned long long seed, unsigned long long g,
                                               int m, int npert, int D, double sigma,
                                               const double* limits, const double* base, double* c,
                                               float* c32 = nullptr) {
    if (sampler == 0) {
        double z0, z1;
        normal_pair(seed, g, (unsigned)m, 0u, &z0, &z1);
        const int k = 2 * m;
        const double v0 = base[k] + (sigma * z0) * limits[k % D];
        c[k] = v0;
        if (c32) c32[k] = (float)v0;
        if (k + 1 < npert) {
            const double v1 = base[k + 1] + (sigma * z1) * limits[(k + 1) % D];
            c[k + 1] = v1;
            if (c32) c32[k + 1] = (float)v1;
        }
    } else {
        double z[4];
        normal_quad(seed, g, (unsigned)m, 0u, z);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int k = 4 * m + h;
            if (k < npert) {
                const double v = base[k] + (sigma * z[h]) * limits[k % D];
                c[k] = v;
                if (c32) c32[k] = (float)v;
            }
        }
    }
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

// the same from a basis row already in registers (prefetched ahead of its use)
template <int D, int P>
__device__ __forceinline__ void eval_pt_r(const double* ctrl, const double (&Nr)[P + 1], int span, double* q) {
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

// DEEP=false: checkCollision's ncon > 0 for one candidate.  Every active lane of the wave
//   must belong to that candidate: the scan stops for the whole wave at the first pair where
//   any lane finds a contact (returns 1 on every lane — the candidate is infeasible whatever
//   the other waypoints give), or when *stop (the candidate's LDS flag, cleared by another
//   wave of the same candidate) reads 0.  Returns 0 when no lane has a contact.
// DEEP=true : returns 0, *cost = sum over deep contacts of -1/(center_dist + 1e-4) + static.
// REC (DEEP only, pairs k < 64): instead of summing, record each deep pair's contact count and
// cost term — rec_nd[k] = nd, rec_term[k] = -1/(centre distance + 1e-4) — so that pairs split
// over several lanes can be summed afterwards in pair order, bit-identical to the sum.  REC 1:
// rec_nd is unsigned char (LDS, k_tsp_pp); REC 2: rec_nd is unsigned and both are written with
// write-through agent-scope stores (another workgroup reads them, k_tsp_pp2).
// REC 3 (DEEP, MODE 1, NM 1; k_tsp<..., DEF>): every pair k < npairs gets a record — rec_nd[k]
// = its deep-contact count, or kBbPend + fi for a deep box-box pair whose contact polygon (face fi)
// is counted later by the workgroup over its compacted deferred pairs (bb_clip_count(_up)) —
// and rec_term[k] its cost term; rec_pose receives the mover pose (position, the five non-zero
// entries of the yaw rotation) those later counts recompute the geom poses from.
// REC 4 (k_tsp<..., DEF 2>): the records of REC 3 without the terms — the lane itself sums its
// records after the pair loop (tsp_lane_sum), recomputing each term from the recorded pose.
constexpr int kBbPend = 16;
#ifndef SSPP_TSP_LEAN_GEOM
#ifdef SSPP_TSP_STATS  // (the statistics read the geom record at every pair)
#define SSPP_TSP_LEAN_GEOM 0
#else
#define SSPP_TSP_LEAN_GEOM 1
#endif
#endif
template <int D, int NM, int MODE, bool DEEP, bool ONEGEOM, int CB = 1, int REC = 0, bool UP = false>
__device__ int point_collide(const double* q, const KScene& sc, const SceneT& T,
                             unsigned long long mask, double* cost, int* stop = nullptr,
                             void* rec_nd = nullptr, double* rec_term = nullptr, double* rec_pose = nullptr) {
    static_assert(REC < 3 || (DEEP && MODE == 1 && NM == 1), "deferred box-box polygons: yaw-only single mover");
    constexpr bool RECD = REC == 3 || REC == 4;  // records with deferred box-box polygons
    static_assert(!ONEGEOM || NM == 1, "single moving geom implies a single mover");
    const cgeom_t geoms = (cgeom_t)T.geoms;
    const cpair_t pairs = (cpair_t)T.pairs;
    double mp[NM][3], mR[NM][9];
    mover_poses<D, NM, MODE>(q, (cmover_t)T.movers, mp, mR);
    if (RECD) {
        rec_pose[0] = mp[0][0]; rec_pose[1] = mp[0][1]; rec_pose[2] = mp[0][2];
        rec_pose[3] = mR[0][0]; rec_pose[4] = mR[0][1]; rec_pose[5] = mR[0][3]; rec_pose[6] = mR[0][4];
        rec_pose[7] = mR[0][8];
    }
    if (DEEP) TSP_STAT(6, true);  // waypoint lanes
    double acc = 0.0;
    int cur = -1;
    double gp[3], gmat[9];
    bool have_rot = true;  // multi-geom movers: a geom's rotation is formed at its first near pair
    DGeom G;
    // Several moving geoms: SSPP_TSP_LEAN_GEOM bit 0 keeps only the current geom's index, bounding
    // radius and position across the pair loop and re-loads its record (scalar loads) at each
    // near pair, instead of ~26 VGPRs of record held through every pair; bit 1 also re-forms its
    // rotation per near pair instead of caching it (measured slower: the default is bit 0 only)
    constexpr bool LREC = !ONEGEOM && (SSPP_TSP_LEAN_GEOM & 1) != 0;  // record re-loaded per near pair
    constexpr bool LROT = !ONEGEOM && (SSPP_TSP_LEAN_GEOM & 2) != 0;  // rotation re-formed per near pair
    double grb = 0.0;
    constexpr bool ZR = MODE == 1;  // yaw-only mover rotation
    if (ONEGEOM) {  // every pair shares one moving geom: pose once, mover pose dies here
        cur = pairs[0].gm;
        G = load_geom(geoms + cur);
        geom_pos_t<ZR>(mp[0], mR[0], G, gp);
        geom_rot_t<ZR>(mR[0], G, gmat);
    }
    const int np = sc.npairs;
    // REC 4 with a visit order: v runs over the geom-grouped order (the mask's bits are in that
    // order too), k is the pair's index for its record
    const bool VIS = REC == 4 && T.visit != nullptr;
    for (int v = 0; v < np; ++v) {
        if (v < 64) {
            // skip culled pairs with a scalar bit scan
            const unsigned long long rest = mask >> v;
            if (rest == 0ull) break;
            v += __builtin_ctzll(rest);
            if (v >= np) break;
        }
        const DPair pr = load_pair(VIS ? (cpair_t)T.visit + v : pairs + v);
        const int k = VIS ? pr.pad : v;  // the pair's record index
        if (!ONEGEOM && pr.gm != cur) {
            cur = pr.gm;
            if (LREC) {
                const DGeom Gn = load_geom(geoms + cur);
                grb = Gn.rbound;
                const bool second = NM > 1 && Gn.mover == 1;
                geom_pos_t<ZR>(second ? mp[NM - 1] : mp[0], second ? mR[NM - 1] : mR[0], Gn, gp);
            } else {
                G = load_geom(geoms + cur);
                const bool second = NM > 1 && G.mover == 1;
                geom_pos_t<ZR>(second ? mp[NM - 1] : mp[0], second ? mR[NM - 1] : mR[0], G, gp);
            }
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
        const bool near = pair_near(pr, LREC ? grb : G.rbound, gp, op, om);
        int nd = 0, nc = 0;
        if (DEEP) {
            TSP_STAT(0, true);
            TSP_STAT(1, near);
            TSP_STAT(2, near && G.type == 6 && pr.otype == 6);
            TSP_STAT(3, near && (G.type == 5 || pr.otype == 5));
            TSP_STAT(4, near && (G.type == 0 || pr.otype == 0));
        }
        if (near) {
            if (LREC) G = load_geom(geoms + cur);
            if (LROT || (!ONEGEOM && !have_rot)) {
                const bool second = NM > 1 && G.mover == 1;
                geom_rot_t<ZR>(second ? mR[NM - 1] : mR[0], G, gmat);
                have_rot = true;
            }
            const bool gfirst = (G.type < pr.otype) || (G.type == pr.otype && G.orig < pr.oorig);
            if (RECD && G.type == 6 && pr.otype == 6) {
                // box-box: the SAT decision now, the contact polygon later (collide's DEEP path
                // runs box_box_deep_count(_up) unconditionally: margin >= 0 > kDeep)
                const int c = gfirst ? (UP ? box_box_deep_class_up(gp, gmat, G.size, op, om, pr.osize)
                                           : box_box_deep_class(gp, gmat, G.size, op, om, pr.osize))
                                     : (UP ? box_box_deep_class_up(op, om, pr.osize, gp, gmat, G.size)
                                           : box_box_deep_class(op, om, pr.osize, gp, gmat, G.size));
                nd = c < 0 ? 0 : (c == 6 ? 1 : kBbPend + c);
            } else if (gfirst) {
                nc = collide<DEEP, CB, DEEP, false, UP>(G.type, gp, gmat, G.size, pr.otype, op, om, pr.osize, pr.margin, &nd);
            } else {
                nc = collide<DEEP, CB, DEEP, false, UP>(pr.otype, op, om, pr.osize, G.type, gp, gmat, G.size, pr.margin, &nd);
            }
        }
        if (DEEP) TSP_STAT(5, nd > 0);
        if (RECD) ((unsigned char*)rec_nd)[k] = (unsigned char)nd;
        if (!DEEP) {
            // the loop trip is wave-uniform, so every active lane reaches this vote
            if (__ballot(nc > 0) != 0ull) return 1;
            if (stop && __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
                return 1;
        } else if (REC != 4 && nd > 0) {
            const double dc[3] = {op[0] - gp[0], op[1] - gp[1], op[2] - gp[2]};
            const double cd = sqrt(dot3(dc, dc));
            const double term = -1.0 / (cd + 1e-4);
            if (REC == 1) {
                ((unsigned char*)rec_nd)[k] = (unsigned char)nd;
                rec_term[k] = term;
            } else if (REC == 3) {
                rec_term[k] = term;
            } else if (REC == 2) {
                __hip_atomic_store((unsigned*)rec_nd + k, (unsigned)nd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned long long*)rec_term + k, (unsigned long long)__double_as_longlong(term),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                for (int i = 0; i < nd; ++i) acc = acc + term;
            }
        }
    }
    if (DEEP && REC == 0) *cost = acc + sc.static_cost;
    return 0;
}

// A deep box-box pair's contact polygon (bb_clip_count(_up), reference face fi) for the moving geom
// G at the mover pose `ps` (position, the five non-zero entries of the yaw rotation: REC 3/4's
// record) against the static partner of pair pr; the operand order of collide's box-box call.
template <bool UP>
__device__ __forceinline__ int tsp_clip(const double* ps, const DGeom& G, const DPair& pr, int fi) {
    const double mp0[3] = {ps[0], ps[1], ps[2]};
    const double mR0[9] = {ps[3], ps[4], 0.0, ps[5], ps[6], 0.0, 0.0, 0.0, ps[7]};
    double gp[3], gm[9];
    geom_pos_t<true>(mp0, mR0, G, gp);
    geom_rot_t<true>(mR0, G, gm);
    const bool gfirst = G.orig < pr.oorig;  // both boxes
    return gfirst ? (UP ? bb_clip_count_up(gp, gm, G.size, pr.opos, pr.omat, pr.osize, fi)
                        : bb_clip_count(gp, gm, G.size, pr.opos, pr.omat, pr.osize, fi))
                  : (UP ? bb_clip_count_up(pr.opos, pr.omat, pr.osize, gp, gm, G.size, fi)
                        : bb_clip_count(pr.opos, pr.omat, pr.osize, gp, gm, G.size, fi));
}

// REC 4's sum, after the pair loop: the lane's records in pair order, each deep pair adding
// its term -1/(centre distance + 1e-4) nd times — point_collide's additions in its order, so the
// cost is bit-identical — with a deferred polygon counted here (tsp_clip), where the pair loop's
// state is dead: the polygon's registers no longer add to the loop's.  The trip over the pairs is
// wave-uniform; a pair no lane of the wave recorded costs one ballot.
template <bool UP>
__device__ __forceinline__ double tsp_lane_sum(bool has, const unsigned char* rn, const double* ps, int np,
                                               const KScene& sc, const SceneT& T) {
    const cgeom_t geoms = (cgeom_t)T.geoms;
    const cpair_t pairs = (cpair_t)T.pairs;
    double acc = 0.0;
    for (int k = 0; k < np; ++k) {
        const int nd0 = has ? rn[k] : 0;
        if (__ballot(nd0 != 0) == 0ull) continue;
        const DPair pr = load_pair(pairs + k);
        const DGeom G = load_geom(geoms + pr.gm);
        if (nd0 != 0) {
            const int nd = nd0 >= kBbPend ? tsp_clip<UP>(ps, G, pr, nd0 - kBbPend) : nd0;
            const double mp0[3] = {ps[0], ps[1], ps[2]};
            const double mR0[9] = {ps[3], ps[4], 0.0, ps[5], ps[6], 0.0, 0.0, 0.0, ps[7]};
            double gp[3];
            geom_pos_t<true>(mp0, mR0, G, gp);
            const double dc[3] = {pr.opos[0] - gp[0], pr.opos[1] - gp[1], pr.opos[2] - gp[2]};
            const double term = -1.0 / (sqrt(dot3(dc, dc)) + 1e-4);
            for (int r = 0; r < nd; ++r) acc = acc + term;
        }
    }
    return acc + sc.static_cost;
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
// (inline, bb by value: an out-of-line call took bb's address, so every lane of every workgroup
// wrote the 32-byte record to scratch first — 64 B per lane of private segment for the
// robocrane kernels and a third of their HBM writes)
template <int NT = kBlock>
__device__ __forceinline__ void finish_batch(const BlockBest bb, BlockBest* __restrict__ part, ArgminSync* sync,
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


// ================================================================ coarse-to-fine feasibility
// k_sspp_c2f: SamplingPathPlanner scoring (include/sspp.h:194-225), workgroup = NT threads in
// waves of CPW = 64 / G1 candidates (G1 phase-1 lanes per candidate; lanes past CPW * G1 idle).
//
// checkCollision (include/sspp.h:132-150) stops at the first waypoint in contact, so the result
// is an OR over waypoints and pairs; the order in which they are examined cannot change it.
// An infeasible candidate is typically in contact over a long stretch of its path (robocrane,
// config 2: ~55 of 129 waypoints), so a handful of well-chosen waypoints finds almost all of
// them.  The host orders the W+1 collision waypoints (ord table: the job's hit order, then
// breadth-first interval bisection); then per workgroup:
//   prologue the initial spline once per workgroup in LDS (the control points sampleWithNoise
//            leaves alone, include/sspp.h:118-129: rows outside [p, n-p)), each candidate's
//            perturbed rows [p, n-p) drawn in-kernel (Philox4x32-10 + Box-Muller);
//   phase 1  G1 lanes per candidate test the first n1 <= G1 waypoints of that order; a
//            candidate's lanes leave the pair loop together at the first pair any of them
//            touches (ballot over the candidate's lane group);
//   phase 2  the survivors (few: the feasible ones plus the rare misses) are compacted in LDS
//            and their remaining waypoints spread over all NT lanes in rounds; a contact clears
//            the candidate's LDS flag and the next round drops the candidate;
//   settle   cylinder-box pairs the scans left undecided (collide<..., DEFER>) get the exact
//            test, out of line, for the (rare) candidates that have no other contact;
//   phase 3  arc length of the collision-free candidates, in the canonical reduction order of
//            oracle/sspp_oracle.c::or_canon_sum;
//   phase 4  block argmin + the fused batch argmin (finish_batch).
//   split    (multi-step throughput launches) survivors go through the launch's survivor queue.
// ---------------------------------------------------------------- split launch: the survivor queue
// A split k_sspp_c2f launch (multi-step throughput launches) does not finish its
// phase-1 survivors in the workgroup that sampled them: each workgroup appends its survivors to
// a job-owned queue (rows written through to the coherent level, then a ready word per slot),
// writes the final outputs of the others, and then every workgroup of the launch pops survivors,
// one at a time, until the queue is empty (surv_finish: phase 2 in passes of NT waypoints, phase
// 3, the outputs).  A survivor therefore runs on whichever workgroup is free, in parallel with
// the others, instead of in sequence behind its workgroup's other survivors (the one-round tail
// of a 20-step launch).  The queue is sharded (workgroup b produces into and consumes from
// shard b % 64).  A workgroup pops with a ticket (one fetch-add on the shard's taken counter: a
// compare-and-swap pop serialises a shard's consumers on the atomic's round trip, 93 vs 61 us) and
// waits until its slot is reserved, or leaves once every producer of the shard has pushed and
// the ticket is past the final count.  No ticket is ever dropped: a ticket whose wait exceeds the
// launch's linger (SsppC2F::linger, 10 ms by default; SSPP_OPT_SPLIT_LINGER_US) is handed over
// to the launch's last workgroup (SurvPtrs::orphan), which finishes it after every producer has
// pushed.  So waiting cannot deadlock even when other kernels share the chip (a waiter blocks at
// most one workgroup slot for at most the linger), and the ready words of every reserved slot are
// re-armed by the last workgroup, whatever happened.  The last workgroup also counts the finished
// survivors against the reserved slots: a shortfall (lost work; never observed, and impossible
// unless the queue's storage is overrun) is written to every step record's `reserved` field, and
// every host consumer of a record refuses it (SSPP_E_INCOMPLETE).
// A reserved slot's producer is resident (it reserved the slot) and sets the ready word shortly.
// The ready word and the rows are agent-scope atomics ordered by s_waitcnt (SSPP_QUEUE_FENCES).
// Each step's argmin: a feasible survivor takes part in an agent-scope atomicMin on its arc's bits
// (non-negative doubles order like their bits) and the feasible count; one whose arc was not
// above the minimum it saw is listed; the last workgroup to finish (sharded arrival counters, as
// finish_batch) picks the lowest global id at each step's minimum from that list, writes the
// records and re-arms the queue for the next launch on the job's stream.
constexpr unsigned long long kLingerTicksDefault = 1000000;  // 10 ms of the 100 MHz wall clock
#ifdef SSPP_DEBUG_PROGRESS  // progress beacons of the split launch: plain stores into a [grid][8]
// buffer (device memory for timing; mapped host memory to watch a launch that does not finish)
#define SSPP_BEACON(B_PH, B_X, B_Y)                                                                              \
    do {                                                                                                        \
        if (q.beacon && threadIdx.x == 0) {                                                                     \
            q.beacon[8 * blockIdx.x + 1] = (unsigned)(B_X);                                                     \
            q.beacon[8 * blockIdx.x + 2] = (unsigned)(B_Y);                                                     \
            q.beacon[8 * blockIdx.x] = (unsigned)(B_PH);                                                        \
        }                                                                                                       \
    } while (0)
// wave 1's progress (thread 64) in the workgroup's fourth word
#define SSPP_BEACON1(B_PH)                                                                                      \
    do {                                                                                                        \
        if (q.beacon && threadIdx.x == 64) q.beacon[8 * blockIdx.x + 3] = (unsigned)(B_PH);                    \
    } while (0)
// the 100 MHz wall clock's low word at a workgroup event, word 4 + B_K of its record
#define SSPP_BEACON_T(B_K)                                                                                      \
    do {                                                                                                        \
        if (q.beacon && threadIdx.x == 0) q.beacon[8 * blockIdx.x + 4 + (B_K)] = (unsigned)wall_clock64();    \
    } while (0)
// the last workgroup's epilogue stages: word B_K after the grid's records
#define SSPP_BEACON_E(B_K)                                                                                      \
    do {                                                                                                        \
        if (q.beacon && threadIdx.x == 0) q.beacon[8 * gridDim.x + (B_K)] = (unsigned)wall_clock64();          \
    } while (0)
#else
#define SSPP_BEACON(B_PH, B_X, B_Y) do { } while (0)
#define SSPP_BEACON1(B_PH) do { } while (0)
#define SSPP_BEACON_T(B_K) do { } while (0)
#define SSPP_BEACON_E(B_K) do { } while (0)
#endif
// Ready-word ordering.  Every access to the queue's shared data (rows, ready words, counters)
// is an agent-scope atomic (global_load / global_store ... sc1: coherent across the XCDs, not
// held in a non-coherent cache level), and the protocol orders them with s_waitcnt: the producer
// waits for its row stores to complete (vmcnt(0), each thread, then the workgroup barrier)
// before it stores the ready word, and the consumer issues its row loads only after its load of
// the word has returned.  That is the hardware ordering of CDNA4 for sc1 accesses.  The C++
// release / acquire pair (SSPP_QUEUE_FENCES 1) compiles to buffer_wbl2 sc1 (write back this
// XCD's whole L2) before each word store and buffer_inv sc1 (invalidate it) after each word
// load: 49.4 -> 73.4 us per 20-step launch (profiles/r06d_*), for data that never passes
// through those caches.  It stays a build option (tools/runs, A/B); the default is the
// relaxed form.
#ifndef SSPP_QUEUE_FENCES
#define SSPP_QUEUE_FENCES 0
#endif
#if SSPP_QUEUE_FENCES
#define SSPP_QUEUE_RELEASE_ORDER __ATOMIC_RELEASE
#define SSPP_QUEUE_ACQUIRE() __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent")
#else
#define SSPP_QUEUE_RELEASE_ORDER __ATOMIC_RELAXED
#define SSPP_QUEUE_ACQUIRE() do { } while (0)
#endif
#ifndef SSPP_SPLIT_PRIO  // split launches: issue priority by phase (s_setprio; A/B: 0)
#define SSPP_SPLIT_PRIO 1
#endif
#ifndef SSPP_PRIO_ALL  // the same priorities in the unsplit instances (A/B)
#define SSPP_PRIO_ALL 0
#endif
#ifndef SSPP_SPLIT_PRIO_CONSUMER  // the priority of a wave past phase 1 (push, queued survivors)
#define SSPP_SPLIT_PRIO_CONSUMER 0
#endif
#ifndef SSPP_QUEUE_WAITERS  // tickets per shard that may wait for slots not reserved yet
#define SSPP_QUEUE_WAITERS 4
#endif
#ifndef SSPP_LINGER_SLEEP  // s_sleep between a waiting wave's polls (x 64 clocks)
#define SSPP_LINGER_SLEEP 16
#endif
constexpr int kSurvShards = 64;      // queue shards: workgroup b produces into and consumes from b % 64
struct SurvShard {
    unsigned count;                    // slots reserved by the shard's producers
    unsigned taken;                    // slots popped by its consumers
    unsigned pushed;                   // producers whose slots are all ready
    unsigned served;                   // its survivors finished (checked against count by the last workgroup;
                                       // one counter per shard: a single launch-wide counter took every
                                       // consumer through one contended atomic, 47 -> 75 us per 20-step launch)
    unsigned pad[28];                  // own 128-byte line
};
struct SurvQ {
    SurvShard shard[kSurvShards];
    unsigned nlist;                    // entries of the argmin list (SurvPtrs::res)
    unsigned lost;                     // survivors the launch could not finish (0; see above)
    unsigned norphan;                  // tickets handed over to the last workgroup (SurvPtrs::orphan)
    unsigned pad1;
    unsigned long long handoffs;       // tickets handed over, over the job's life (never re-armed)
    unsigned long long lost_total;     // lost survivors over the job's life (never re-armed)
    unsigned pad2[24];
    unsigned arrive_sh[8][32];         // arrival counters (8 shards, own cache lines)
    unsigned arrive_top[32];
    unsigned long long bestbits[kMaxSteps];  // per step: min arc of a feasible survivor (bits)
    unsigned count_feas[kMaxSteps];    // per step: feasible survivors
};
// a slot's ready word: bit 63 ready, bit 62 undecided cylinder-box pair, bits 32..39 the step of
// the launch, bits 0..31 the candidate within the step (0: not ready; re-armed by the last
// workgroup of the launch that used it)
__host__ __device__ inline unsigned long long surv_word(int step, long long lc, bool defer) {
    return (1ull << 63) | ((unsigned long long)defer << 62) | ((unsigned long long)(unsigned)step << 32) |
           (unsigned long long)(unsigned)lc;
}
struct SurvBest {                      // the argmin list: a feasible arc not above the minimum it saw
    unsigned long long bits, id, step, pad;
};
struct SurvPtrs {
    SurvQ* hdr;
    unsigned long long* rec;  // [cap] ready words
    double* ctrl;      // [cap][nrd]  the survivors' own control-point rows
    float* ctrl32;     // [cap][nrd]  their FP32 copies
    SurvBest* res;     // [cap]       the argmin list (SurvQ::nlist entries)
    unsigned* orphan;  // [cap]       handed-over tickets (global slots; one per workgroup at most)
#ifdef SSPP_DEBUG_PROGRESS
    unsigned* beacon;  // debugging builds: [grid][8] progress / timing words (SSPP_BEACON)
#endif
    long long cap;
    int shard_cap;     // slots per shard: shard s owns [s * shard_cap, (s + 1) * shard_cap)
};

struct SsppC2F {
    KScene sc;
    int has_scene;
    int sampler;   // 0 FP64 Box-Muller pairs (default), 1 FP32 quads (opt-in)
    int p, n, W;
    double sigma;
    unsigned long long seed;
    long long first_id, B;
    int g1, cpw, cpb;  // phase-1 lanes per candidate, candidates per wave (64 / g1) and workgroup
    int npts, n1;  // collision waypoints per candidate (W+1), phase-1 waypoints (<= g1)
    int lpc;       // canonical lanes of the arc-length sum (or_lanes_for(W-1))
    // several independent steps (batches) per launch: workgroup b belongs to step b / nblk_step;
    // step s scores ids first_id + s * step_stride + [0, B) into arc/feasible + s * B, its own
    // argmin records / counters (part + s * nblk_step, sync + s) and best[s]
    int nblk_step;
    long long step_stride;
    int arc_all;   // 0: arc length only for collision-free candidates (+inf otherwise)
    // control-point rows kept per candidate: [r0, r1) — sampled candidates [p, n-p) (the others
    // are the initial spline's, one shared copy per workgroup), caller splines [0, n)
    int r0, r1;
    int nt;        // launch shape (host side): threads per workgroup, dynamic LDS bytes
    int lds;
    int ctrl_feas; // ctrl_out rows only for candidates with no contact
    // FP32-filtered scan (sspp_filter.h): on when f32 != 0; feps = the certified margin (m),
    // fplim = the largest |mover root coordinate| it is certified for
    int f32;
    float feps, fplim;
    int split;     // the survivor queue (SurvQ) instead of phases 2-4 in the workgroup
    int nsteps;    // steps in this launch
    int drop_orphans;            // tests only (SSPP_OPT_SPLIT_DROP): the last workgroup drops the
                                 // handed-over tickets, which the lost-work check must report
    unsigned long long linger;   // wall-clock ticks a ticket waits before it is handed over
};

#ifdef SSPP_C2F_STATS
#define C2F_STAT(i, v) do { const unsigned long long v_ = (v); if ((threadIdx.x & 63) == 0 && v_) atomicAdd(&g_c2f_stats[i], v_); } while (0)
#else
#define C2F_STAT(i, v) do { } while (0)
#endif

// LDS offset (in doubles) of control-point row j of a candidate whose own rows [r0, r1) start at
// `mine`; the other rows are the workgroup's shared copy of the initial spline at `fix`.
__device__ __forceinline__ int crow(int mine, int fix, int r0, int r1, int j, int D) {
    return (j >= r0 && j < r1) ? mine + (j - r0) * D : fix + j * D;
}
// eval_pt on split rows: the same products and fma order, so bit-identical to eval_pt on the
// candidate's full control-point array
template <int D, int P>
__device__ __forceinline__ void eval_split(const double* sm, int mine, int fix, int r0, int r1,
                                           const double (&Nr)[P + 1], int span, double* q) {
    int o[P + 1];
#pragma unroll
    for (int r = 0; r <= P; ++r) o[r] = crow(mine, fix, r0, r1, span - P + r, D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        double acc = Nr[0] * sm[o[0] + d];
#pragma unroll
        for (int r = 1; r <= P; ++r) acc = fma(Nr[r], sm[o[r] + d], acc);
        q[d] = acc;
    }
}
template <int D, int P>
__device__ __forceinline__ void eval_split_g(const double* sm, int mine, int fix, int r0, int r1,
                                             const double* __restrict__ row, int span, double* q) {
    double Nr[P + 1];
#pragma unroll
    for (int r = 0; r <= P; ++r) Nr[r] = row[r];
    eval_split<D, P>(sm, mine, fix, r0, r1, Nr, span, q);
}

// Pair loop of one waypoint per lane.  All 64 lanes run the (wave-uniform) loop; `live` lanes
// test the pairs of their own mask.  gbits = the lanes of this lane's candidate within the
// wave: when any of them touches, all of them stop (returns true for the group).  flag: non-null
// in phase 2 (work counters only).  Lanes of the same survivor in another wave are not stopped
// inside a pass: polling the survivor's LDS flag at every pair measured slower (1128-1142 against
// 1143-1152 M cand/s on the 20-step run), and the next round drops the decided survivors anyway.
// A cylinder-box pair that passes the bounding-sphere test sets dfr (undecided) and counts as
// no contact here (collide<..., DEFER>); the settle step decides it with the exact test.
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
        bool nr = false;
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
            nr = pair_near(pr, G.rbound, gp, op, om);
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
        C2F_STAT(2, __popcll(__ballot(nr)));                // lanes past the sphere test (narrowphase)
        C2F_STAT(flag ? 10 : 9, __ballot(nr) != 0ull);      // wave iterations running a narrowphase
        C2F_STAT(flag ? 4 : 0, 1);                          // wave pair iterations (phase 2 / 1)
        C2F_STAT(flag ? 5 : 1, __popcll(__ballot(live && (k >= 64 || ((mymask >> k) & 1ull)))));
        if (__ballot(nc > 0) & gbits) { ghit = true; live = false; }
        if (__ballot(live) == 0ull) break;
    }
    return ghit;
}

// ---------------------------------------------------------------- FP32-filtered scan (sspp_filter.h)
// eval_split on the FP32 copies of the control points (LDS, written beside the doubles)
template <int D, int P>
__device__ __forceinline__ void eval_split32(const float* sm, int mine, int fix, int r0, int r1,
                                             const float (&Nr)[P + 1], int span, float* q) {
    int o[P + 1];
#pragma unroll
    for (int r = 0; r <= P; ++r) o[r] = crow(mine, fix, r0, r1, span - P + r, D);
#pragma unroll
    for (int d = 0; d < D; ++d) {
        float acc = Nr[0] * sm[o[0] + d];
#pragma unroll
        for (int r = 1; r <= P; ++r) acc = fmaf(Nr[r], sm[o[r] + d], acc);
        q[d] = acc;
    }
}

// mover_poses<D, NM, 0> in FP32: false when a quaternion is left to FP64 (sspf::quat_rot32) or
// a root position lies outside the range eps is certified for (|x| <= plim)
template <int D, int NM>
__device__ __forceinline__ bool mover_poses32(const float* q, cmover_t movers, float (&mp)[NM][3],
                                              float (&mR)[NM][9], float plim) {
    bool ok = true;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
        float qp[7];
#pragma unroll
        for (int k = 0; k < 7; ++k)
            qp[k] = (7 * m + k < D) ? q[(7 * m + k < D) ? 7 * m + k : 0] : (float)movers[m].qpos0[k];
        ok = ok && sspf::quat_rot32(qp + 3, mR[m]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            mp[m][k] = qp[k];
            ok = ok && fabsf(qp[k]) <= plim;
        }
    }
    return ok;
}

// scan_pairs in FP32 (same wave-uniform loop, masks and group semantics): returns true for the
// lanes of a group in which some lane has a CERTAIN contact; `amb` receives, per lane, the pairs
// (bits k < 64) the filter left to FP64.  A group with a certain contact needs no FP64 pass.
template <int D, int NM, bool ONEGEOM>
__device__ __forceinline__ bool scan_pairs32(const float* q, bool live, unsigned long long mymask,
                                             unsigned long long umask, unsigned long long gbits,
                                             const KScene& sc, const SceneT& T, float eps, float plim,
                                             unsigned long long& amb) {
    const cgeom_t geoms = (cgeom_t)T.geoms;
    const cpair_t pairs = (cpair_t)T.pairs;
    const int np = sc.npairs;
    amb = 0ull;
    float mp[NM][3], mR[NM][9];
    if (!mover_poses32<D, NM>(q, (cmover_t)T.movers, mp, mR, plim)) {
        if (live) amb = mymask & (np >= 64 ? ~0ull : ((1ull << np) - 1ull));
        live = false;
    }
    int cur = -1, gtype = 0, gmover = 0, grelrot = 0;
    float gp[3], gmat[9], gsize[3], grb = 0.0f;
    bool have_rot = true;
    // the moving geom's pose (geom_pose in FP32); its rotation only where a pair needs it
#define SSPF_LOAD_GEOM(IDX, P, R)                                                        \
    do {                                                                                 \
        const SSPP_CONST DGeom* g_ = geoms + (IDX);                                      \
        gtype = g_->type; gmover = g_->mover; grelrot = g_->relrot; grb = g_->frbound;   \
        gsize[0] = g_->fsize[0]; gsize[1] = g_->fsize[1]; gsize[2] = g_->fsize[2];       \
        const float pos_[3] = {g_->fpos[0], g_->fpos[1], g_->fpos[2]};                   \
        float t_[3];                                                                     \
        sspf::matvec3f((R), pos_, t_);                                                   \
        gp[0] = (P)[0] + t_[0]; gp[1] = (P)[1] + t_[1]; gp[2] = (P)[2] + t_[2];          \
    } while (0)
#define SSPF_GEOM_ROT(IDX, R)                                                            \
    do {                                                                                 \
        if (grelrot) {                                                                   \
            const SSPP_CONST DGeom* g_ = geoms + (IDX);                                  \
            float gm_[9];                                                                \
            for (int e_ = 0; e_ < 9; ++e_) gm_[e_] = g_->fmat[e_];                       \
            sspf::matmul3f((R), gm_, gmat);                                              \
        } else {                                                                         \
            for (int e_ = 0; e_ < 9; ++e_) gmat[e_] = (R)[e_];                           \
        }                                                                                \
    } while (0)
    if (ONEGEOM) {
        cur = pairs[0].gm;
        SSPF_LOAD_GEOM(cur, mp[0], mR[0]);
        SSPF_GEOM_ROT(cur, mR[0]);
    }
    bool ghit = false;
    const float pad = (float)kHullPad;
    for (int k = 0; k < np; ++k) {
        if (k < 64) {
            const unsigned long long rest = umask >> k;
            if (rest == 0ull) break;
            k += __builtin_ctzll(rest);
            if (k >= np) break;
        }
        const SSPP_CONST DPair* pr = pairs + k;
        if (!ONEGEOM && pr->gm != cur) {
            cur = pr->gm;
            const bool second = NM > 1 && geoms[cur].mover == 1;
            SSPF_LOAD_GEOM(cur, second ? mp[NM - 1] : mp[0], second ? mR[NM - 1] : mR[0]);
            have_rot = false;
        }
        int r = sspf::kNo;
        if (live && (k >= 64 || ((mymask >> k) & 1ull))) {
            float op[3], om[9], os[3];
            const int otype = pr->otype;
#pragma unroll
            for (int e = 0; e < 3; ++e) { op[e] = pr->fopos[e]; os[e] = pr->fosize[e]; }
#pragma unroll
            for (int e = 0; e < 9; ++e) om[e] = pr->fomat[e];
            if (NM > 1 && pr->omover >= 0) {
                const bool second = pr->omover == 1;
                const float* R = second ? mR[NM - 1] : mR[0];
                const float* P = second ? mp[NM - 1] : mp[0];
                float t[3], om2[9];
                sspf::matvec3f(R, op, t);
                op[0] = P[0] + t[0]; op[1] = P[1] + t[1]; op[2] = P[2] + t[2];
                sspf::matmul3f(R, om, om2);
#pragma unroll
                for (int e = 0; e < 9; ++e) om[e] = om2[e];
            }
            const float margin = pr->fmargin;
            const int nr = sspf::pair_near32(pr->forbound, otype, margin, os, grb, gp, op, om, eps, pad);
            if (nr != sspf::kNo) {
                if (!ONEGEOM && !have_rot) {
                    const bool second = NM > 1 && gmover == 1;
                    SSPF_GEOM_ROT(cur, second ? mR[NM - 1] : mR[0]);
                    have_rot = true;
                }
                const bool gfirst = (gtype < otype) || (gtype == otype && geoms[cur].orig < pr->oorig);
                r = gfirst ? sspf::collide32(gtype, gp, gmat, gsize, otype, op, om, os, margin, eps)
                           : sspf::collide32(otype, op, om, os, gtype, gp, gmat, gsize, margin, eps);
                if (r == sspf::kHit && nr == sspf::kAmb) r = sspf::kAmb;  // FP64 might cull it
                if (r == sspf::kAmb && k < 64) amb |= 1ull << k;
            }
        }
        C2F_STAT(13, 1);                                   // FP32 wave pair iterations
        C2F_STAT(3, __popcll(__ballot(r != sspf::kNo)));   // FP32 lanes past the culls
        if (__ballot(r == sspf::kHit) & gbits) { ghit = true; live = false; }
        if (__ballot(live) == 0ull) break;
    }
#undef SSPF_LOAD_GEOM
#undef SSPF_GEOM_ROT
    return ghit;
}

// sum of a per-lane count over the wave
__device__ __forceinline__ int wave_sum_u32(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
// OR of a per-lane 64-bit mask over the wave, in scalar registers (the FP64 pass's pair loop
// bound: only the pairs some lane left ambiguous)
__device__ __forceinline__ unsigned long long wave_or64(unsigned long long m) {
    unsigned lo = (unsigned)m, hi = (unsigned)(m >> 32);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        lo |= (unsigned)__shfl_xor((int)lo, off, 64);
        hi |= (unsigned)__shfl_xor((int)hi, off, 64);
    }
    return ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)hi) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((int)lo);
}

// ================================================================ hit census (job creation)
// The waypoint order of k_sspp_c2f's phase 1 is chosen from where sampled candidates of the
// job's own distribution touch the scene: one workgroup per census candidate draws it
// (sampleWithNoise, the job's sigma / limits, an independent seed) and tests every collision
// waypoint u = i / W, one per lane, against the sampled-candidate pair table (scan_pairs; a
// cylinder-box pair left undecided counts as no contact: the census only steers the order).
// Output: hit bits [M][ceil((W+1) / 64)], bit i = contact at waypoint i.
constexpr int kCensusThreads = 256;
template <int D, int NM, int P, bool ONEGEOM>
__global__ __launch_bounds__(kCensusThreads) void k_sspp_census(
    KScene sc, SceneT T, int n, int W, int sampler, double sigma, unsigned long long seed,
    const double* __restrict__ tab, const int* __restrict__ span, const double* __restrict__ init_ctrl,
    const double* __restrict__ limits, unsigned long long* __restrict__ hits) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int P1 = P + 1;
    const int tid = threadIdx.x, m = blockIdx.x, ndof = n * D, nw = (W + 64) >> 6;
    const int r0 = P < n ? P : n, r1 = n - P > r0 ? n - P : r0, nrd = (r1 - r0) * D;
    double* s_fix = smem;             // [n][D]
    double* s_own = s_fix + ndof;     // [r1 - r0][D]
    double* s_lim = s_own + nrd;      // [D]
    for (int e = tid; e < ndof; e += kCensusThreads) s_fix[e] = init_ctrl[e];
    if (tid < D) s_lim[tid] = limits[tid];
    for (int w = tid; w < nw; w += kCensusThreads) hits[(long long)m * nw + w] = 0ull;
    __syncthreads();
    for (int it = tid; it < sample_items(sampler, nrd); it += kCensusThreads)
        sample_item_to(sampler, seed, (unsigned long long)m, it, nrd, D, sigma, s_lim, s_fix + r0 * D, s_own);
    __syncthreads();
    for (int j0 = 0; j0 <= W; j0 += kCensusThreads) {  // workgroup-uniform
        const int j = j0 + tid;
        const bool live = j <= W;
        double q[D];
        eval_split_g<D, P>(smem, ndof, 0, r0, r1, tab + (live ? j : 0) * P1, span[live ? j : 0], q);
        bool dfr = false;
        const bool h = scan_pairs<D, NM, ONEGEOM>(q, live, ~0ull, ~0ull, 1ull << (tid & 63), nullptr, sc, T, dfr);
        if (h && live) atomicOr(hits + (long long)m * nw + (j >> 6), 1ull << (j & 63));
    }
}

#ifndef SSPP_CB_INLINE
#define SSPP_CB_INLINE __attribute__((noinline))
#endif
// The exact cylinder-box test (witnesses + candidate search, sspd::cyl_box_overlap) of one
// waypoint of one candidate over its cylinder-box pairs.  Out of line: it runs only for the
// candidates the scans left undecided, and its registers stay out of the kernel's pair loops.
template <int D, int NM, int P>
__device__ SSPP_CB_INLINE bool c2f_cb_exact(const double* sm, int mine, int fix, int r0, int r1,
                                                       const double* __restrict__ row, int span,
                                                       unsigned long long mask, int np, SceneT T) {
    double q[D];
    eval_split_g<D, P>(sm, mine, fix, r0, r1, row, span, q);
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

// A queued survivor's own rows (slot t) into LDS at o_own, doubles and their FP32 copies
template <int NT>
__device__ __forceinline__ void surv_load_rows(const SurvPtrs& q, unsigned t, int nrd, double* smem, float* s_f32,
                                               int o_own) {
    int e0 = threadIdx.x;
    asm volatile("" : "+v"(e0));  // (the LDS offsets per survivor, not held across the queue loop)
    for (int e = e0; e < nrd; e += NT) {
        const long long o = (long long)t * nrd + e;
        smem[o_own + e] = __longlong_as_double(
            (long long)__hip_atomic_load((unsigned long long*)q.ctrl + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        s_f32[o_own + e] =
            __uint_as_float(__hip_atomic_load((unsigned*)q.ctrl32 + o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
}

// One queued survivor, finished by the whole workgroup (the split launch's consumers, see SurvQ):
// phase 2 over waypoints j0 .. npts-1 of the job's order in passes of NT (a colliding survivor
// usually stops after its first pass; 124 remaining waypoints are one pass of the 128-thread
// shape), phase 3 in k_sspp_c2f's canonical order (each wave its 64-lane groups), the outputs and
// the step's argmin candidates.  Its rows are at o_own of smem / s_f32; s_ctl holds [feasible,
// defer], s_vsum the group sums.  Every thread calls it (it synchronises).
template <int D, int NM, int P, bool ONEGEOM, int NT>
__device__ __forceinline__ void surv_finish(const SsppC2F& a, const SceneT& TT, const double* __restrict__ otab,
                                            const float* __restrict__ otab32, const int* __restrict__ ospan,
                                            const double* __restrict__ atab, const int* __restrict__ aspan,
                                            const double* smem, const float* s_f32, int o_fix, int o_own, int* s_ctl,
                                            double* s_vsum, unsigned long long word, unsigned slot,
                                            double* __restrict__ arc, unsigned char* __restrict__ feasible,
                                            bool with_best, const SurvPtrs& q) {
    constexpr int P1 = P + 1;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // what derives from the lane index is recomputed here, not held
    const int lane = tid & 63, wv = tid >> 6;
    const int r0 = a.r0, r1 = a.r1, nch = a.W - 1;
    const int step = (int)((word >> 32) & 0xFFu), lc = (int)(unsigned)word;
    const int j0 = a.n1, R = a.npts - j0;
#ifdef SSPP_WG_TIMING
    const unsigned long long w_t0 = wall_clock64(), c0 = clock64();
    unsigned w_np = 0, w_nf = 0;
#endif
    SSPP_BEACON(20, slot, 0);
    for (int jb = 0; jb < R; jb += NT) {  // workgroup-uniform
        // a uniform exit once a pass has found a contact (every thread's read precedes the barrier)
        if (jb > 0 && !__syncthreads_or(__hip_atomic_load(s_ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
            break;
        const int jj = jb + tid;
        const bool live = jj < R;
        const int j = j0 + (live ? jj : 0);
        if (__ballot(live) == 0ull) continue;
        bool h;
        if (a.f32) {
            float q32[D], N32[P1];
#pragma unroll
            for (int r = 0; r < P1; ++r) N32[r] = otab32[j * P1 + r];
            eval_split32<D, P>(s_f32, o_own, o_fix, r0, r1, N32, ospan[j], q32);
            unsigned long long amb;
            h = scan_pairs32<D, NM, ONEGEOM>(q32, live, ~0ull, ~0ull, ~0ull, a.sc, TT, a.feps, a.fplim, amb);
            const bool need = live && !h && amb != 0ull;
            if (__ballot(need) != 0ull && __ballot(h) == 0ull) {  // one contact decides the survivor
#ifdef SSPP_WG_TIMING
                ++w_nf;
#endif
                double qd[D];
                bool dfr = false;
                eval_split_g<D, P>(smem, o_own, o_fix, r0, r1, otab + j * P1, ospan[j], qd);
                h = scan_pairs<D, NM, ONEGEOM>(qd, need, amb, wave_or64(need ? amb : 0ull), ~0ull, nullptr, a.sc,
                                               TT, dfr) || h;
            }
        } else {
            double qd[D];
            bool dfr = false;
            eval_split_g<D, P>(smem, o_own, o_fix, r0, r1, otab + j * P1, ospan[j], qd);
            h = scan_pairs<D, NM, ONEGEOM>(qd, live, ~0ull, ~0ull, ~0ull, nullptr, a.sc, TT, dfr);
        }
        if (__ballot(h) != 0ull && lane == 0) __hip_atomic_store(s_ctl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef SSPP_WG_TIMING
        ++w_np;
#endif
    }
    SSPP_BEACON(21, slot, 0);
    __syncthreads();
    const bool feas = __builtin_amdgcn_readfirstlane(s_ctl[0]) != 0;
    SSPP_BEACON(22, slot, feas);
#ifdef SSPP_WG_TIMING
    const unsigned long long c1 = clock64();
#endif
    double total = INFINITY;
    if (feas) {
        // phase 3: lane partials over lpc lanes, xor butterfly per 64-lane group, groups in order
        const int lpc = a.lpc, nvw = lpc >> 6;
        for (int vw = wv; vw < nvw; vw += NT / 64) {  // wave-uniform
            double acc = 0.0;
            for (int base = vw * 64; base < nch; base += lpc) {
                const int jc = base + lane, jj = jc < nch ? jc : nch - 1;
                double qa[D], qb[D];
                eval_split_g<D, P>(smem, o_own, o_fix, r0, r1, atab + (jj + 1) * P1, aspan[jj + 1], qb);
#pragma unroll
                for (int d = 0; d < D; ++d) qa[d] = __shfl_up(qb[d], 1, 64);
                if (lane == 0) eval_split_g<D, P>(smem, o_own, o_fix, r0, r1, atab + jj * P1, aspan[jj], qa);
                if (jc < nch) acc = acc + dist_nd<D>(qa, qb);
            }
            acc = wave_sum(acc);
            if (lane == 0) s_vsum[vw] = acc;
        }
        SSPP_BEACON(23, slot, 0);
        __syncthreads();
        total = s_vsum[0];
        for (int w = 1; w < nvw; ++w) total = total + s_vsum[w];
    }
    if (tid == 0) {
        const long long c = (long long)step * a.B + lc;
        arc[c] = total;
        feasible[c] = (unsigned char)feas;
        if (with_best) {
            if (feas && total < INFINITY) {
                const unsigned long long bits = (unsigned long long)__double_as_longlong(total);
                const unsigned long long seen =
                    __hip_atomic_fetch_min(q.hdr->bestbits + step, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (bits <= seen) {  // may be the step's minimum: listed for the last arriver
                    const unsigned k = __hip_atomic_fetch_add(&q.hdr->nlist, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&q.res[k].bits, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&q.res[k].id, (unsigned long long)(a.first_id + step * a.step_stride + lc),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&q.res[k].step, (unsigned long long)step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (feas) __hip_atomic_fetch_add(q.hdr->count_feas + step, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#ifdef SSPP_WG_TIMING
        unsigned long long* t = g_p2_w + 8 * (slot & ((8u << 10) - 1u));
        t[0] = w_t0; t[1] = wall_clock64(); t[2] = w_np; t[3] = w_nf; t[4] = feas;
        t[5] = c1 - c0; t[6] = clock64() - c1; t[7] = blockIdx.x;
#endif
    }
    (void)slot;
    SSPP_BEACON(24, slot, 0);
    __syncthreads();  // the next survivor may overwrite the rows and the flags
}

// Occupancy per shape: one- and two-wave workgroups of a single-geom mover at 5 waves per SIMD
// (96 VGPRs: 20 waves per CU, so the 20-step launch of 4096-candidate steps at 128 x 4 is one
// resident round); 4-wave workgroups and multi-geom movers at 4 (128 VGPRs; at 5 they spill).
// Round 6 (tools/kres.py, profiles/r06pmc_*): the robocrane d7 instances at 128 threads spill
// no VGPR, split and unsplit; the split one has no scratch at all (Registers).
#ifndef SSPP_C2F_WAVES_PER_EU
#define SSPP_C2F_WAVES_PER_EU 5
#endif
#ifndef SSPP_C2F_WAVES_PER_EU_WIDE
#define SSPP_C2F_WAVES_PER_EU_WIDE 4
#endif
// Workgroups of up to 128 threads run at SSPP_C2F_WAVES_PER_EU (96 VGPRs); the 256-thread
// latency shape carries the phase-2 pair groups (few survivor items over many lanes), which
// cost registers (at 5 waves per SIMD they spill), and runs at SSPP_C2F_WAVES_PER_EU_WIDE.
// profiling builds only (tools/build_variant.sh -DSSPP_ABLATE=mask): 1 no sampling, 2 no
// collision, 4 no arc, 8 no phase 2, 16 no phase 1, 64 return at entry (launch cost only)
#ifndef SSPP_ABLATE
#define SSPP_ABLATE 0
#endif
// CBX: the pair table has cylinder-box pairs, so the kernel carries the settle step (its
// out-of-line exact test costs the whole kernel registers: 96 -> 128 VGPRs and scratch)
// SPLIT: the split launch's instance (single-geom movers without cylinder-box pairs): phase 1,
// then the survivor queue; the in-workgroup phases 2-4 are unreachable there and compiled out, so
// the queue costs the unsplit instances no registers
template <int D, int NM, int P, bool ONEGEOM, int NT, bool CBX, bool SPLIT = false>
#ifndef SSPP_C2F_FIVE_MAX  // profiling builds: the largest workgroup at SSPP_C2F_WAVES_PER_EU
#define SSPP_C2F_FIVE_MAX 128
#endif
#ifndef SSPP_C2F_GP_NT     // profiling builds: the workgroup size that carries the pair groups
#define SSPP_C2F_GP_NT 256
#endif
__global__ __launch_bounds__(NT, (NT <= SSPP_C2F_FIVE_MAX && ONEGEOM) ? SSPP_C2F_WAVES_PER_EU : SSPP_C2F_WAVES_PER_EU_WIDE) void k_sspp_c2f(
    SsppC2F a, SceneT T, const double* __restrict__ otab, const float* __restrict__ otab32,
    const int* __restrict__ ospan,
    const double* __restrict__ atab, const int* __restrict__ aspan,
    const double* __restrict__ init_ctrl, const double* __restrict__ limits,
    const double* __restrict__ ctrl_in, double* __restrict__ ctrl_out, double* __restrict__ arc,
    unsigned char* __restrict__ feasible, BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best,
    SurvPtrs q) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int P1 = P + 1;
    constexpr int NB = 3 * NM;  // AABB extents per candidate (x, y, z per mover)
    constexpr int ABL = SSPP_ABLATE;
    const int tid = threadIdx.x, cpb = a.cpb, n = a.n, W = a.W, g1 = a.g1;
    const int ndof = n * D, nch = W - 1;
    const int r0 = a.r0, r1 = a.r1, nrd = (r1 - r0) * D;  // doubles kept per candidate
    const int step = blockIdx.x / a.nblk_step, blk = blockIdx.x - step * a.nblk_step;
    const long long cand0 = (long long)blk * cpb;
    const int nvalid = (int)min((long long)cpb, a.B - cand0);
    const long long first_id = a.first_id + step * a.step_stride;
    if (ABL & 64) return;
    if constexpr (SPLIT) SSPP_BEACON_T(0);
    // split launches: issue priority by phase — a wave still sampling goes before one in phase 1,
    // which goes before one finishing queued survivors.  The SIMD's arbiter otherwise favours the
    // oldest waves: at 5 waves per SIMD the first-dispatched waves finished phase 1 at ~12 us and
    // the last at ~25-36 us (profiles/r06c_beacons*), whose survivors then formed the launch's tail
    if constexpr ((SPLIT || SSPP_PRIO_ALL) && SSPP_SPLIT_PRIO) __builtin_amdgcn_s_setprio(2);
#ifdef SSPP_WG_TIMING
    const unsigned long long wg_t0 = wall_clock64();
    int wg_ns = -1;
#endif
    WG_PH(0);
    double* const arc_base = arc;  // the split launch's consumers write any step's outputs
    unsigned char* const feas_base = feasible;
    sspp_best* const best_base = best;
    if (step) {
        arc += step * a.B;
        feasible += step * a.B;
        if (ctrl_out) ctrl_out += step * a.B * ndof;
        part += step * a.nblk_step;
        sync += step;
        if (best) best += step;
    }
    // LDS (doubles): the shared initial spline [n][D], the candidates' own rows [cpb][r1-r0][D],
    // the limits [D], then the hull boxes (phase 2) — reused by phase 3's sums — and the flags
    const int o_fix = 0, o_own = ndof;
    double* s_lim = smem + o_own + cpb * nrd;                 // [D] sampleWithNoise limits
    const int nvw3 = a.lpc >> 6, rbox = 2 * NB > nvw3 + 1 ? 2 * NB : nvw3 + 1;
    double* s_box = s_lim + D;                                // [cpb][2][NB] (hull)
    double* s_vsum = s_box;                                   // [cpb][lpc/64] (phase 3)
    double* s_arc = s_box + cpb * nvw3;                       // [cpb] (phase 3, outputs)
    unsigned long long* s_mask = (unsigned long long*)(s_box + cpb * rbox);  // [cpb]
    int* s_feas = (int*)(s_mask + cpb);                       // [cpb]
    int* s_surv = s_feas + cpb;                               // [cpb + 1] (last = count)
    int* s_defer = s_surv + cpb + 1;                          // [cpb] undecided cylinder-box pair
    // FP32 copies of the control points (filtered scan), at the same offsets as the doubles
    float* s_f32 = (float*)(s_defer + cpb);                   // [ndof + cpb * nrd]

    // ---- per-lane layout: wave w holds candidates [w cpw, (w + 1) cpw), g1 lanes each
    const int wv = tid >> 6, ln = tid & 63;
    const int lg = ln / g1, l = ln - lg * g1;
    const bool in_grp = lg < a.cpw;
    const int g = wv * a.cpw + (in_grp ? lg : 0);
    const unsigned long long gbits = g1 >= 64 ? ~0ull : (((1ull << g1) - 1ull) << (lg * g1));

    // ---- prologue.  Every independent global read of the prologue and phase 1 (the initial
    // spline, the limits, this lane's phase-1 basis row) is issued here, so their L2 round trips
    // overlap instead of following one another.
    const int row_p1 = l < a.npts ? l : 0;
    const bool f32 = a.f32 != 0;
    // the filtered scan's row in FP32 (the FP64 passes read their row when they need it)
    float N32_p1[P1];
#pragma unroll
    for (int r = 0; r < P1; ++r) N32_p1[r] = otab32[row_p1 * P1 + r];
    const int span_p1 = ospan[row_p1];
    for (int rr = tid; rr < ndof; rr += NT) {
        const double v = init_ctrl[rr];
        smem[o_fix + rr] = v;
        if (f32) s_f32[o_fix + rr] = (float)v;
    }
    if (tid < D) s_lim[tid] = limits[tid];
    if (ctrl_in) {  // element e = sl * ndof + r walked with add-with-carry
        const int dsl = NT / ndof, dr = NT - dsl * ndof;
        int sl = tid / ndof, r = tid - sl * ndof;
        const double* src = ctrl_in + cand0 * ndof;
        for (; sl < nvalid; sl += dsl) {
            const double v = src[sl * ndof + r];
            smem[o_own + sl * ndof + r] = v;
            if (f32) s_f32[o_own + sl * ndof + r] = (float)v;
            r += dr;
            if (r >= ndof) { r -= ndof; ++sl; }
        }
    }
    __syncthreads();
    WG_PH(1);
    if (!ctrl_in && nrd > 0) {
        // sampleWithNoise: item t = (candidate sl, sampler item m), spread over the workgroup,
        // walked with add-with-carry (no integer division per item); each item writes
        // init + (sigma z) limits into the candidate's own rows (unsampled slots: the init rows)
        const int nq = sample_items(a.sampler, nrd);
        const double* base = smem + o_fix + r0 * D;
        const int dsl = NT / nq, dm = NT - dsl * nq;
        int sl = tid / nq, m = tid - sl * nq;
        for (int t = tid; t < nvalid * nq; t += NT) {
            double* dst = smem + o_own + sl * nrd;
            float* dst32 = f32 ? s_f32 + o_own + sl * nrd : nullptr;
            if (!(ABL & 1)) {
                sample_item_to(a.sampler, a.seed, (unsigned long long)(first_id + cand0 + sl), m, nrd, D, a.sigma,
                               s_lim, base, dst, dst32);
            } else {
                const int per = a.sampler ? 4 : 2;
                for (int h = 0; h < per; ++h) {
                    const int k = per * m + h;
                    if (k < nrd) { dst[k] = base[k]; if (dst32) dst32[k] = (float)base[k]; }
                }
            }
            sl += dsl;
            m += dm;
            if (m >= nq) { m -= nq; ++sl; }
        }
        __syncthreads();
    }
    WG_PH(2);
    if constexpr ((SPLIT || SSPP_PRIO_ALL) && SSPP_SPLIT_PRIO) __builtin_amdgcn_s_setprio(1);

    const SceneT TT = T;
    const bool collide_on = a.has_scene && !(ABL & 2);
    const int np = a.sc.npairs;
    // ---- phase 1: G1 lanes per candidate, first n1 waypoints of the coarse-to-fine order
    {
        const bool valid = in_grp && g < nvalid;
        bool ghit = false, dfr = false;
        if (collide_on) {
            const bool live = valid && l < a.n1 && !a.sc.static_block && !(ABL & 16);
            const int own = o_own + (valid ? g : 0) * nrd;
            if (f32) {
                // FP32 first; FP64 only for the pairs it leaves ambiguous, in groups with no
                // certain contact (sspp_filter.h)
                float q32[D];
                eval_split32<D, P>(s_f32, own, o_fix, r0, r1, N32_p1, span_p1, q32);
                unsigned long long amb;
                ghit = scan_pairs32<D, NM, ONEGEOM>(q32, live, ~0ull, ~0ull, gbits, a.sc, TT, a.feps, a.fplim, amb);
                const bool need = live && !ghit && amb != 0ull;
                C2F_STAT(11, __popcll(__ballot(need)));
                if (__ballot(need) != 0ull) {
                    double q[D];
                    eval_split_g<D, P>(smem, own, o_fix, r0, r1, otab + row_p1 * P1, span_p1, q);
                    ghit = scan_pairs<D, NM, ONEGEOM>(q, need, amb, wave_or64(need ? amb : 0ull), gbits, nullptr,
                                                      a.sc, TT, dfr) || ghit;
                }
            } else {
                double q[D];
                eval_split_g<D, P>(smem, own, o_fix, r0, r1, otab + row_p1 * P1, span_p1, q);
                ghit = scan_pairs<D, NM, ONEGEOM>(q, live, ~0ull, ~0ull, gbits, nullptr, a.sc, TT, dfr);
            }
        }
        const bool gdef = (__ballot(dfr) & gbits) != 0ull;
        if (in_grp && l == 0 && g < cpb) {
            s_feas[g] = valid && !ghit && !(collide_on && a.sc.static_block);
            s_defer[g] = gdef;
        }
    }
    __syncthreads();
    WG_PH(3);
    if constexpr ((SPLIT || SSPP_PRIO_ALL) && SSPP_SPLIT_PRIO) __builtin_amdgcn_s_setprio(SSPP_SPLIT_PRIO_CONSUMER);
    if constexpr (SPLIT) {
        static_assert(NM == 1 && ONEGEOM && !CBX, "split launches: single-geom movers without cylinder-box pairs");
        // the lane index through an empty asm: the split tail's LDS / output offsets are
        // recomputed from it instead of the prologue's being held (spilled) across phase 1
        int tid_s = threadIdx.x;
        asm volatile("" : "+v"(tid_s));
        const int tid = tid_s;
        SSPP_BEACON(3, 0, 0);
        SSPP_BEACON_T(1);
        // ---- producer: one queue reservation per workgroup (survivors in candidate order), the
        // survivors' rows written through to the coherent level, then each slot's ready word; the
        // other candidates' outputs are final here
        if (tid < 64) {
            const bool f = tid < nvalid && s_feas[tid] != 0;
            const unsigned long long m = __ballot(f);
            unsigned base = 0;
            if (tid == 0 && m)
                base = __hip_atomic_fetch_add(&q.hdr->shard[blockIdx.x % kSurvShards].count, (unsigned)__popcll(m),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            base = (unsigned)__shfl((int)base, 0, 64) + (unsigned)((blockIdx.x % kSurvShards) * q.shard_cap);
            if (tid < cpb) s_surv[tid] = f ? (int)(base + __popcll(m & ((1ull << tid) - 1ull))) : -1;
        }
        __syncthreads();
        for (int e = tid; e < nvalid * nrd; e += NT) {
            const int sl = e / nrd, r = e - sl * nrd, slot = s_surv[sl];
            if (slot >= 0) {
                const long long o = (long long)slot * nrd + r;
                __hip_atomic_store((unsigned long long*)q.ctrl + o,
                                   (unsigned long long)__double_as_longlong(smem[o_own + sl * nrd + r]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((unsigned*)q.ctrl32 + o, __float_as_uint(s_f32[o_own + sl * nrd + r]),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's row stores are done
        __syncthreads();                                   // ... and every other thread's
        if (tid < nvalid) {
            const int slot = s_surv[tid];
            if (slot >= 0) {
                __hip_atomic_store(q.rec + slot, surv_word(step, cand0 + tid, s_defer[tid] != 0), SSPP_QUEUE_RELEASE_ORDER,
                                   __HIP_MEMORY_SCOPE_AGENT);
            } else {
                arc[tid + cand0] = INFINITY;
                feasible[tid + cand0] = 0;
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ready words are stored
        __syncthreads();  // the rows in LDS are free: each wave finishes survivors in its own slot
        if (tid == 0)
            __hip_atomic_fetch_add(&q.hdr->shard[blockIdx.x % kSurvShards].pushed, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        SSPP_BEACON(4, __popcll(__ballot(tid < nvalid && s_surv[tid] >= 0)), __smid());
        SSPP_BEACON_T(2);
        // ---- consumers: every workgroup pops survivors until the queue is empty; the launch's last
        // workgroup to arrive then finishes the handed-over slots in the same loop (one copy of
        // surv_finish in the kernel: a second inlined copy for the hand-over list raised the
        // instance's SGPR spills 385 -> 539)
        const unsigned nb_all = gridDim.x, shs = blockIdx.x % kSurvShards;
        const unsigned nwg_s = (nb_all - shs + kSurvShards - 1) / kSurvShards;  // producers of the shard
        SurvShard* const sh = q.hdr->shard + shs;
        int* s_ctl = s_surv;      // [0] feasible, [1] slot, [2..3] the ready word
        int* s_last = s_surv + cpb;
        bool last = false;        // workgroup-uniform: the launch's last workgroup, on the hand-over list
        unsigned ko = 0, no = 0;  // (thread 0) position in the hand-over list, its length
        unsigned handed = 0;      // (thread 0) this workgroup handed a ticket over (it then leaves)
#ifdef SSPP_DEBUG_PROGRESS
        unsigned nfin = 0;        // (thread 0) survivors this workgroup finished (beacon word 3)
#endif
        for (;;) {  // workgroup-uniform (the slot and word come from LDS through readfirstlane)
            if (tid == 0) {
                unsigned t = ~0u;
                unsigned long long w = 0ull;
                if (!last) {
                    // a ticket: the shard's next slot in reservation order, reserved now or later —
                    // unless SSPP_QUEUE_WAITERS tickets already wait for slots not reserved yet:
                    // then this workgroup leaves (those waiters, and every producer after its
                    // push, serve the slots still to come; a waiter leaves once the shard is done)
                    const unsigned tk0 = __hip_atomic_load(&sh->taken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned ct0 = __hip_atomic_load(&sh->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((int)(tk0 - ct0) < SSPP_QUEUE_WAITERS) {
                        t = __hip_atomic_fetch_add(&sh->taken, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        SSPP_BEACON(5, t, ct0);
                        const unsigned long long w0 = wall_clock64();
                        for (;;) {
                            if (t < __hip_atomic_load(&sh->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
                            // every producer has pushed (its count is then final), the ticket past it
                            if (__hip_atomic_load(&sh->pushed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= nwg_s &&
                                __hip_atomic_load(&sh->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= t) {
                                t = ~0u;
                                break;
                            }
                            if (wall_clock64() - w0 >= a.linger) {
                                // handed over: the last workgroup finishes this slot (if it is
                                // ever reserved) once every producer has pushed
                                const unsigned k = __hip_atomic_fetch_add(&q.hdr->norphan, 1u, __ATOMIC_RELAXED,
                                                                          __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store(q.orphan + k, t + shs * (unsigned)q.shard_cap, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                                handed = 1;
                                t = ~0u;
                                break;
                            }
                            __builtin_amdgcn_s_sleep(SSPP_LINGER_SLEEP);
                        }
                    }
                    if (t != ~0u) {  // the producer is resident (it reserved the slot): its word lands shortly
                        t += shs * (unsigned)q.shard_cap;
                        SSPP_BEACON(6, t, 0);
                        const unsigned long long w1 = wall_clock64();
                        while ((w = __hip_atomic_load(q.rec + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0ull) {
                            if (wall_clock64() - w1 >= a.linger) break;  // bounded too: handed over
                            __builtin_amdgcn_s_sleep(1);
                        }
                        if (w == 0ull) {
                            const unsigned k = __hip_atomic_fetch_add(&q.hdr->norphan, 1u, __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(q.orphan + k, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            handed = 1;
                            t = ~0u;
                        } else {
                            SSPP_QUEUE_ACQUIRE();  // pairs with the producer's release
                            __hip_atomic_store(q.rec + t, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
                        }
                    }
                } else {
                    // the hand-over list: every producer has pushed (all workgroups arrived), so a
                    // reserved slot's word is set; a slot past its shard's final count was never
                    // reserved (SSPP_OPT_SPLIT_DROP, tests: every slot is dropped instead)
                    while (ko < no && w == 0ull) {
                        const unsigned slot = __hip_atomic_load(q.orphan + ko, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ++ko;
                        const unsigned sh_o = slot / (unsigned)q.shard_cap, lt = slot - sh_o * (unsigned)q.shard_cap;
                        if (!a.drop_orphans &&
                            lt < __hip_atomic_load(&q.hdr->shard[sh_o].count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                            w = __hip_atomic_load(q.rec + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (w != 0ull) {
                                SSPP_QUEUE_ACQUIRE();
                                __hip_atomic_store(q.rec + slot, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                t = slot;
                            }
                        }
                    }
                    SSPP_BEACON(11, ko, no);
                }
                s_ctl[0] = 1;
                s_ctl[1] = (int)t;
                s_ctl[2] = (int)(unsigned)(w >> 32);
                s_ctl[3] = (int)(unsigned)w;
            }
            __syncthreads();
            const unsigned t = (unsigned)__builtin_amdgcn_readfirstlane(s_ctl[1]);
            if (t == ~0u) {
                if (last) break;
#ifdef SSPP_WG_TIMING
                if (tid == 0 && blockIdx.x < (1 << 16)) {
                    g_wg_t[4 * blockIdx.x] = wg_t0;
                    g_wg_t[4 * blockIdx.x + 1] = wall_clock64();
                    g_wg_t[4 * blockIdx.x + 2] = __smid();
                    g_wg_t[4 * blockIdx.x + 3] = 0ull;
                }
#endif
                SSPP_BEACON(8, 0, 0);
                SSPP_BEACON_T(3);
                // ---- completion: sharded arrival; the last workgroup goes on with the hand-over list.
                // An arrival adds 1 + (handed over << 16), so the last arriver learns the list's
                // length from the counters' old values (no further round trip on its critical path)
                const unsigned nblk = gridDim.x;
                const int shd = blockIdx.x & 7, nsh = nblk < 8 ? (int)nblk : 8;
                if (tid == 0) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // outputs, list entries, hand-overs
                    const unsigned shard_n = (nblk - shd + 7) >> 3;
                    const unsigned prev = __hip_atomic_fetch_add(&q.hdr->arrive_sh[shd][0], 1u + (handed << 16),
                                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    int lst = 0;
                    if ((prev & 0xFFFFu) == shard_n - 1) {
                        const unsigned sho = (prev >> 16) + handed;  // the shard's hand-overs
                        const unsigned pt = __hip_atomic_fetch_add(&q.hdr->arrive_top[0], 1u + (sho << 16),
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        lst = (pt & 0xFFFFu) == (unsigned)nsh - 1;
                        if (lst) {
                            SSPP_QUEUE_ACQUIRE();
                            no = (pt >> 16) + sho;
                        }
                    }
                    s_last[0] = lst;
                    s_last[1] = (int)no;  // (s_last[1] is s_defer[0], which only the producers use)
                }
                __syncthreads();
                const int lst = __builtin_amdgcn_readfirstlane(s_last[0]);
                SSPP_BEACON(9 + lst, no, 0);
                if (lst) SSPP_BEACON_E(0);
                if (!lst) return;
                if (__builtin_amdgcn_readfirstlane(s_last[1]) == 0) break;  // nothing was handed over
                last = true;
                continue;
            }
            const unsigned long long w = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane(s_ctl[2]) << 32) |
                                         (unsigned)__builtin_amdgcn_readfirstlane(s_ctl[3]);
            SSPP_BEACON(7, t, (unsigned)w);
            surv_load_rows<NT>(q, t, nrd, smem, s_f32, o_own);
            __syncthreads();
            surv_finish<D, NM, P, ONEGEOM, NT>(a, TT, otab, otab32, ospan, atab, aspan, smem, s_f32, o_fix, o_own,
                                               s_ctl, s_vsum, w, t, arc_base, feas_base, best_base != nullptr, q);
            if (tid == 0)
                __hip_atomic_fetch_add(&q.hdr->shard[t / (unsigned)q.shard_cap].served, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
#ifdef SSPP_DEBUG_PROGRESS
            if (tid == 0 && q.beacon) q.beacon[8 * blockIdx.x + 3] = ++nfin;
#endif
        }
#ifdef SSPP_WG_TIMING
        const unsigned long long t_ep = wall_clock64();
#endif
        // the last workgroup: every handed-over slot is finished
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the outputs, list entries and counts
        __syncthreads();
        SSPP_BEACON(12, no, 0);
        SSPP_BEACON_E(1);
        // LDS is free: the per-step minimum bits, ids and feasible counts, the lost survivors
        int tid_e = threadIdx.x;
        asm volatile("" : "+v"(tid_e));  // (as at the producer: no offsets held across the queue)
        const int tid_ep = tid_e;
        unsigned long long* s_bits = (unsigned long long*)smem;
        unsigned long long* s_id = s_bits + kMaxSteps;
        unsigned* s_cnt = (unsigned*)(s_id + kMaxSteps);
        unsigned* s_lost = s_cnt + kMaxSteps;
        const int nsteps = a.nsteps;
        // one round trip for the header, the list's first NT entries (each thread reads entry tid
        // before it knows the list's length; entries past it are stale and unused) and, one shard
        // per thread, the reserved and the finished slots: the lost-work check
        const unsigned nl = __hip_atomic_load(&q.hdr->nlist, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned c_sh = 0, sv_sh = 0;
        if (tid_ep < kSurvShards) {
            c_sh = __hip_atomic_load(&q.hdr->shard[tid_ep].count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sv_sh = __hip_atomic_load(&q.hdr->shard[tid_ep].served, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        unsigned long long rb = 0ull, rid = 0ull, rst = 0ull;
        if (best_base) {
            rb = __hip_atomic_load(&q.res[tid_ep].bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            rid = __hip_atomic_load(&q.res[tid_ep].id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            rst = __hip_atomic_load(&q.res[tid_ep].step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int e = tid_ep; e < nsteps; e += NT) {
            s_bits[e] = __hip_atomic_load(q.hdr->bestbits + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_cnt[e] = __hip_atomic_load(q.hdr->count_feas + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_id[e] = ~0ull;
        }
        const unsigned short_sh = c_sh > sv_sh ? c_sh - sv_sh : 0u;  // this shard's survivors not finished
        if (tid_ep < 64) {
            const unsigned tot = (unsigned)wave_sum_u32((int)short_sh);
            if (tid_ep == 0) s_lost[0] = tot;
        }
        __syncthreads();
        const unsigned lost = (unsigned)__builtin_amdgcn_readfirstlane((int)s_lost[0]);
        SSPP_BEACON_E(2);
        // a shard with unfinished slots still holds their ready words: re-armed here (every finished
        // slot was re-armed by its consumer), so nothing stale reaches the next launch
        if (short_sh)
            for (unsigned e = 0; e < c_sh; ++e)
                __hip_atomic_store(q.rec + (unsigned)tid_ep * (unsigned)q.shard_cap + e, 0ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (tid_ep == 0) {
            if (lost) __hip_atomic_fetch_add(&q.hdr->lost_total, (unsigned long long)lost, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            if (no) __hip_atomic_fetch_add(&q.hdr->handoffs, (unsigned long long)no, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        }
        if (best_base) {
            if ((unsigned)tid_ep < nl && rb == s_bits[rst]) atomicMin(s_id + rst, rid);
            for (unsigned i = tid_ep + NT; i < nl; i += NT) {
                const unsigned long long bits = __hip_atomic_load(&q.res[i].bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long id = __hip_atomic_load(&q.res[i].id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int st = (int)__hip_atomic_load(&q.res[i].step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (bits == s_bits[st]) atomicMin(s_id + st, id);
            }
        }
        __syncthreads();
        SSPP_BEACON_E(3);
        for (int e = tid_ep; e < nsteps; e += NT) {
            if (best_base) {
                const bool has = s_id[e] != ~0ull;
                best_base[e].cost = has ? __longlong_as_double((long long)s_bits[e]) : INFINITY;
                best_base[e].index = has ? (long long)s_id[e] : -1;
                best_base[e].count = s_cnt[e];
                best_base[e].reserved = lost;
            }
            __hip_atomic_store(q.hdr->bestbits + e, 0x7FF0000000000000ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(q.hdr->count_feas + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int e = tid_ep; e < kSurvShards; e += NT) {
            __hip_atomic_store(&q.hdr->shard[e].count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->shard[e].taken, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->shard[e].pushed, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->shard[e].served, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid_ep == 0) {
            for (int k = 0; k < 8; ++k) __hip_atomic_store(&q.hdr->arrive_sh[k][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->arrive_top[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->nlist, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->lost, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q.hdr->norphan, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            SSPP_BEACON(13, (unsigned)wall_clock64(), lost);
#ifdef SSPP_WG_TIMING
            g_p2_t[8 * 4095] = t_ep;
            g_p2_t[8 * 4095 + 1] = wall_clock64();
            g_p2_t[8 * 4095 + 2] = gridDim.x;
#endif
        }
        return;
    }
    // ---- phase 2: survivors' remaining waypoints over the whole workgroup
    const int j0 = a.n1;
    const int R = a.npts - j0;
    if (collide_on && R > 0 && !(ABL & 8)) {
        if (tid < 64) {  // survivors compacted by one wave ballot (cpb <= 64), in candidate order
            const bool f = tid < nvalid && s_feas[tid] != 0;
            const unsigned long long m = __ballot(f);
            if (f) s_surv[__popcll(m & ((1ull << tid) - 1ull))] = tid;
            if (tid == 0) s_surv[cpb] = __popcll(m);
        }
        __syncthreads();
        int ns = s_surv[cpb];
        if (tid == 0) C2F_STAT(6, ns);
#ifdef SSPP_WG_TIMING
        wg_ns = ns;
#endif
        // the survivors' hull masks: AABB of the control points per (survivor, mover, axis),
        // then one (survivor, pair) test per thread (pair_may_touch; exact, see above).  Only
        // survivors: phase 1 stops at the first touching pair anyway, and computing the masks
        // for every candidate cost more than it saved (robocrane: 1.11 vs 1.22 G cand/s)
        // with 8 pairs or fewer the masks cull too little to pay for their two barriers and the
        // hull pass: robocrane (4 pairs) kernel 54.9 -> 53.7 us at 20 steps, 79.9 -> 78.1 us at
        // 1000 (profiles/r04aa_mask_ab.txt); the scan tests every pair exactly either way
#ifndef SSPP_P2_MASK_MIN
#define SSPP_P2_MASK_MIN 9
#endif
        const bool hull = np <= 64 && np >= SSPP_P2_MASK_MIN;  // otherwise every pair is scanned
        if (ns > 0 && hull) {
            for (int e = tid; e < ns * NB; e += NT) {
                const int si = e / NB, md = e - si * NB, m = md / 3, d = md - m * 3;
                const int sl = s_surv[si], col = 7 * m + d;
                double lo, hi;
                if (col < D) {
                    const int own = o_own + sl * nrd;
                    lo = hi = smem[crow(own, o_fix, r0, r1, 0, D) + col];
                    for (int j = 1; j < n; ++j) {
                        const double v = smem[crow(own, o_fix, r0, r1, j, D) + col];
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
        // Rounds: each round gives every live survivor the next cnt waypoints of the order
        // (cnt = NT / live survivors, so a round is one pass of the workgroup), then drops the
        // survivors it decided.  An infeasible survivor is usually decided by its first waypoints,
        // so the feasible ones then get the whole workgroup instead of a share of lanes that
        // idle on decided candidates.
        for (int jb = 0;;) {  // workgroup-uniform
            if (jb > 0) {
                __syncthreads();  // this round's flag updates are visible
                if (tid < 64) {   // in-place compaction by one wave (reads precede the writes)
                    const int s = tid < ns ? s_surv[tid] : 0;
                    const bool f = tid < ns && s_feas[s] != 0;
                    const unsigned long long m = __ballot(f);
                    if (f) s_surv[__popcll(m & ((1ull << tid) - 1ull))] = s;
                    if (tid == 0) s_surv[cpb] = __popcll(m);
                }
                __syncthreads();
                ns = __builtin_amdgcn_readfirstlane(s_surv[cpb]);
            }
            if (ns == 0) break;
            const int cnt = min(R - jb, max(1, NT / ns));
            unsigned long long um = 0ull;
            if (hull)
                for (int i = 0; i < ns; ++i) um |= s_mask[s_surv[i]];
            else
                um = ~0ull;
            const unsigned long long umask =  // workgroup-uniform: scalar registers
                ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(um >> 32)) << 32) |
                (unsigned)__builtin_amdgcn_readfirstlane((int)um);
            const int items = ns * cnt;
            // Few items for many lanes (a single-step launch's 4-wave workgroup with one survivor):
            // gp pair groups, each a 64-aligned copy of the item range on its own waves, group g
            // scanning the pairs k = g (mod gp).  A contact in any group clears the survivor's flag,
            // which stops the others; the result is the same OR over (waypoint, pair).
            int gp = 1, stride = items;
            if (NT == SSPP_C2F_GP_NT && np <= 64 && items > 0) {
                const int s64 = (items + 63) & ~63;
                while (gp < 8 && s64 * gp * 2 <= NT) gp *= 2;
                if (gp > 1) stride = s64;
            }
            const unsigned long long gsel = gp == 2 ? 0x5555555555555555ull
                                          : gp == 4 ? 0x1111111111111111ull
                                          : gp == 8 ? 0x0101010101010101ull : ~0ull;
            // one pass: items <= NT (cnt <= NT / ns), and with pair groups stride * gp <= NT
            {
                const int grp = gp > 1 ? tid / stride : 0;   // wave-uniform: stride is a multiple of 64
                const int it = tid - grp * stride;
                const unsigned long long gmask = gp > 1 ? gsel << grp : ~0ull;
                // waypoint-major items: item it = (waypoint jj of the round) x ns + survivor si, so
                // a pass holds the most telling remaining waypoints of every survivor
                bool live = it < items;
                const int jj = live ? it / ns : 0;
                const int si = live ? it - jj * ns : 0;
                const int s = s_surv[si];
                const int j = j0 + jb + jj;
                live = live && __hip_atomic_load(s_feas + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
                // a wave whose survivors have all been decided skips the spline / pose work
                if (__ballot(live) != 0ull) {
                    // lanes of this wave that work on the same survivor
                    unsigned long long gb = 0ull;
                    for (int q = 0; q < ns; ++q) {  // wave-uniform
                        const unsigned long long m = __ballot(it < items && si == q);
                        if (si == q) gb = m;
                    }
                    if (it >= items) gb = 0ull;
                    bool dfr = false, h;
                    const unsigned long long mym = (hull ? s_mask[s] : ~0ull) & gmask;
                    if (f32) {
                        float q32[D], N32[P1];
#pragma unroll
                        for (int r = 0; r < P1; ++r) N32[r] = otab32[j * P1 + r];
                        eval_split32<D, P>(s_f32, o_own + s * nrd, o_fix, r0, r1, N32, ospan[j], q32);
                        unsigned long long amb;
                        h = scan_pairs32<D, NM, ONEGEOM>(q32, live, mym, umask & gmask, gb, a.sc, TT, a.feps, a.fplim, amb);
                        const bool need = live && !h && amb != 0ull;
                        C2F_STAT(12, __popcll(__ballot(need)));
                        if (__ballot(need) != 0ull) {
                            double q[D];
                            eval_split_g<D, P>(smem, o_own + s * nrd, o_fix, r0, r1, otab + j * P1, ospan[j], q);
                            h = scan_pairs<D, NM, ONEGEOM>(q, need, amb, wave_or64(need ? amb : 0ull), gb, s_feas + s,
                                                           a.sc, TT, dfr) || h;
                        }
                    } else {
                        double q[D];
                        eval_split_g<D, P>(smem, o_own + s * nrd, o_fix, r0, r1, otab + j * P1, ospan[j], q);
                        h = scan_pairs<D, NM, ONEGEOM>(q, live, mym, umask & gmask, gb, s_feas + s, a.sc, TT, dfr);
                    }
                    if (h) __hip_atomic_store(s_feas + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (dfr) __hip_atomic_store(s_defer + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            jb += cnt;
            if (jb >= R) break;
        }
    }
    WG_PH(4);
    // ---- settle: candidates with no contact but an undecided cylinder-box pair get the exact
    // test at every collision waypoint (the OR over waypoints and pairs is unchanged)
    if (CBX && collide_on) {
        __syncthreads();
        if (tid < 64) {
            const bool u = tid < nvalid && s_feas[tid] != 0 && s_defer[tid] != 0;
            const unsigned long long m = __ballot(u);
            if (u) s_surv[__popcll(m & ((1ull << tid) - 1ull))] = tid;
            if (tid == 0) s_surv[cpb] = __popcll(m);
        }
        __syncthreads();
        const int nu = s_surv[cpb];
        for (int i = 0; i < nu; ++i) {  // workgroup-uniform
            const int s = s_surv[i];
            for (int j = tid; j < a.npts; j += NT) {
                if (__hip_atomic_load(s_feas + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) break;
                if (c2f_cb_exact<D, NM, P>(smem, o_own + s * nrd, o_fix, r0, r1, otab + j * P1, ospan[j], ~0ull, np, TT))
                    __hip_atomic_store(s_feas + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    // ---- phase 3: arc length (computeArcLength, include/sspp.h:152-169) of the listed
    // candidates: the collision-free ones (findBestPath scores only successful paths), or all
    // of them with arc_all.  Each candidate's chords are summed in the canonical order of
    // oracle/sspp_oracle.c::or_canon_sum: lpc lane partials (chords vl, vl+lpc, ...), an xor
    // butterfly per 64 lanes, 64-lane groups in order.
    __syncthreads();
    if (tid < cpb) s_arc[tid] = INFINITY;
    if (!(ABL & 4)) {
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
        // evaluating it again.
        const int lpc = a.lpc, nvw = lpc >> 6, lane = tid & 63;
        for (int vw = tid >> 6; vw < nl * nvw; vw += NT / 64) {  // wave-uniform
            const int si = vw / nvw, v = vw - si * nvw;
            const int own = o_own + s_list[si] * nrd;
            double acc = 0.0;
            for (int base = v * 64; base < nch; base += lpc) {  // wave-uniform trip count
                const int j = base + lane, jj = j < nch ? j : nch - 1;
                double qa[D], qb[D];
                eval_split_g<D, P>(smem, own, o_fix, r0, r1, atab + (jj + 1) * P1, aspan[jj + 1], qb);
#pragma unroll
                for (int d = 0; d < D; ++d) qa[d] = __shfl_up(qb[d], 1, 64);
                if (lane == 0) eval_split_g<D, P>(smem, own, o_fix, r0, r1, atab + jj * P1, aspan[jj], qa);
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
    WG_PH(5);
    if (tid == 0) C2F_STAT(7, nvalid);
    if (tid < nvalid) {
        const long long c = cand0 + tid;
        if (s_feas[tid]) C2F_STAT(8, 0);
        arc[c] = s_arc[tid];
        feasible[c] = (unsigned char)(s_feas[tid] != 0);
    }
    if (ctrl_out) {  // [B][n][D] rows: every candidate, or (ctrl_feas, plan()) the feasible ones
        double* dst = ctrl_out + cand0 * ndof;
        for (int e = tid; e < nvalid * ndof; e += NT) {
            const int sl = e / ndof, r = e - sl * ndof, j = r / D;
            if (!a.ctrl_feas || s_feas[sl]) dst[e] = smem[crow(o_own + sl * nrd, o_fix, r0, r1, j, D) + (r - j * D)];
        }
    }
    // block argmin over the workgroup's feasible candidates: one wave, lexicographic (cost, id)
    // xor butterfly (exact, order independent: the lowest id wins ties like the serial scan).
    // findBestPath (include/sspp.h:171-192) takes a path only when its cost < the running
    // minimum from +inf, so a feasible candidate with an infinite or NaN arc is never the best
    // (it still counts as feasible).
    BlockBest bb;
    if (tid < 64) {
        const bool f = tid < nvalid && s_feas[tid] != 0;
        const bool fa = f && s_arc[tid] < INFINITY;
        double bc = fa ? s_arc[tid] : INFINITY;
        long long bi = fa ? first_id + cand0 + tid : -1;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double oc = __shfl_xor(bc, off, 64);
            const long long oi = __shfl_xor(bi, off, 64);
            if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
        }
        bb.cost = bi < 0 ? INFINITY : bc; bb.idx = bi; bb.count = __popcll(__ballot(f)); bb.pad = 0;
    }
    finish_batch<NT>(bb, part, sync, best, a.nblk_step, blk);
    WG_PH(6);
#ifdef SSPP_WG_TIMING
    if (tid == 0 && blockIdx.x < (1 << 16)) {
        g_wg_t[4 * blockIdx.x] = wg_t0;
        g_wg_t[4 * blockIdx.x + 1] = wall_clock64();
        g_wg_t[4 * blockIdx.x + 2] = __smid();
        g_wg_t[4 * blockIdx.x + 3] = (unsigned long long)(long long)wg_ns;
    }
#endif
}

// ---------------------------------------------------------------- TaskSpacePlanner kernel
// tab: (cp+1) rows of 3 basis values at u = i * (1/cp); Minv: the collocation matrix's QR
// program (spline_host.cpp qr_program: [n][n] reflectors | [n] |v|^2 | [n][n] R).
#ifndef SSPP_TSP_WAVES_PER_EU
#define SSPP_TSP_WAVES_PER_EU 3
#endif
#ifndef SSPP_TSP_WAVES_PER_EU_CB  // with the exact cylinder-box test (its live state doubles)
#define SSPP_TSP_WAVES_PER_EU_CB 2
#endif
// The per-problem values of a TaskSpacePlanner launch: a k_tsp launch's own (TspK), or one goal's
// of a multi-goal launch (k_tsp_group, TspGoals)
struct TspVar {
    const double* start;
    const double* end;
    const double* fixed;
    const int* nfixed;
    unsigned long long seed;
    long long first_id;
};
__device__ __forceinline__ TspVar tsp_var(const TspK& a) {
    return TspVar{a.start, a.end, a.fixed, a.nfixed, a.seed, a.first_id};
}
// multi-goal launches (sspp_ces_plan_group): one CES iteration of up to kMaxGoals independent
// planners, goal g's workgroups [g nblk, (g + 1) nblk); the goal's problem, distribution and
// output buffers ride in the kernel arguments
constexpr int kMaxGoals = 16;
struct TspGoal {
    double start[4], end[4];
    unsigned long long seed;
    long long first_id;
    const double* fixed;
    const int* nfixed;
    const double* mean;
    const double* sigma;
    double *vias_out, *oL, *oCnf, *oCwf, *ocost;
    unsigned char* ostatus;
};
struct TspGoals {
    TspGoal g[kMaxGoals];
    int n, nblk;
};

// k_tsp's prologue, shared with k_tsp_pp: the candidates' via sets (given, CES fixed seeds or
// Sampler::sample_set draws) into s_V [cpb][n][4], vias_out, then PathModel::fromVias into
// s_ctrl [cpb][n][4].  Every thread of the workgroup calls it (it synchronises).
__device__ __forceinline__ void tsp_prologue(const TspK& a, const TspVar& pv, const double* __restrict__ Minv,
                                             const double* __restrict__ mean,
                                             const double* __restrict__ sigma,
                                             const double* __restrict__ vias_in,
                                             double* __restrict__ vias_out, int tid, int nthr, int cpb,
                                             long long cand0, long long nvalid, long long nfx,
                                             double* s_V, double* s_ctrl) {
    constexpr int D = 4;
    const int n = a.n, K = a.K, ndof = n * D;
    for (int e = tid; e < cpb * 2 * D; e += nthr) {
        const int s = e / (2 * D), r = e - s * 2 * D;
        if (r < D) s_V[s * ndof + r] = pv.start[r];
        else s_V[s * ndof + (n - 1) * D + (r - D)] = pv.end[r - D];
    }
    if (vias_in) {
        for (int e = tid; e < nvalid * K * D; e += nthr) {
            const int s = e / (K * D), r = e - s * K * D;
            s_V[s * ndof + D + r] = vias_in[(cand0 + s) * K * D + r];
        }
    } else {
        // Sampler::sample_set (tsp_sampler.h:12-51) with Philox streams per (candidate, via, dim)
        for (int e = tid; e < cpb * K * D; e += nthr) {
            const int s = e / (K * D), r = e - s * K * D;
            if (s >= nvalid) continue;
            const int v = r / D, i = r - v * D;
            long long gi = cand0 + s;
            if (a.ces) {
                const long long slot = a.slot0 + cand0 + s;
                if (slot < nfx) {  // mean set / forwarded best: no sampling
                    s_V[s * ndof + D + r] = pv.fixed[(slot * K + v) * D + i];
                    continue;
                }
                gi = slot - nfx;
                if (gi >= a.samples) {  // padding slot
                    s_V[s * ndof + D + r] = mean[v * D + i];
                    continue;
                }
            }
            const unsigned long long g = (unsigned long long)(pv.first_id + gi);
            const double m = mean[v * D + i], sg = sigma[v * D + i];
            double val;
            if (i < 3) {
                bool ok = false;
                val = 0.0;
                for (int t = 0; t < 99; ++t) {
                    double z0, z1;
                    normal_pair(pv.seed, g, (unsigned)(((v * 4 + i) << 7) | t), 1u, &z0, &z1);
                    val = z0 * sg;
                    val = val + m;
                    if (!(val < a.lo[i] || val > a.hi[i])) { ok = true; break; }
                }
                if (!ok) {
                    double u = uniform01(pv.seed, g, (unsigned)(((v * 4 + i) << 7) | 127), 1u);
                    val = u * (a.hi[i] - a.lo[i]);
                    val = val + a.lo[i];
                }
                if (i == 2 && val < a.z_min) val = a.z_min;
            } else if (a.lo[3] != a.hi[3]) {
                double z0, z1;
                normal_pair(pv.seed, g, (unsigned)((v * 4 + 3) << 7), 1u, &z0, &z1);
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
        for (int e = tid; e < nvalid * K * D; e += nthr) {
            const int s = e / (K * D), r = e - s * K * D;
            vias_out[(cand0 + s) * K * D + r] = s_V[s * ndof + D + r];
        }
    }
    // PathModel::fromVias: SplineFitting::Interpolate's Householder QR solve, replayed from the
    // host-factored program (reflectors, |v|^2, R) in oracle qr_solve's operation order, one
    // lane per (candidate, dimension): control points bit-identical to the oracle's
    for (int e = tid; e < cpb * D; e += nthr) {
        const int s = e / D, d = e - s * D;
        const double* Vs = s_V + s * ndof;
        double* c = s_ctrl + s * ndof;
        for (int i = 0; i < n; ++i) c[i * D + d] = Vs[i * D + d];
        const double* vn = Minv + n * n;
        const double* R = vn + n;
        for (int k = 0; k < n; ++k) {
            const double q = vn[k];
            if (q == 0.0) continue;
            const double* v = Minv + k * n;
            double sd = 0.0;
            for (int i = k; i < n; ++i) sd = fma(v[i], c[i * D + d], sd);
            sd = 2.0 * sd / q;
            for (int i = k; i < n; ++i) c[i * D + d] = c[i * D + d] - sd * v[i];
        }
        for (int i = n - 1; i >= 0; --i) {
            double t = c[i * D + d];
            for (int cc = i + 1; cc < n; ++cc) t = t - R[i * n + cc] * c[cc * D + d];
            c[i * D + d] = t / R[i * n + i];
        }
    }
    __syncthreads();

}

// CB: the scene has cylinder-box pairs (without them the exact cylinder-box code is compiled
// out: it costs registers even when it never runs)
// Several moving geoms (the gripper's 7): 3 waves per SIMD, 168 VGPRs with ~50 spilled, beats
// 2 waves without spills (multi-goal 40.6 against 34.6 M cand/s; 4 waves: 29.8)
#ifndef SSPP_TSP_WAVES_PER_EU_MG
#define SSPP_TSP_WAVES_PER_EU_MG 3
#endif
// DEF (one waypoint per lane, at most kDefPairs pairs): box-box contact polygons deferred — the
// waypoint loop records every pair's count / term (REC 3), the workgroup then counts the
// polygons of its compacted deep box-box pairs (all lanes busy, instead of the lanes of each
// wave that happen to hold one), and each lane sums its records in pair order: the same additions
// in the same order as the inline form, so the costs are bit-identical.
constexpr int kDefPairs = 8;
#ifndef SSPP_TSP_SUB_LAUNDER
#define SSPP_TSP_SUB_LAUNDER 1
#endif
// 4 waves per SIMD, no spills.  5 waves (96 VGPRs, ~75 spilled) measured 106.0 against 101.6 M
// cand/s on stacking, but its spills raised the HBM traffic from 1.4x to 140x the algorithmic bytes
#ifndef SSPP_TSP_WAVES_PER_EU_DEF
#define SSPP_TSP_WAVES_PER_EU_DEF 4
#endif
// k_tsp's body: workgroup blk of a problem (k_tsp: the launch's; k_tsp_group: a goal's)
template <int NM, bool ONEGEOM, int CB, bool UP, int DEF>
__device__ __forceinline__ void tsp_body(
    const TspK& a, const TspVar& pv, const SceneT& T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ Minv, const double* __restrict__ mean,
    const double* __restrict__ sigma, const double* __restrict__ vias_in,
    double* __restrict__ vias_out, double* __restrict__ oL, double* __restrict__ oCnf,
    double* __restrict__ oCwf, double* __restrict__ ocost, unsigned char* __restrict__ ostatus,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best, int blk) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int D = 4, P = 2, P1 = 3;
    const int tid = threadIdx.x, lpc = a.lpc, cpb = a.cpb, n = a.n, cp = a.cp;
    const int slot = tid / lpc, lane = tid - slot * lpc;
    // rep sub-batches of cpb candidates per workgroup: one prologue (sampling, QR) over all of
    // them, then the waypoint loop per sub-batch (tsp_rep: fewer, longer workgroups)
    // (forms in SSPP_TSP_REP_FORMS only: elsewhere the loop's live state costs spills)
    constexpr bool REP_OK = ((SSPP_TSP_REP_FORMS >> (DEF == 1 ? 3 : DEF == 2 ? 4 : 0)) & 1) != 0;
    const int rep = (REP_OK && a.rep > 1) ? a.rep : 1, cpr = cpb * rep;
    const long long candR = (long long)blk * cpr;
    const int ndof = n * D;
    double* s_V = smem;                      // [cpr][n][4]
    double* s_ctrl = s_V + cpr * ndof;       // [cpr][n][4]
    double* s_wsum = s_ctrl + cpr * ndof;    // [3][4]
    double* s_best = s_wsum + 3 * (kBlock / 64);
    int* s_stat = (int*)(s_best + (cpr > 4 ? cpr : 4));  // [cpr]
    // DEF 1: per-lane records [kBlock][np] (terms, counts), mover poses [kBlock][8], deferred list;
    // DEF 2: per-lane counts [kBlock][np] and mover poses only
    const int npr = DEF ? a.sc.npairs : 0;
    double* s_rterm = (double*)(s_stat + ((cpr + 1) & ~1));
    double* s_rpose = s_rterm + (DEF == 1 ? kBlock * npr : 0);
    unsigned char* s_rnd = (unsigned char*)(s_rpose + (DEF ? kBlock * 8 : 0));
    int* s_items = (int*)(s_rnd + ((kBlock * npr + 3) & ~3));
    int* s_nitems = s_items + kBlock * npr;

    const long long nvR = min((long long)cpr, a.B - candR);
    const long long nfx = a.ces ? (long long)*pv.nfixed : 0;  // uniform: scalar load
    tsp_prologue(a, pv, Minv, mean, sigma, vias_in, vias_out, tid, kBlock, cpr, candR, nvR, nfx, s_V, s_ctrl);

    // one sub-batch; the forms without sub-batches compile it once, with no loop around it
    const int tid_o = tid, slot_o = slot, lane_o = lane;
    auto sub = [&](const int r) -> bool {
#if SSPP_TSP_SUB_LAUNDER
    // the lane's indices through an empty asm per sub-batch: what derives from them (LDS record
    // pointers, the basis rows of its waypoint) is recomputed per sub-batch instead of being
    // hoisted in front of the loop and held (spilled) across it
    int tid = tid_o;
    if constexpr (REP_OK) asm volatile("" : "+v"(tid));
    const int slot = REP_OK ? tid / lpc : slot_o, lane = REP_OK ? tid - slot * lpc : lane_o;
#endif
    const long long cand0 = candR + (long long)r * cpb;
    const long long nvalid = min((long long)cpb, a.B - cand0);  // <= 0 past a ragged batch's end
    if (REP_OK && nvalid <= 0) return false;  // past a ragged batch's end
    if (r > 0) __syncthreads();  // the previous sub-batch is done with the sums and records
    // Evaluator::eval_one_pass (tsp_evaluator.h:18-32), waypoint i = 1..cp per lane
    const bool valid = slot < nvalid;
    const double* myc = s_ctrl + (r * cpb + slot) * ndof;
    const unsigned long long mask = hull_mask<D, NM, 1>(myc, n, a.sc.npairs, (cpair_t)T.pairs,
                                                        (cgeom_t)T.geoms, (cmover_t)T.movers,
                                                        DEF == 2 ? T.visit : nullptr);
    double aL = 0.0, aC = 0.0, aW = 0.0;
    // cp <= lpc: one waypoint per lane, so s((i-1)du) is the previous lane's s(i du); take it
    // by shuffle (bit-identical: same eval_pt inputs) except on a wave's first lane
    const bool one_pass = cp <= lpc;
    if (DEF == 1) {  // host-checked: one waypoint per lane (cp <= lpc), np <= kDefPairs, NM == 1
        if (tid == 0) *s_nitems = 0;
        unsigned char* rn = s_rnd + tid * npr;
        double* rt = s_rterm + tid * npr;
        for (int k = 0; k < npr; ++k) rn[k] = 0;
        const bool has = valid && lane < cp;
        if (has) {
            const int i = lane + 1;
            double pv[4], pc[4];
            eval_pt<D, P>(myc, tab + i * P1, span[i], pc);
#pragma unroll
            for (int d = 0; d < D; ++d) pv[d] = __shfl_up(pc[d], 1, 64);
            if ((tid & 63) == 0) eval_pt<D, P>(myc, tab + (i - 1) * P1, span[i - 1], pv);
            aL = aL + dist_nd<D>(pv, pc);
            // (the waypoint's height pz is read back from the recorded mover pose after the
            // records are counted: a register less across the pair loop)
#ifndef SSPP_PROF_NOCOLL  // profiling variant only
            point_collide<D, NM, 1, true, ONEGEOM, CB, 3, UP>(pc, a.sc, T, mask, nullptr, nullptr, rn, rt,
                                                             s_rpose + tid * 8);
#else
            s_rpose[tid * 8 + 2] = pc[2];
#endif
        }
        __syncthreads();
        // compact the deferred (lane, pair) records: one wave ballot + one LDS add per wave
        for (int e0 = 0; e0 < kBlock * npr; e0 += kBlock) {  // workgroup-uniform
            const int e = e0 + tid;
            const bool pend = e < kBlock * npr && s_rnd[e] >= kBbPend;
            const unsigned long long m = __ballot(pend);
            int base = 0;
            if ((tid & 63) == 0 && m) base = atomicAdd(s_nitems, __popcll(m));
            base = __shfl(base, 0, 64);
            if (pend) s_items[base + __popcll(m & ((1ull << (tid & 63)) - 1ull))] = e;
        }
        __syncthreads();
        const int nit = *s_nitems;
        const cgeom_t geoms = (cgeom_t)T.geoms;
        const cpair_t pairs = (cpair_t)T.pairs;
        for (int it = tid; it < nit; it += kBlock) {
            const int e = s_items[it], ln = e / npr, k = e - ln * npr;
            const int fi = s_rnd[e] - kBbPend;
            const double* ps = s_rpose + ln * 8;
            const double mp0[3] = {ps[0], ps[1], ps[2]};
            const double mR0[9] = {ps[3], ps[4], 0.0, ps[5], ps[6], 0.0, 0.0, 0.0, ps[7]};
            const DPair pr = pairs[k];
            const DGeom G = geoms[pr.gm];
            double gp[3], gm[9];
            geom_pos_t<true>(mp0, mR0, G, gp);
            geom_rot_t<true>(mR0, G, gm);
            const bool gfirst = G.orig < pr.oorig;  // both boxes
            const int nd = gfirst ? (UP ? bb_clip_count_up(gp, gm, G.size, pr.opos, pr.omat, pr.osize, fi)
                                        : bb_clip_count(gp, gm, G.size, pr.opos, pr.omat, pr.osize, fi))
                                  : (UP ? bb_clip_count_up(pr.opos, pr.omat, pr.osize, gp, gm, G.size, fi)
                                        : bb_clip_count(pr.opos, pr.omat, pr.osize, gp, gm, G.size, fi));
            s_rnd[e] = (unsigned char)nd;
        }
        __syncthreads();
        if (has) {  // this waypoint's cost: the records in pair order (point_collide's sum)
            double acc = 0.0;
            for (int k = 0; k < npr; ++k) {
                const int nd = rn[k];
                if (nd == 0) continue;
                const double term = rt[k];
                for (int r = 0; r < nd; ++r) acc = acc + term;
            }
            const double c = acc + a.sc.static_cost;
            const double pz = s_rpose[tid * 8 + 2];  // the mover position is the waypoint's (MODE 1)
            const double deficit = (a.floor_z_min + a.floor_margin) - pz;
            const double fp = deficit > 0.0 ? (a.floor_scale * deficit) * deficit : 0.0;
            aC = aC + c;
            aW = aW + (c + fp);
        }
    } else if (DEF == 2) {  // host-checked: one waypoint per lane (cp <= lpc), np <= 64, NM == 1
        unsigned char* rn = s_rnd + tid * npr;
        double* ps = s_rpose + tid * 8;
        for (int k = 0; k < npr; ++k) rn[k] = 0;
        const bool has = valid && lane < cp;
        if (has) {
            const int i = lane + 1;
            double pv[4], pc[4];
            eval_pt<D, P>(myc, tab + i * P1, span[i], pc);
#pragma unroll
            for (int d = 0; d < D; ++d) pv[d] = __shfl_up(pc[d], 1, 64);
            if ((tid & 63) == 0) eval_pt<D, P>(myc, tab + (i - 1) * P1, span[i - 1], pv);
            aL = aL + dist_nd<D>(pv, pc);
            point_collide<D, NM, 1, true, ONEGEOM, CB, 4, UP>(pc, a.sc, T, mask, nullptr, nullptr, rn, nullptr, ps);
        }
        const double c = tsp_lane_sum<UP>(has, rn, ps, npr, a.sc, T);  // every lane: wave ballots
        if (has) {
            const double pz = ps[2];  // the mover position is the waypoint's (MODE 1)
            const double deficit = (a.floor_z_min + a.floor_margin) - pz;
            const double fp = deficit > 0.0 ? (a.floor_scale * deficit) * deficit : 0.0;
            aC = aC + c;
            aW = aW + (c + fp);
        }
    } else if (valid) {
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
            point_collide<D, NM, 1, true, ONEGEOM, CB, 0, UP>(pc, a.sc, T, mask, &c);
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
        s_stat[r * cpb + slot] = st;
        s_best[r * cpb + slot] = cost;
    }
    return true;
    };
    if constexpr (REP_OK) {
        for (int r = 0; r < rep; ++r)  // workgroup-uniform
            if (!sub(r)) break;
    } else {
        sub(0);
    }
    __syncthreads();
    BlockBest bb;
    if (tid == 0) {
        bb.cost = INFINITY; bb.idx = -1; bb.count = 0; bb.pad = 0;
        for (int s = 0; s < nvR; ++s) {
            if (!s_stat[s]) continue;
            bb.count++;
            if (s_best[s] < bb.cost) { bb.cost = s_best[s]; bb.idx = pv.first_id + candR + s; }
        }
    }
    if (part || best) finish_batch(bb, part, sync, best);  // (CES slot mode: records unused)
}

template <int NM, bool ONEGEOM, int CB, bool UP = false, int DEF = 0>
__global__ __launch_bounds__(kBlock, DEF == 1 ? SSPP_TSP_WAVES_PER_EU_DEF
                                              : (CB == 1 ? SSPP_TSP_WAVES_PER_EU_CB
                                                         : (ONEGEOM ? SSPP_TSP_WAVES_PER_EU : SSPP_TSP_WAVES_PER_EU_MG))) void k_tsp(
    TspK a, SceneT T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ Minv, const double* __restrict__ mean,
    const double* __restrict__ sigma, const double* __restrict__ vias_in,
    double* __restrict__ vias_out, double* __restrict__ oL, double* __restrict__ oCnf,
    double* __restrict__ oCwf, double* __restrict__ ocost, unsigned char* __restrict__ ostatus,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    tsp_body<NM, ONEGEOM, CB, UP, DEF>(a, tsp_var(a), T, tab, span, Minv, mean, sigma, vias_in, vias_out, oL, oCnf,
                                       oCwf, ocost, ostatus, part, sync, best, (int)blockIdx.x);
}

// one CES iteration's evaluation of every goal of a multi-goal launch (sspp_ces_plan_group): the
// same body per workgroup, the goal's values and buffers from the arguments
template <int NM, bool ONEGEOM, int CB, bool UP = false, int DEF = 0>
__global__ __launch_bounds__(kBlock, DEF == 1 ? SSPP_TSP_WAVES_PER_EU_DEF
                                              : (CB == 1 ? SSPP_TSP_WAVES_PER_EU_CB
                                                         : (ONEGEOM ? SSPP_TSP_WAVES_PER_EU : SSPP_TSP_WAVES_PER_EU_MG))) void k_tsp_group(
    TspK a, TspGoals G, SceneT T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ Minv) {
    const int g = (int)blockIdx.x / G.nblk, blk = (int)blockIdx.x - g * G.nblk;
    const TspGoal& q = G.g[g];
    const TspVar pv{q.start, q.end, q.fixed, q.nfixed, q.seed, q.first_id};
    tsp_body<NM, ONEGEOM, CB, UP, DEF>(a, pv, T, tab, span, Minv, q.mean, q.sigma, nullptr, q.vias_out, q.oL, q.oCnf,
                                       q.oCwf, q.ocost, q.ostatus, nullptr, nullptr, nullptr, blk);
}

// ---------------------------------------------------------------- TaskSpacePlanner, pair-split
// Latency form of k_tsp for small batches (the anytime CES loop: 17 slots x 40 check points):
// one workgroup per candidate, G waves; wave g evaluates the pairs k = g, g + G, ... of the
// candidate's (<= 64) waypoints, one waypoint per lane, so a lane runs ~np/G pair tests instead
// of np.  Deep pairs are recorded per (waypoint, pair) in LDS; wave 0 then sums each waypoint's
// terms in pair order and runs k_tsp's epilogue (same lanes, shuffles and reductions), so every
// output is bit-identical to k_tsp's.  Needs cp <= 64 and np <= 64 (host check).
template <int NM, bool ONEGEOM, int CB, int G>
__global__ __launch_bounds__(64 * G, 2) void k_tsp_pp(
    TspK a, SceneT T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ Minv, const double* __restrict__ mean,
    const double* __restrict__ sigma, const double* __restrict__ vias_in,
    double* __restrict__ vias_out, double* __restrict__ oL, double* __restrict__ oCnf,
    double* __restrict__ oCwf, double* __restrict__ ocost, unsigned char* __restrict__ ostatus,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int D = 4, P = 2, P1 = 3, NT = 64 * G;
    const int tid = threadIdx.x, n = a.n, cp = a.cp, np = a.sc.npairs;
    const int g = tid >> 6, lane = tid & 63;
    const long long cand0 = blockIdx.x;
    const int ndof = n * D;
    double* s_V = smem;                       // [n][4]
    double* s_ctrl = s_V + ndof;              // [n][4]
    double* s_term = s_ctrl + ndof;           // [64 waypoints][64 pairs]
    unsigned char* s_nd = (unsigned char*)(s_term + 64 * 64);  // [64][64]
    const long long nvalid = 1;
    const long long nfx = a.ces ? (long long)*a.nfixed : 0;
    for (int e = tid; e < 64 * 64 / 4; e += NT) ((unsigned*)s_nd)[e] = 0u;
    tsp_prologue(a, tsp_var(a), Minv, mean, sigma, vias_in, vias_out, tid, NT, 1, cand0, nvalid, nfx, s_V, s_ctrl);
    const unsigned long long mask = hull_mask<D, NM, 1>(s_ctrl, n, np, (cpair_t)T.pairs,
                                                        (cgeom_t)T.geoms, (cmover_t)T.movers);
    // this wave's pairs: k = g (mod G)
    unsigned long long gm = 0ull;
    for (int k = g; k < 64; k += G) gm |= 1ull << k;
    const int i = lane + 1;  // waypoint
    double pc[4];
    if (lane < cp) {
        eval_pt<D, P>(s_ctrl, tab + i * P1, span[i], pc);
#ifndef SSPP_PROF_NOCOLL
        if (mask & gm)
            point_collide<D, NM, 1, true, ONEGEOM, CB, 1>(pc, a.sc, T, mask & gm, nullptr, nullptr,
                                                          s_nd + lane * 64, s_term + lane * 64);
#endif
    }
    __syncthreads();
    // ---- wave 0: k_tsp's per-lane waypoint epilogue (lpc = 64, one waypoint per lane)
    double aL = 0.0, aC = 0.0, aW = 0.0;
    BlockBest bb;
    if (g == 0) {
        double pv[4];
        if (lane < cp) {
#pragma unroll
            for (int d = 0; d < D; ++d) pv[d] = pc[d];
        }
        // s((i-1)du) is the previous lane's s(i du), as in k_tsp's one-pass form
#pragma unroll
        for (int d = 0; d < D; ++d) pv[d] = __shfl_up(pv[d], 1, 64);
        if (lane < cp) {
            if (lane == 0) eval_pt<D, P>(s_ctrl, tab + (i - 1) * P1, span[i - 1], pv);
            aL = aL + dist_nd<D>(pv, pc);
            double acc = 0.0;
            const unsigned char* rn = s_nd + lane * 64;
            const double* rt = s_term + lane * 64;
            for (int k = 0; k < np; ++k) {
                const int nd = rn[k];
                if (nd == 0) continue;
                const double term = rt[k];
                for (int r = 0; r < nd; ++r) acc = acc + term;
            }
            const double c = acc + a.sc.static_cost;
            const double deficit = (a.floor_z_min + a.floor_margin) - pc[2];
            const double fp = deficit > 0.0 ? (a.floor_scale * deficit) * deficit : 0.0;
            aC = aC + c;
            aW = aW + (c + fp);
        }
    }
    if (g == 0) {
        aL = wave_sum(aL);
        aC = wave_sum(aC);
        aW = wave_sum(aW);
    }
    if (tid == 0) {
        double L = aL, Cn = aC, Cw = aW;
        int st = Cn == 0.0;
        double cost = L + a.w_col * Cw;
        if (a.ces && a.slot0 + cand0 >= nfx + a.samples) {  // padding slot
            st = 0; cost = INFINITY; L = 0.0; Cn = 0.0; Cw = 0.0;
        }
        oL[cand0] = L; oCnf[cand0] = Cn; oCwf[cand0] = Cw; ocost[cand0] = cost;
        ostatus[cand0] = (unsigned char)st;
        bb.cost = st ? cost : INFINITY; bb.idx = st ? a.first_id + cand0 : -1; bb.count = st; bb.pad = 0;
    }
    finish_batch<NT>(bb, part, sync, best);
}

// k_tsp_pp over npg workgroups per candidate: workgroup (cand, pg) evaluates pair group
// pg * G + g (pairs k = that group mod npg * G) on its waves, one waypoint per lane, and stores
// every (waypoint, pair) of its groups — contact count (0 when not deep) and term — as
// write-through agent-scope stores; its last arriving workgroup (agent-scope acquire) sums each
// waypoint in pair order and runs the epilogue.  Same outputs as k_tsp, bit for bit.
template <int NM, bool ONEGEOM, int CB, int G>
__global__ __launch_bounds__(64 * G, 2) void k_tsp_pp2(
    TspK a, SceneT T, const double* __restrict__ tab, const int* __restrict__ span,
    const double* __restrict__ Minv, const double* __restrict__ mean,
    const double* __restrict__ sigma, const double* __restrict__ vias_in,
    double* __restrict__ vias_out, double* __restrict__ oL, double* __restrict__ oCnf,
    double* __restrict__ oCwf, double* __restrict__ ocost, unsigned char* __restrict__ ostatus,
    BlockBest* __restrict__ part, ArgminSync* sync, sspp_best* best) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    constexpr int D = 4, P = 2, P1 = 3, NT = 64 * G;
    __shared__ int s_last;
    const int tid = threadIdx.x, n = a.n, cp = a.cp, np = a.sc.npairs, npg = a.npg;
    const int g = tid >> 6, lane = tid & 63;
    const long long cand0 = blockIdx.x / npg;
    const int pg = blockIdx.x - (int)cand0 * npg;
    const int ngr = npg * G, gg = pg * G + g;  // pair groups in all, this wave's group
    const int ndof = n * D;
    double* s_V = smem;           // [n][4]
    double* s_ctrl = s_V + ndof;  // [n][4]
    const long long nfx = a.ces ? (long long)*a.nfixed : 0;
    tsp_prologue(a, tsp_var(a), Minv, mean, sigma, vias_in, pg == 0 ? vias_out : nullptr, tid, NT, 1, cand0, 1, nfx,
                 s_V, s_ctrl);
    const unsigned long long mask = hull_mask<D, NM, 1>(s_ctrl, n, np, (cpair_t)T.pairs,
                                                        (cgeom_t)T.geoms, (cmover_t)T.movers);
    unsigned long long gm = 0ull;
    for (int k = gg; k < np; k += ngr) gm |= 1ull << k;
    const int i = lane + 1;
    unsigned* rn = a.rec_nd + (cand0 * 64 + lane) * 64;
    double* rt = a.rec_term + (cand0 * 64 + lane) * 64;
    if (lane < cp && gm) {
        double pc[4];
        eval_pt<D, P>(s_ctrl, tab + i * P1, span[i], pc);
        // this lane's groups' entries: 0 unless the pair is deep (then count and term)
        for (int k = gg; k < np; k += ngr) __hip_atomic_store(rn + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifndef SSPP_PROF_NOCOLL
        if (mask & gm)
            point_collide<D, NM, 1, true, ONEGEOM, CB, 2>(pc, a.sc, T, mask & gm, nullptr, nullptr, rn, rt);
#endif
    }
    // publish: every storing wave drains, the workgroup meets, one lane counts the arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.arrive + cand0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == (unsigned)npg - 1u;
        if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            __hip_atomic_store(a.arrive + cand0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (!s_last) return;
    double aL = 0.0, aC = 0.0, aW = 0.0;
    BlockBest bb;
    if (g == 0) {
        double pc[4], pv[4];
        if (lane < cp) eval_pt<D, P>(s_ctrl, tab + i * P1, span[i], pc);
#pragma unroll
        for (int d = 0; d < D; ++d) pv[d] = __shfl_up(lane < cp ? pc[d] : 0.0, 1, 64);
        if (lane < cp) {
            if (lane == 0) eval_pt<D, P>(s_ctrl, tab + (i - 1) * P1, span[i - 1], pv);
            aL = aL + dist_nd<D>(pv, pc);
            double acc = 0.0;
            for (int k = 0; k < np; ++k) {
                if (!((mask >> k) & 1ull)) continue;  // culled pairs were never evaluated
                const unsigned nd = __hip_atomic_load(rn + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (nd == 0u) continue;
                const double term = __hip_atomic_load(rt + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (unsigned r = 0; r < nd; ++r) acc = acc + term;
            }
            const double c = acc + a.sc.static_cost;
            const double deficit = (a.floor_z_min + a.floor_margin) - pc[2];
            const double fp = deficit > 0.0 ? (a.floor_scale * deficit) * deficit : 0.0;
            aC = aC + c;
            aW = aW + (c + fp);
        }
        aL = wave_sum(aL);
        aC = wave_sum(aC);
        aW = wave_sum(aW);
    }
    if (tid == 0) {
        double L = aL, Cn = aC, Cw = aW;
        int st = Cn == 0.0;
        double cost = L + a.w_col * Cw;
        if (a.ces && a.slot0 + cand0 >= nfx + a.samples) {  // padding slot
            st = 0; cost = INFINITY; L = 0.0; Cn = 0.0; Cw = 0.0;
        }
        oL[cand0] = L; oCnf[cand0] = Cn; oCwf[cand0] = Cw; ocost[cand0] = cost;
        ostatus[cand0] = (unsigned char)st;
        bb.cost = st ? cost : INFINITY; bb.idx = st ? a.first_id + cand0 : -1; bb.count = st; bb.pad = 0;
    }
    finish_batch<NT>(bb, part, sync, best, (int)a.B, (int)cand0);
}

// ---------------------------------------------------------------- argmin over block results


// TaskSpacePlanner batches up to this size take k_tsp_pp (one workgroup per candidate)
constexpr int64_t kTspPpMaxBatch = 512;
// extra LDS of k_tsp<..., DEF>: records (terms, counts), poses, the deferred list and its count
inline size_t tsp_def_lds(int np) {
    return sizeof(double) * (size_t)kBlock * (np + 8) + (((size_t)kBlock * np + 3) & ~(size_t)3) +
           sizeof(int) * ((size_t)kBlock * np + 1) + 16;
}

// extra LDS of k_tsp<..., DEF 2>: per-lane counts and mover poses
inline size_t tsp_def2_lds(int np) {
    return sizeof(double) * (size_t)kBlock * 8 + (((size_t)kBlock * np + 7) & ~(size_t)7) + 16;
}
// k_tsp's LDS before the DEF records, for rep sub-batches of cpb candidates (tsp_body's layout)
inline size_t tsp_base_lds(int cpb, int n, int rep) {
    const int cpr = cpb * (rep > 1 ? rep : 1);
    return sizeof(double) * ((size_t)2 * cpr * n * 4 + 3 * (kBlock / 64) + (cpr > 4 ? cpr : 4)) +
           sizeof(int) * (size_t)((cpr + 1) & ~1);
}

inline int lanes_for(int items) {
    int l = ((items + 63) / 64) * 64;
    return std::min(std::max(l, 64), kBlock);
}

}  // namespace sspk

using namespace sspk;

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
    DPair* d_visit = nullptr;  // the pairs grouped by moving geom (SceneT::visit)
    int device = 0;
};

struct sspp_job {
    int kind = 0;  // 0 sspp, 1 tsp
    const sspp_scene* scene = nullptr;
    int D = 0, p = 0, n = 0, W = 0, nknots = 0, K = 0, cp = 0;
    int lpc = 0, cpb = 0, nm = 1;
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
    int64_t part_cap = 0;      // BlockBest records d_part holds
    int sampler = 0;           // 0 FP64 Box-Muller pairs (default), 1 FP32 quads (opt-in)
    int arc_all = 0;           // arc length for every candidate (else collision-free only)
    // k_sspp_c2f launch shape: chosen per launch from the candidates it holds unless forced by
    // sspp_job_set_option (SSPP_OPT_SHAPE_NT / _G1, tests and tuning); the effective values of
    // the last launch are readable (sspp_job_get_option)
    int opt_nt = 0, opt_g1 = 0;
    int last_nt = 0, last_g1 = 0;
    int pair_order = 0;        // effective pair order of the tables (SSPP_ORDER_*)
    int wp_order = 0;          // effective collision-waypoint order (SSPP_ORDER_*)
    int f32 = 1;               // k_sspp_c2f's FP32-filtered scan (SSPP_OPT_F32; results identical)
    int last_f32 = 0;          // whether the last launch ran it
    double prepass_ms = 0.0;   // host time of the hit-order pre-pass at creation
    double* d_otab = nullptr;  // collision rows in the job's waypoint order
    float* d_otab32 = nullptr; // the same rows in FP32 (k_sspp_c2f's filtered scan)
    int* d_ospan = nullptr;
    std::vector<int> h_wps;    // that order
    DPair* d_pairs = nullptr;  // this job's pair table (ordered)
    DPair* d_pairs_s = nullptr;  // the same without the pairs no sampled candidate can reach
    int np_full = 0, np_samp = 0, cb_full = 0, cb_samp = 0, og_full = 1, og_samp = 1;
    ArgminSync* d_sync = nullptr;  // sharded arrival counters of the fused argmin [kMaxSteps]
    std::vector<double> h_knots;   // host copies: the knot vector, and the values the device
    std::vector<double> h_stage;   // holds (init | limits; sspp_job_update_sspp skips equal updates)
    std::vector<DPair> h_pairs, h_pairs_s;
    int ctrl_feas = 0;               // k_sspp_c2f writes ctrl_out rows of feasible candidates only
    // TaskSpacePlanner options (sspp_job_set_option): evaluation form (-1 automatic, 0 k_tsp,
    // 1 k_tsp_pp, 2 k_tsp_pp2) and the generic (non-upright) narrowphase
    int tsp_form = -1, tsp_generic = 0, last_form = -1;
    int tsp_rep = -1, last_rep = 1;     // SSPP_OPT_TSP_REP
    unsigned* d_pp_nd = nullptr;     // k_tsp_pp2 records / arrival counters (allocated on first use)
    double* d_pp_term = nullptr;
    unsigned* d_pp_arrive = nullptr;
    int64_t pp_cap = 0;
    unsigned char* h_pin = nullptr;  // pinned source of sspp_job_update_sspp's async copies
    size_t h_pin_bytes = 0;
    hipEvent_t upd_ev = nullptr;     // recorded after those copies: the next update waits on it
    bool upd_pending = false;
    double start[4], end[4], lo[4], hi[4];
    double z_min = 0, w_col = 1, floor_z_min = 0, floor_margin = 0.01, floor_scale = 10;
    // asynchronous hit-order pre-pass (the drop-in planner's first plan(): DESIGN.md §5): the
    // census runs on its own stream and a host thread orders the tables; the next launch after
    // it lands swaps them in.  Until then the job scans in gap / bisection order (identical results).
    std::thread prepass_thread;
    std::atomic<int> prepass_state{0};  // 0 none, 1 running, 2 result ready, 3 applied or dropped
    std::vector<int> pre_wps;           // the thread's result: waypoint order,
    std::vector<DPair> pre_pairs, pre_pairs_s;  // pair tables (hit order) for the creation's values
    double pre_ms = 0.0;                // census + host ordering, wall time
    int pre_gen = 0;                    // tables_gen the result was computed for
    int tables_gen = 0;                 // bumped by every update that re-derives the pair tables
    hipStream_t pre_stream = nullptr;
    hipEvent_t pre_ev = nullptr;
    unsigned long long* d_hits = nullptr;
    unsigned long long* h_hits = nullptr;  // pinned
    DPair* d_census_pairs = nullptr;    // the census's own copy of the sampled table
    std::vector<void*> retired;         // device tables replaced while kernels may still read them
    double create_ms = 0.0;             // host time of sspp_job_create_sspp
    // split launches: the survivor queue (SurvQ), grown on demand
    int opt_split = 1;                  // SSPP_OPT_SPLIT
    int last_split = 0;
    SurvQ* d_sq_hdr = nullptr;
    unsigned long long* d_sq_rec = nullptr;
    double* d_sq_ctrl = nullptr;
    float* d_sq_ctrl32 = nullptr;
    SurvBest* d_sq_res = nullptr;
    unsigned* d_sq_orphan = nullptr;
    int opt_linger_us = 10000;          // SSPP_OPT_SPLIT_LINGER_US (10 ms)
    int opt_split_drop = 0;             // SSPP_OPT_SPLIT_DROP (tests)
    unsigned* dbg_beacon = nullptr;     // SSPP_OPT_DEBUG_BEACONS (-DSSPP_DEBUG_PROGRESS builds)
    long long sq_cap = 0;               // survivors the buffers hold (x sq_nrd doubles each)
    int sq_nrd = 0;
};


namespace sspk {

// generic: the TaskSpacePlanner generic box-box narrowphase even where every pair is upright
inline KScene kscene(const sspp_scene* s, bool tsp, bool generic = false) {
    KScene k{};
    if (!s) return k;
    k.npairs = (int)s->pairs.size();
    k.onegeom = 1;
    for (const DPair& p : s->pairs) k.onegeom &= (p.gm == s->pairs[0].gm);
    k.static_block = (!tsp && s->count_static && s->static_contacts > 0) ? 1 : 0;
    k.static_cost = tsp ? s->static_cost : 0.0;
    k.upright = (tsp && !generic) ? 1 : 0;
    k.cbup = k.upright;
    for (const DPair& p : s->pairs) {
        const DGeom& g = s->geoms[p.gm];
        const int tg = g.type;
        k.cylbox |= (tg == 5 && p.otype == 6) || (tg == 6 && p.otype == 5);
        // the mover's yaw rotation keeps m[2] = m[5] = m[6] = m[7] = 0 exactly (mover_poses
        // MODE 1, geom_rot_t, matmul3 for a moving partner) when the relative rotations have them
        if (tg == 6 && p.otype == 6)
            k.upright &= (!g.relrot || sspd::upright3(g.mat)) && sspd::upright3(p.omat);
        // cylinder axis vertical (the mover's yaw keeps it so), box upright
        if (tg == 5 && p.otype == 6)
            k.cbup &= (!g.relrot || sspd::cyl_vertical(g.mat)) && sspd::upright3(p.omat);
        if (tg == 6 && p.otype == 5)
            k.cbup &= (!g.relrot || sspd::upright3(g.mat)) && sspd::cyl_vertical(p.omat);
    }
    return k;
}

inline SceneT scene_t(const sspp_scene* s) {
    SceneT t{};
    if (!s) return t;
    t.geoms = s->d_geoms;
    t.pairs = s->d_pairs;
    t.movers = s->d_movers;
    t.visit = s->d_visit;
    return t;
}

struct SsppPtrs {
    const double* ctrl_in;
    double* ctrl_out;
    double* arc;
    unsigned char* feasible;
    sspp_best* best;
    SurvPtrs q;  // the split launch's survivor queue (k.split)
    int* split_used = nullptr;  // out: whether the launch was split (one resident round only)
};

// the job's pair table: sampled candidates use the reachable subset, caller splines the full one
inline SceneT scene_t_job(const sspp_job* j, bool sampled) {
    SceneT t = scene_t(j->scene);
    if (j->d_pairs) { t.pairs = sampled ? j->d_pairs_s : j->d_pairs; t.visit = nullptr; }  // (another order)
    return t;
}
inline KScene kscene_job(const sspp_job* j, bool sampled) {
    KScene k = kscene(j->scene, false);
    if (j->d_pairs) {
        k.npairs = sampled ? j->np_samp : j->np_full;
        k.onegeom = sampled ? j->og_samp : j->og_full;
        k.cylbox = sampled ? j->cb_samp : j->cb_full;
    }
    return k;
}

// the split launch's second kernel: a persistent grid of the chip's resident capacity
// whether a launch of nblk workgroups is one resident round (the split launch's waiting waves
// need every producer resident); the occupancy query is cached per (kernel, LDS)
inline bool c2f_one_round(const sspp_job* j, const void* fn, int nt, int lds, int nblk) {
    static thread_local const void* c_fn = nullptr;
    static thread_local int c_lds = -1, c_wgs = 0, c_dev = -1;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (fn != c_fn || lds != c_lds || dev != c_dev) {
        int per_cu = 0, ncu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, nt, (size_t)lds) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            per_cu = ncu = 0;
        c_fn = fn; c_lds = lds; c_dev = dev; c_wgs = per_cu * ncu;
    }
    (void)j;
    return nblk <= c_wgs;
}

template <int D, int NM, int P, int NT>
hipError_t launch_c2f_nt(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk, hipStream_t st,
                         const SurvPtrs& q) {
    const double* atab = j->d_tab + (size_t)(j->W + 1) * (P + 1);
    const int* aspan = j->d_span + (j->W + 1);
    const SceneT T = scene_t_job(j, !o.ctrl_in);
#define SSPP_LAUNCH_C2F(NMV, OGV, CBV, SPV)                                                               \
    do {                                                                                                  \
        SsppC2F kk = k;                                                                                   \
        kk.split = SPV;                                                                                   \
        if (o.split_used) *o.split_used = SPV;                                                            \
        hipLaunchKernelGGL((k_sspp_c2f<D, NMV, P, OGV, NT, CBV, SPV>), dim3(nblk), dim3(NT), kk.lds, st, kk, T, \
                           j->d_otab, j->d_otab32, j->d_ospan, atab, aspan, j->d_init, j->d_limits, o.ctrl_in,   \
                           o.ctrl_out, o.arc, o.feasible, j->d_part, j->d_sync, o.best, q);              \
    } while (0)
    const bool og = NM == 1 && k.sc.onegeom && k.sc.npairs > 0;
    if (og && k.sc.cylbox) SSPP_LAUNCH_C2F(1, true, true, false);
    else if (og && k.split && c2f_one_round(j, (const void*)k_sspp_c2f<D, 1, P, true, NT, false, true>, NT, k.lds, nblk))
        SSPP_LAUNCH_C2F(1, true, false, true);
    else if (og) SSPP_LAUNCH_C2F(1, true, false, false);
    else if (k.sc.cylbox) SSPP_LAUNCH_C2F(NM, false, true, false);
    else SSPP_LAUNCH_C2F(NM, false, false, false);
#undef SSPP_LAUNCH_C2F
    return hipGetLastError();
}

// three workgroup sizes: one- and two-wave workgroups (throughput shapes) and 4-wave workgroups
// (a single plan() batch, latency shape); DESIGN.md §5
template <int D, int NM, int P>
hipError_t launch_c2f(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk, hipStream_t st) {
    const SurvPtrs q = o.q;
    if (k.nt == 64) return launch_c2f_nt<D, NM, P, 64>(k, j, o, nblk, st, q);
    if (k.nt == 128) return launch_c2f_nt<D, NM, P, 128>(k, j, o, nblk, st, q);
    return launch_c2f_nt<D, NM, P, 256>(k, j, o, nblk, st, q);
}

// ---- per-dof entry points, instantiated one dof per translation unit (sspp_inst.hip, built
// with -DSSPK_D=1..9) so the kernels compile in parallel; the host code (sspp_kernels.hip)
// switches on the job's dof
// the hit census of a sampled job (k_sspp_census): M candidates, every collision waypoint
template <int D, int NM, int P>
hipError_t launch_census(const sspp_job* j, int M, unsigned long long seed, unsigned long long* d_hits,
                         const DPair* pairs, hipStream_t st) {
    const KScene sc = kscene_job(j, true);
    SceneT T = scene_t_job(j, true);
    if (pairs) { T.pairs = pairs; T.visit = nullptr; }  // the asynchronous pre-pass's own copy of the sampled table
    const int r0 = std::min(P, j->n), r1 = std::max(r0, j->n - P);
    const size_t lds = sizeof(double) * ((size_t)j->n * D + (size_t)(r1 - r0) * D + D);
    if (NM == 1 && sc.onegeom && sc.npairs > 0)
        hipLaunchKernelGGL((k_sspp_census<D, 1, P, true>), dim3(M), dim3(kCensusThreads), lds, st, sc, T, j->n, j->W,
                           j->sampler, j->sigma, seed, j->d_tab, j->d_span, j->d_init, j->d_limits, d_hits);
    else
        hipLaunchKernelGGL((k_sspp_census<D, NM, P, false>), dim3(M), dim3(kCensusThreads), lds, st, sc, T, j->n,
                           j->W, j->sampler, j->sigma, seed, j->d_tab, j->d_span, j->d_init, j->d_limits, d_hits);
    return hipGetLastError();
}

// one (dof, degree) per translation unit: sharing a unit with the other degree's kernels changed
// the register allocation of the robocrane kernel (0 -> 275 spilled VGPRs at the same source)
template <int D, int P>
hipError_t entry_c2f_p(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk, hipStream_t st) {
    if (j->nm == 2) {
        if constexpr (D == 9) return launch_c2f<9, 2, P>(k, j, o, nblk, st);
        return hipErrorInvalidValue;
    }
    return launch_c2f<D, 1, P>(k, j, o, nblk, st);
}
template <int D, int P>
hipError_t entry_census_p(const sspp_job* j, int M, unsigned long long seed, unsigned long long* d_hits,
                          const DPair* pairs, hipStream_t st) {
    if (j->nm == 2) {
        if constexpr (D == 9) return launch_census<9, 2, P>(j, M, seed, d_hits, pairs, st);
        return hipErrorInvalidValue;
    }
    return launch_census<D, 1, P>(j, M, seed, d_hits, pairs, st);
}
template <int D>
hipError_t entry_c2f(const SsppC2F& k, const sspp_job* j, const SsppPtrs& o, int nblk, hipStream_t st) {
#ifdef SSPP_DEV_ONLY  // variant builds for experiments: degree 3 only (fast compile)
    if (j->p != 3) return hipErrorInvalidValue;
    return entry_c2f_p<D, 3>(k, j, o, nblk, st);
#else
    return j->p == 3 ? entry_c2f_p<D, 3>(k, j, o, nblk, st) : entry_c2f_p<D, 2>(k, j, o, nblk, st);
#endif
}
template <int D>
hipError_t entry_census(const sspp_job* j, int M, unsigned long long seed, unsigned long long* d_hits,
                        const DPair* pairs, hipStream_t st) {
#ifdef SSPP_DEV_ONLY
    if (j->p != 3) return hipErrorInvalidValue;
    return entry_census_p<D, 3>(j, M, seed, d_hits, pairs, st);
#else
    return j->p == 3 ? entry_census_p<D, 3>(j, M, seed, d_hits, pairs, st)
                     : entry_census_p<D, 2>(j, M, seed, d_hits, pairs, st);
#endif
}

// TaskSpacePlanner evaluation (k_tsp), its own translation unit (SSPK_D = 0)
template <int Unused>
hipError_t entry_tsp(const TspK& k, const sspp_job* j, int nblk, const double* mean, const double* sigma,
                     const double* d_vias, double* d_vias_out, double* d_L, double* d_Cnf, double* d_Cwf,
                     double* d_cost, uint8_t* d_status, sspp_best* d_best, hipStream_t st, int pp) {
    const SceneT tt = scene_t(j->scene);
    if (pp == 2) {  // k_tsp_pp2: k.npg 8-wave workgroups per candidate (nblk = B * npg)
        const size_t lds = sizeof(double) * (size_t)2 * j->n * 4;
#define SSPP_LAUNCH_TSPPP2(OG, CBV)                                                                       \
        hipLaunchKernelGGL((k_tsp_pp2<1, OG, CBV, 8>), dim3(nblk), dim3(512), lds, st, k, tt, j->d_tab,   \
                           j->d_span, j->d_Minv, mean, sigma, d_vias, d_vias_out, d_L, d_Cnf, d_Cwf, d_cost, \
                           d_status, j->d_part, j->d_sync, d_best)
        const bool og = k.sc.onegeom && k.sc.npairs > 0;
        const int cbm = k.sc.cylbox ? (k.sc.cbup ? 2 : 1) : 0;
        if (og && cbm == 1) SSPP_LAUNCH_TSPPP2(true, 1);
        else if (og && cbm == 2) SSPP_LAUNCH_TSPPP2(true, 2);
        else if (og) SSPP_LAUNCH_TSPPP2(true, 0);
        else if (cbm == 1) SSPP_LAUNCH_TSPPP2(false, 1);
        else if (cbm == 2) SSPP_LAUNCH_TSPPP2(false, 2);
        else SSPP_LAUNCH_TSPPP2(false, 0);
#undef SSPP_LAUNCH_TSPPP2
        return hipGetLastError();
    }
    if (pp == 1) {  // k_tsp_pp: one 8-wave workgroup per candidate (cp <= 64, npairs <= 64)
        const size_t lds = sizeof(double) * ((size_t)2 * j->n * 4 + 64 * 64) + 64 * 64;
#define SSPP_LAUNCH_TSPPP(OG, CBV)                                                                       \
        hipLaunchKernelGGL((k_tsp_pp<1, OG, CBV, 8>), dim3(nblk), dim3(512), lds, st, k, tt, j->d_tab,   \
                           j->d_span, j->d_Minv, mean, sigma, d_vias, d_vias_out, d_L, d_Cnf, d_Cwf, d_cost, \
                           d_status, j->d_part, j->d_sync, d_best)
        const bool og = k.sc.onegeom && k.sc.npairs > 0;
        const int cbm = k.sc.cylbox ? (k.sc.cbup ? 2 : 1) : 0;
        if (og && cbm == 1) SSPP_LAUNCH_TSPPP(true, 1);
        else if (og && cbm == 2) SSPP_LAUNCH_TSPPP(true, 2);
        else if (og) SSPP_LAUNCH_TSPPP(true, 0);
        else if (cbm == 1) SSPP_LAUNCH_TSPPP(false, 1);
        else if (cbm == 2) SSPP_LAUNCH_TSPPP(false, 2);
        else SSPP_LAUNCH_TSPPP(false, 0);
#undef SSPP_LAUNCH_TSPPP
        return hipGetLastError();
    }
#define SSPP_LAUNCH_TSP(OG, CBV, UPV, DEFV)                                                             \
    hipLaunchKernelGGL((k_tsp<1, OG, CBV, UPV, DEFV>), dim3(nblk), dim3(kBlock), lds, st, k, tt, j->d_tab, \
                       j->d_span, j->d_Minv, mean, sigma, d_vias, d_vias_out, d_L, d_Cnf, d_Cwf, d_cost, \
                       d_status, j->d_part, j->d_sync, d_best)
    const bool og = k.sc.onegeom && k.sc.npairs > 0;
    const int cbm = k.sc.cylbox ? (k.sc.cbup ? 2 : 1) : 0;
    const bool up = k.sc.upright && cbm != 1;
    // pp == 3: the deferred-polygon form (host-checked: one waypoint per lane, <= kDefPairs pairs);
    // pp == 4: the lane-local deferred polygons (one waypoint per lane, <= 64 pairs)
    const int def = pp == 3 ? 1 : (pp == 4 ? 2 : 0);
    const size_t base = tsp_base_lds(j->cpb, j->n, k.rep);
    const size_t lds = def == 1 ? base + tsp_def_lds(k.sc.npairs) : (def == 2 ? base + tsp_def2_lds(k.sc.npairs) : base);
#define SSPP_LAUNCH_TSP_ALL(DEFV)                                                                         \
    if (og && cbm == 1) SSPP_LAUNCH_TSP(true, 1, false, DEFV);                                            \
    else if (og && cbm == 2) { if (up) SSPP_LAUNCH_TSP(true, 2, true, DEFV); else SSPP_LAUNCH_TSP(true, 2, false, DEFV); } \
    else if (og && up) SSPP_LAUNCH_TSP(true, 0, true, DEFV);                                              \
    else if (og) SSPP_LAUNCH_TSP(true, 0, false, DEFV);                                                   \
    else if (cbm == 1) SSPP_LAUNCH_TSP(false, 1, false, DEFV);                                            \
    else if (cbm == 2) { if (up) SSPP_LAUNCH_TSP(false, 2, true, DEFV); else SSPP_LAUNCH_TSP(false, 2, false, DEFV); } \
    else if (up) SSPP_LAUNCH_TSP(false, 0, true, DEFV);                                                   \
    else SSPP_LAUNCH_TSP(false, 0, false, DEFV);
    if (def == 1) { SSPP_LAUNCH_TSP_ALL(1) }
    else if (def == 2) { SSPP_LAUNCH_TSP_ALL(2) }
    else { SSPP_LAUNCH_TSP_ALL(0) }
#undef SSPP_LAUNCH_TSP_ALL
#undef SSPP_LAUNCH_TSP
    return hipGetLastError();
}

// multi-goal evaluation (k_tsp_group): the k_tsp instantiation entry_tsp picks for mode 0 / 3 / 4
template <int Unused>
hipError_t entry_tsp_group(const TspK& k, const TspGoals& goals, const sspp_job* j, int nblk, hipStream_t st,
                           int mode) {
    const SceneT tt = scene_t(j->scene);
#define SSPP_LAUNCH_TSPG(OG, CBV, UPV, DEFV)                                                            \
    hipLaunchKernelGGL((k_tsp_group<1, OG, CBV, UPV, DEFV>), dim3(nblk), dim3(kBlock), lds, st, k, goals, tt, \
                       j->d_tab, j->d_span, j->d_Minv)
    const bool og = k.sc.onegeom && k.sc.npairs > 0;
    const int cbm = k.sc.cylbox ? (k.sc.cbup ? 2 : 1) : 0;
    const bool up = k.sc.upright && cbm != 1;
    const int def = mode == 3 ? 1 : (mode == 4 ? 2 : 0);
    const size_t base = tsp_base_lds(j->cpb, j->n, k.rep);
    const size_t lds = def == 1 ? base + tsp_def_lds(k.sc.npairs) : (def == 2 ? base + tsp_def2_lds(k.sc.npairs) : base);
#define SSPP_LAUNCH_TSPG_ALL(DEFV)                                                                        \
    if (og && cbm == 1) SSPP_LAUNCH_TSPG(true, 1, false, DEFV);                                           \
    else if (og && cbm == 2) { if (up) SSPP_LAUNCH_TSPG(true, 2, true, DEFV); else SSPP_LAUNCH_TSPG(true, 2, false, DEFV); } \
    else if (og && up) SSPP_LAUNCH_TSPG(true, 0, true, DEFV);                                             \
    else if (og) SSPP_LAUNCH_TSPG(true, 0, false, DEFV);                                                  \
    else if (cbm == 1) SSPP_LAUNCH_TSPG(false, 1, false, DEFV);                                           \
    else if (cbm == 2) { if (up) SSPP_LAUNCH_TSPG(false, 2, true, DEFV); else SSPP_LAUNCH_TSPG(false, 2, false, DEFV); } \
    else if (up) SSPP_LAUNCH_TSPG(false, 0, true, DEFV);                                                  \
    else SSPP_LAUNCH_TSPG(false, 0, false, DEFV);
    if (def == 1) { SSPP_LAUNCH_TSPG_ALL(1) }
    else if (def == 2) { SSPP_LAUNCH_TSPG_ALL(2) }
    else { SSPP_LAUNCH_TSPG_ALL(0) }
#undef SSPP_LAUNCH_TSPG_ALL
#undef SSPP_LAUNCH_TSPG
    return hipGetLastError();
}

#define SSPK_ENTRY_DECL(X, D, P)                                                                          \
    X template hipError_t entry_c2f_p<D, P>(const SsppC2F&, const sspp_job*, const SsppPtrs&, int, hipStream_t); \
    X template hipError_t entry_census_p<D, P>(const sspp_job*, int, unsigned long long, unsigned long long*,   \
                                               const DPair*, hipStream_t);
#define SSPK_TSP_DECL(X)                                                                                  \
    X template hipError_t entry_tsp<0>(const TspK&, const sspp_job*, int, const double*, const double*,    \
                                       const double*, double*, double*, double*, double*, double*, uint8_t*, \
                                       sspp_best*, hipStream_t, int);                                       \
    X template hipError_t entry_tsp_group<0>(const TspK&, const TspGoals&, const sspp_job*, int, hipStream_t, int);

}  // namespace sspk
