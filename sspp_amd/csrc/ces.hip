// ces.hip — tsp::Planner's cross-entropy (CES) iteration on the device (gfx950).
//
// Reference (include/sspp/tsp_planner.h:72-145, tsp_elites.h:13-32, tsp_distribution.h:16-83):
//   seeds = [mean set, forwarded best (iterate && last_best_), samples x Sampler::sample_set]
//   evaluate every seed (k_tsp in CES slot mode, sspp_kernels.hip)
//   successes -> top-k by L + w * C_wf (k = max(1, int(|succ| * elite_fraction)))
//             -> CES log weights -> Distribution::update -> best = min cost -> adapt(true)
//   no success -> adapt(false)
// Everything between two evaluations runs in one workgroup of k_ces_update: no host round
// trip, so a planning loop of many iterations is a chain of asynchronous launches.
//
// Deliberate, documented differences:
//   * candidates are ordered by slot (mean set, forwarded best, samples in Philox order); the
//     reference's order of successes_ depends on OpenMP merge timing.  Ties in
//     the elite sort and the best pick go to the lowest slot.
//   * the weighted sums of Distribution::update and the weight normaliser use the canonical
//     512-lane order (lane j % 512 partials, xor butterfly per wave, waves in order) that
//     oracle/sspp_oracle.c::or_canon_sum restates;
//     the reference sums sequentially (differences ~1e-16 relative).
//   * log(k + 0.5) and log(i + 1) come from host tables (glibc log), so every weight is the
//     reference's value bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "model.h"

namespace {

constexpr int kCesThreads = 512;   // 8 waves: 256 VGPRs per lane, no scratch spills in the serial chain
constexpr int kCesWaves = kCesThreads / 64;
constexpr int kMaxVias = 32;
constexpr int kEliteCap = 8192;  // LDS of k_ces_update: 8192 x (8 B weight + 4 B slot) = 96 KiB

struct CesHdr {
    int nfixed;      // fixed slots (mean set [+ forwarded best]) of the current iteration
    int has_best;    // Planner::last_best_ is set
    int nsucc;       // successes of the last update
    int nelite;      // elites of the last update
    long long best_slot;
    double best_cost;
    long long iter;  // completed updates (informational)
    long long pad;
};

struct CesK {
    int K, nslots, samples, cap;
    double frac, inc, dec, sigma_floor, var_beta, mean_lr, sd_min, sd_max, dist_z_min, z_min;
    double lo[4], hi[4];
};

struct CesReset {
    double mean0[kMaxVias * 4];  // Distribution::reset(mean0) values (z + bound clamps applied)
    double sigma0;               // sigma0_ after the stddev clamps
};

constexpr unsigned long long kNoKey = ~0ull;  // okey() of a NaN; marks "not a success"

// order-preserving map double -> u64 (-0 folded onto +0: IEEE compares them equal)
__device__ __forceinline__ unsigned long long okey(double x) {
    if (x == 0.0) x = 0.0;
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = v + __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ double clamp_sd(double s, const CesK& c) {
    s = s < c.sd_min ? c.sd_min : s;          // cwiseMax(stddev_min)
    s = s > c.sd_max ? c.sd_max : s;          // cwiseMin(stddev_max)
    return s < c.sigma_floor ? c.sigma_floor : s;  // cwiseMax(sigma_floor)
}

// Distribution::wrap_angle_diff (tsp_distribution.h:44-50)
__device__ __forceinline__ double wrap_diff(double a, double b, double mn, double mx) {
    const double range = mx - mn;
    double d = a - b;
    while (d > 0.5 * range) d -= range;
    while (d < -0.5 * range) d += range;
    return d;
}

// canonical block sum (or_canon_sum with kCesThreads = 512 lanes): per-wave xor butterfly, then the wave
// totals in wave order; every thread gets the result
__device__ __forceinline__ double block_sum(double v, double* s_red) {
    v = wave_sum64(v);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = s_red[0];
    for (int w = 1; w < kCesWaves; ++w) t = t + s_red[w];
    __syncthreads();
    return t;
}
__device__ __forceinline__ void block_sum4(double (&v)[4], double* s_red) {
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] = wave_sum64(v[d]);
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < 4; ++d) s_red[d * kCesWaves + (threadIdx.x >> 6)] = v[d];
    __syncthreads();
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        double t = s_red[d * kCesWaves];
        for (int w = 1; w < kCesWaves; ++w) t = t + s_red[d * kCesWaves + w];
        v[d] = t;
    }
    __syncthreads();
}

// plan()'s prologue: reset() (iterate == 0) or keep the distribution, then the iteration's
// fixed seeds: mean set with z >= cfg.z_min (tsp_planner.h:82-84) and the forwarded best.
// Planner::reset's initial mean (tsp_planner.h:54-69 + Distribution::reset, tsp_distribution.h:16-29):
// entry e = 4 i + d of the linear vias, the same operations as sspp_ces_begin's host loop (no
// contraction: ces.hip is built with -ffp-contract=off on both sides)
__host__ __device__ inline double ces_mean0(const CesK& c, int total_points, const double* start, const double* end,
                                            int e) {
    const int i = e >> 2, d = e & 3;
    const double t = (double)(i + 1) / (total_points - 1);
    double v = (1.0 - t) * start[d] + t * end[d];
    if (d == 2) v = v < c.z_min ? c.z_min : v;
    if (d == 2) v = v < c.dist_z_min ? c.dist_z_min : v;
    return v < c.lo[d] ? c.lo[d] : (c.hi[d] < v ? c.hi[d] : v);
}

__device__ __forceinline__ void ces_begin_body(const CesK& c, int iterate, const double* mean0, double sigma0,
                                               CesHdr* h, double* mean, double* sigma, const double* lbest,
                                               double* fixed) {
    const int e = threadIdx.x;
    const int hb = iterate ? h->has_best : 0;
    if (e < c.K * 4) {
        double m = iterate ? mean[e] : mean0[e];
        if (!iterate) { mean[e] = m; sigma[e] = sigma0; }
        const int d = e & 3;
        fixed[e] = (d == 2 && m < c.z_min) ? c.z_min : m;
        fixed[c.K * 4 + e] = lbest[e];
    }
    if (e == 0) {
        if (!iterate) h->has_best = 0;
        h->nfixed = 1 + hb;
        h->nsucc = 0;
        h->nelite = 0;
        h->best_slot = -1;
        h->best_cost = INFINITY;
    }
}
__global__ __launch_bounds__(128) void k_ces_begin(CesK c, int iterate, CesReset r, CesHdr* h,
                                                   double* mean, double* sigma,
                                                   const double* lbest, double* fixed) {
    ces_begin_body(c, iterate, r.mean0, r.sigma0, h, mean, sigma, lbest, fixed);
}

// multi-goal iterations (sspp_ces_plan_group): every goal's device state and buffers, goal g in
// blockIdx.z of each batched launch
constexpr int kMaxCesGoals = 16;
struct CesGoalDev {
    CesHdr* h;
    double *mean, *sigma, *lbest, *fixed;
    unsigned char* status;
    double *cost, *vias, *L, *Cnf, *Cwf;
    int *rank, *by_rank, *nsucc, *elite;
    unsigned char* stage;
    double start[4], end[4];
};
struct CesGroupDev {
    CesGoalDev g[kMaxCesGoals];
};
__global__ __launch_bounds__(128) void k_ces_begin_group(CesK c, int iterate, int total_points, double sigma0,
                                                         CesGroupDev G) {
    const CesGoalDev& q = G.g[blockIdx.z];
    __shared__ double s_m0[kMaxVias * 4];
    if (!iterate && threadIdx.x < c.K * 4) s_m0[threadIdx.x] = ces_mean0(c, total_points, q.start, q.end, threadIdx.x);
    __syncthreads();
    ces_begin_body(c, iterate, s_m0, sigma0, q.h, q.mean, q.sigma, q.lbest, q.fixed);
}

// ---- elite selection by rank counting (three launches, no sort, no host round trip) ----
// The elites are the successes of rank < k in the (cost, slot) order — EliteSelector::select's
// partial_sort with ties to the lowest slot.  Ranks are counted tile against tile
// over the whole chip (k_ces_rank: rank[s] += #{j in key tile : (key_j, j) < (key_s, s)}), then
// each success is scattered to by_rank[rank[s]] (k_ces_scatter).  rank[] and the success
// counter are re-armed by the kernels that consume them (zeroed once at creation).
constexpr int kRankTile = 256;
__device__ __forceinline__ void ces_rank_body(int nslots, const double* __restrict__ cost,
                                              const unsigned char* __restrict__ status, int* rank, int* nsucc) {
    __shared__ unsigned long long s_k[kRankTile];
    const int ts = blockIdx.x, tk = blockIdx.y, tid = threadIdx.x;
    const int j0 = tk * kRankTile, s = ts * kRankTile + tid, j = j0 + tid;
    s_k[tid] = (j < nslots && status[j]) ? okey(cost[j]) : kNoKey;  // kNoKey pads the last tile
    const unsigned long long ks = (s < nslots && status[s]) ? okey(cost[s]) : kNoKey;
    __syncthreads();
    if (tk == 0) {  // success count, one atomic per wave
        const unsigned long long m = __ballot(ks != kNoKey);
        if ((tid & 63) == 0 && m) atomicAdd(nsucc, (int)__popcll(m));
    }
    if (ks == kNoKey) return;
    // (key_j, j) < (key_s, s) over the tile; padding entries (kNoKey) never count because
    // ks < kNoKey.  Entries are LDS broadcasts (every lane reads the same address), unrolled so
    // the reads pipeline.
    int cnt = 0;
    const int d = s - j0;  // entries q < d have a lower slot than s
    if (j0 + kRankTile <= nslots) {
#pragma unroll 16
        for (int q = 0; q < kRankTile; ++q) {
            const unsigned long long kj = s_k[q];
            cnt += (kj < ks) || (kj == ks && q < d);
        }
    } else {  // last, partial tile
        const int jn = nslots - j0;
        for (int q = 0; q < jn; ++q) {
            const unsigned long long kj = s_k[q];
            cnt += (kj < ks) || (kj == ks && q < d);
        }
    }
    if (cnt) atomicAdd(rank + s, cnt);
}
__global__ __launch_bounds__(kRankTile) void k_ces_rank(int nslots, const double* __restrict__ cost,
                                                        const unsigned char* __restrict__ status,
                                                        int* rank, int* nsucc) {
    ces_rank_body(nslots, cost, status, rank, nsucc);
}
__device__ __forceinline__ void ces_scatter_body(int nslots, const double* __restrict__ cost,
                                                 const unsigned char* __restrict__ status, int* rank, int* by_rank) {
    const int s = blockIdx.x * 256 + threadIdx.x;
    if (s >= nslots) return;
    if (status[s] && okey(cost[s]) != kNoKey) by_rank[rank[s]] = s;
    rank[s] = 0;  // re-armed for the next update
}
__global__ __launch_bounds__(256) void k_ces_scatter(int nslots, const double* __restrict__ cost,
                                                     const unsigned char* __restrict__ status,
                                                     int* rank, int* by_rank) {
    ces_scatter_body(nslots, cost, status, rank, by_rank);
}

// Pinned staging layout read by sspp_ces_read: [header, 64 B] [L | C_nf | C_wf | cost : n each]
// [vias n*KD] [mean | sigma | last_best : KD each] (f64) [elites : cap] (i32) [status : n] (u8)
constexpr size_t kStageHdr = 64;
struct StageView {
    double *L, *Cnf, *Cwf, *cost, *vias, *mean, *sigma, *lbest;
    int* elites;
    unsigned char* status;
    CesHdr* hdr;
};
__host__ __device__ inline StageView stage_view(unsigned char* base, int n, int KD, int cap) {
    StageView v;
    v.hdr = (CesHdr*)base;
    double* d = (double*)(base + kStageHdr);
    v.L = d; v.Cnf = d + n; v.Cwf = d + 2 * (size_t)n; v.cost = d + 3 * (size_t)n;
    v.vias = d + 4 * (size_t)n;
    v.mean = v.vias + (size_t)n * KD; v.sigma = v.mean + KD; v.lbest = v.sigma + KD;
    v.elites = (int*)(v.lbest + KD);
    v.status = (unsigned char*)(v.elites + cap);
    return v;
}

// Distribution::update + best pick + adapt on the ranked elites, one workgroup.  With
// fused != 0 (n_slots <= kCesThreads: the ICRA-sized lists) the workgroup ranks the successes
// itself, one slot per thread against every other slot in LDS, so an update is one launch
// instead of rank + scatter + update.
// stage != nullptr: the iteration's results also go straight into sspp_ces_read's pinned staging
// (the values this workgroup writes, from registers; the per-slot results of the evaluation),
// so reading it back needs no staging launch.
__device__ __forceinline__ void ces_update_body(
    const CesK& c, int fused, const unsigned char* __restrict__ status, const double* __restrict__ cost,
    const int* __restrict__ by_rank, int* nsucc_p, const double* __restrict__ vias,
    const double* __restrict__ LT, const double* __restrict__ LH, CesHdr* h, double* mean,
    double* sigma, double* lbest, int* elite_out, const double* __restrict__ Lsl,
    const double* __restrict__ Cnfsl, const double* __restrict__ Cwfsl, unsigned char* stage) {
    __shared__ double s_wt[kEliteCap];
    __shared__ int s_idx[kEliteCap];
    __shared__ double s_red[4 * kCesWaves];
    __shared__ double s_ms[2 * 4 * kMaxVias];  // mean | sigma
    const int tid = threadIdx.x;
    const int K = c.K, KD = 4 * K;
    for (int e = tid; e < 2 * KD; e += kCesThreads) s_ms[e] = e < KD ? mean[e] : sigma[e - KD];
    StageView sv{};
    if (stage) {
        const int n = c.nslots;
        sv = stage_view(stage, n, KD, c.cap);
        for (int e = tid; e < n; e += kCesThreads) {
            sv.L[e] = Lsl[e]; sv.Cnf[e] = Cnfsl[e]; sv.Cwf[e] = Cwfsl[e]; sv.cost[e] = cost[e];
            sv.status[e] = status[e];
        }
        for (int e = tid; e < n * KD; e += kCesThreads) sv.vias[e] = vias[e];
    }
    int nsucc;
    if (fused) {
        unsigned long long* s_key = (unsigned long long*)s_wt;  // dead until the weights
        const int ns = c.nslots;
        const unsigned long long ks = (tid < ns && status[tid]) ? okey(cost[tid]) : kNoKey;
        s_key[tid] = ks;
        nsucc = __syncthreads_count(ks != kNoKey);
        if (ks != kNoKey) {
            int r = 0;
            for (int q = 0; q < ns; ++q) {
                const unsigned long long kj = s_key[q];
                r += (kj < ks) || (kj == ks && q < tid);
            }
            s_idx[r] = tid;
        }
        __syncthreads();
    } else {
        nsucc = *nsucc_p;
    }
    if (nsucc == 0) {  // adapt(false)
        if (tid < KD) {
            const double sg = clamp_sd(sigma[tid] * c.inc, c);
            sigma[tid] = sg;
            if (stage) { sv.sigma[tid] = sg; sv.mean[tid] = mean[tid]; sv.lbest[tid] = lbest[tid]; }
        }
        if (tid == 0) {
            h->nsucc = 0; h->nelite = 0; h->best_slot = -1; h->best_cost = INFINITY;
            const long long it = h->iter + 1;
            h->iter = it;
            if (stage) {
                CesHdr o = {h->nfixed, h->has_best, 0, 0, -1, INFINITY, it, 0};
                *sv.hdr = o;
            }
        }
        return;
    }
    int k = (int)((double)nsucc * c.frac) < 1 ? 1 : (int)((double)nsucc * c.frac);
    if (k > nsucc) k = nsucc;  // frac <= 1 is enforced at creation; never read past the ranks
    if (!fused) {
        for (int j = tid; j < k; j += kCesThreads) s_idx[j] = by_rank[j];
        __syncthreads();
        if (tid == 0) *nsucc_p = 0;  // re-armed for the next update (every thread has read it)
    }

    // ---- CES log weights (tsp_elites.h:24-32): w_j = log(k + 0.5) - log(j + 1), normalised.
    // Every sum below is the canonical 512-lane order of or_canon_sum(x, n, 512): thread t
    // accumulates j = t, t + 512, ... in order, xor butterfly per wave, waves in order.
    const double lk = LH[k];
    double a = 0.0;
    for (int j = tid; j < k; j += kCesThreads) a = a + (lk - LT[j + 1]);
    const double sumw = block_sum(a, s_red);
    for (int j = tid; j < k; j += kCesThreads) s_wt[j] = (lk - LT[j + 1]) / sumw;
    __syncthreads();

    // ---- Distribution::update (tsp_distribution.h:52-83) + adapt(true), via by via: every
    // thread gathers its elites' 4 coordinates once per pass, all 512 lanes reduce
    const bool cache = k <= 2 * kCesThreads;  // each thread's <= 2 elites stay in registers
    for (int v = 0; v < K; ++v) {
        double em[4] = {0.0, 0.0, 0.0, 0.0}, xc0[4], xc1[4];
        int r = 0;
        for (int j = tid; j < k; j += kCesThreads, ++r) {
            const double* x = vias + (long long)s_idx[j] * KD + 4 * v;
            const double w = s_wt[j];
            double xv[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) xv[d] = x[d];
            if (cache) {
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    if (r == 0) xc0[d] = xv[d];
                    else xc1[d] = xv[d];
                }
            }
#pragma unroll
            for (int d = 0; d < 4; ++d) em[d] = em[d] + w * xv[d];
        }
        block_sum4(em, s_red);
        double nm[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const double m0 = s_ms[4 * v + d];
            double t = m0 + c.mean_lr * (em[d] - m0);
            if (d == 2) t = t < c.dist_z_min ? c.dist_z_min : t;
            nm[d] = t < c.lo[d] ? c.lo[d] : (c.hi[d] < t ? c.hi[d] : t);  // std::clamp
        }
        const bool wrap = c.lo[3] != c.hi[3];
        double ve[4] = {0.0, 0.0, 0.0, 0.0};
        r = 0;
        for (int j = tid; j < k; j += kCesThreads, ++r) {
            double xv[4];
            if (cache) {
#pragma unroll
                for (int d = 0; d < 4; ++d) xv[d] = r == 0 ? xc0[d] : xc1[d];
            } else {
                const double* x = vias + (long long)s_idx[j] * KD + 4 * v;
#pragma unroll
                for (int d = 0; d < 4; ++d) xv[d] = x[d];
            }
            const double w = s_wt[j];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const double df = (d == 3 && wrap) ? wrap_diff(xv[3], nm[3], c.lo[3], c.hi[3]) : xv[d] - nm[d];
                ve[d] = ve[d] + w * (df * df);
            }
        }
        block_sum4(ve, s_red);
        if (tid < 4) {
            const int d = tid;
            const double s0 = s_ms[KD + 4 * v + d];
            const double pv = s0 * s0;
            const double blend = (1.0 - c.var_beta) * pv + c.var_beta * ve[d];
            double sg = clamp_sd(sqrt(blend), c);
            sg = clamp_sd(sg * c.dec, c);  // adapt(true)
            mean[4 * v + d] = nm[d];
            sigma[4 * v + d] = sg;
            if (stage) { sv.mean[4 * v + d] = nm[d]; sv.sigma[4 * v + d] = sg; }
        }
    }

    // ---- best = first minimum in slot order (std::min_element): rank 0
    const int b = s_idx[0];
    for (int e = tid; e < KD; e += kCesThreads) {
        const double x = vias[(long long)b * KD + e];
        lbest[e] = x;
        if (stage) sv.lbest[e] = x;
    }
    for (int j = tid; j < k; j += kCesThreads) {
        elite_out[j] = s_idx[j];
        if (stage) sv.elites[j] = s_idx[j];
    }
    if (tid == 0) {
        h->has_best = 1;
        h->nsucc = nsucc;
        h->nelite = k;
        h->best_slot = b;
        h->best_cost = cost[b];
        const long long it = h->iter + 1;
        h->iter = it;
        if (stage) {
            CesHdr o = {h->nfixed, 1, nsucc, k, (long long)b, cost[b], it, 0};
            *sv.hdr = o;
        }
    }
}

__global__ __launch_bounds__(kCesThreads) void k_ces_update(
    CesK c, int fused, const unsigned char* __restrict__ status, const double* __restrict__ cost,
    const int* __restrict__ by_rank, int* nsucc_p, const double* __restrict__ vias,
    const double* __restrict__ LT, const double* __restrict__ LH, CesHdr* h, double* mean,
    double* sigma, double* lbest, int* elite_out, const double* __restrict__ Lsl,
    const double* __restrict__ Cnfsl, const double* __restrict__ Cwfsl, unsigned char* stage) {
    ces_update_body(c, fused, status, cost, by_rank, nsucc_p, vias, LT, LH, h, mean, sigma, lbest, elite_out, Lsl,
                    Cnfsl, Cwfsl, stage);
}
__global__ __launch_bounds__(kRankTile) void k_ces_rank_group(int nslots, CesGroupDev G) {
    const CesGoalDev& q = G.g[blockIdx.z];
    ces_rank_body(nslots, q.cost, q.status, q.rank, q.nsucc);
}
__global__ __launch_bounds__(256) void k_ces_scatter_group(int nslots, CesGroupDev G) {
    const CesGoalDev& q = G.g[blockIdx.z];
    ces_scatter_body(nslots, q.cost, q.status, q.rank, q.by_rank);
}
__global__ __launch_bounds__(kCesThreads) void k_ces_update_group(CesK c, int fused, const double* __restrict__ LT,
                                                                  const double* __restrict__ LH, CesGroupDev G) {
    const CesGoalDev& q = G.g[blockIdx.z];
    ces_update_body(c, fused, q.status, q.cost, q.by_rank, q.nsucc, q.vias, LT, LH, q.h, q.mean, q.sigma, q.lbest,
                    q.elite, q.L, q.Cnf, q.Cwf, q.stage);
}

// Multi-rank exchange: a rank's slots as packed records [L, C_nf, C_wf, cost, status, vias]
__global__ __launch_bounds__(256) void k_ces_pack(int n, int KD, const double* L, const double* Cnf,
                                                  const double* Cwf, const double* cost,
                                                  const unsigned char* st, const double* vias,
                                                  double* out) {
    const int R = 5 + KD;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < (long long)n * R;
         e += (long long)gridDim.x * 256) {
        const int i = (int)(e / R), f = (int)(e - (long long)i * R);
        double v;
        if (f == 0) v = L[i];
        else if (f == 1) v = Cnf[i];
        else if (f == 2) v = Cwf[i];
        else if (f == 3) v = cost[i];
        else if (f == 4) v = (double)st[i];
        else v = vias[(long long)i * KD + (f - 5)];
        out[e] = v;
    }
}
__global__ __launch_bounds__(256) void k_ces_unpack(int n, int KD, const double* in, double* L,
                                                    double* Cnf, double* Cwf, double* cost,
                                                    unsigned char* st, double* vias) {
    const int R = 5 + KD;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < (long long)n * R;
         e += (long long)gridDim.x * 256) {
        const int i = (int)(e / R), f = (int)(e - (long long)i * R);
        const double v = in[e];
        if (f == 0) L[i] = v;
        else if (f == 1) Cnf[i] = v;
        else if (f == 2) Cwf[i] = v;
        else if (f == 3) cost[i] = v;
        else if (f == 4) st[i] = (unsigned char)v;
        else vias[(long long)i * KD + (f - 5)] = v;
    }
}

// sspp_ces_read's staging: header, per-slot results, distribution and elites written straight
// into the planner's pinned host buffer (one launch, then one stream synchronisation)
__global__ __launch_bounds__(256) void k_ces_stage(int n, int KD, int cap, const CesHdr* __restrict__ h,
                                                   const double* L, const double* Cnf, const double* Cwf,
                                                   const double* cost, const double* vias, const double* mean,
                                                   const double* sigma, const double* lbest,
                                                   const int* __restrict__ elite,
                                                   const unsigned char* __restrict__ st,
                                                   unsigned char* out) {
    const long long nv = (long long)n * KD, nd = 4LL * n + nv + 3LL * KD;
    double* od = (double*)(out + kStageHdr);
    int* oi = (int*)(od + nd);
    unsigned char* ob = (unsigned char*)(oi + cap);
    const int nel = h->nelite;
    const long long gid = (long long)blockIdx.x * 256 + threadIdx.x, stride = (long long)gridDim.x * 256;
    if (gid < (long long)(sizeof(CesHdr) / 8))
        ((long long*)out)[gid] = ((const long long*)h)[gid];
    for (long long e = gid; e < nd + cap + n; e += stride) {
        if (e < nd) {
            const double* src;
            long long i = e;
            if (i < 4LL * n) {
                const int f = (int)(i / n);
                src = f == 0 ? L : f == 1 ? Cnf : f == 2 ? Cwf : cost;
                i -= (long long)f * n;
            } else if ((i -= 4LL * n) < nv) {
                src = vias;
            } else {
                i -= nv;
                const int f = (int)(i / KD);
                src = f == 0 ? mean : f == 1 ? sigma : lbest;
                i -= (long long)f * KD;
            }
            od[e] = src[i];
        } else if (e < nd + cap) {
            const int j = (int)(e - nd);
            if (j < nel) oi[j] = elite[j];
        } else {
            ob[e - nd - cap] = st[e - nd - cap];
        }
    }
}

int hip_err(hipError_t e, const char* what) {
    return sspp::set_error(SSPP_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

struct sspp_ces {
    sspp_job* job = nullptr;
    sspp_ces_config cfg{};
    int K = 0, world = 1, spr = 0, nslots = 0, cap = 0;
    long long iter = 0;  // completed evaluations: Philox ids of iteration t start at t * samples
    double lo[4], hi[4];
    double start[4] = {0, 0, 0, 0}, end[4] = {0, 0, 0, 0};
    CesHdr* d_hdr = nullptr;
    double *d_mean = nullptr, *d_sigma = nullptr, *d_lbest = nullptr, *d_fixed = nullptr;
    double *d_L = nullptr, *d_Cnf = nullptr, *d_Cwf = nullptr, *d_cost = nullptr, *d_vias = nullptr;
    unsigned char* d_status = nullptr;
    int* d_elite = nullptr;
    int* d_rank = nullptr;     // [n_slots] rank of each success in the (cost, slot) order
    int* d_by_rank = nullptr;  // [n_slots] slot of rank r
    int* d_nsucc = nullptr;
    double *d_LT = nullptr, *d_LH = nullptr;
    hipStream_t last = nullptr;         // stream of the last enqueued operation (sspp_ces_read waits on it)
    bool mixed = false;                 // operations since the last read used more than one stream
    bool any_op = false;
    unsigned char* h_stage = nullptr;   // pinned: k_ces_stage's output
    size_t stage_bytes = 0;
    long long staged_iter = -1;         // iteration whose results k_ces_update already staged
    int fused = 1;                      // SSPP_OPT_CES_FUSED (sspp_ces_set_option)
};

// every enqueuing entry point notes its stream: sspp_ces_read waits on the last one, or on the
// whole device when the operations since the previous read were spread over several streams
static void note_stream(sspp_ces* p, hipStream_t s) {
    if (p->any_op && s != p->last) p->mixed = true;
    p->any_op = true;
    p->last = s;
}

static CesK ces_k(const sspp_ces* p) {
    CesK c{};
    c.K = p->K; c.nslots = p->nslots; c.samples = p->cfg.samples; c.cap = p->cap;
    c.frac = p->cfg.elite_fraction; c.inc = p->cfg.inc; c.dec = p->cfg.dec;
    c.sigma_floor = p->cfg.sigma_floor; c.var_beta = p->cfg.var_beta; c.mean_lr = p->cfg.mean_lr;
    c.sd_min = p->cfg.stddev_min; c.sd_max = p->cfg.stddev_max;
    c.dist_z_min = p->cfg.dist_z_min; c.z_min = p->cfg.z_min;
    for (int i = 0; i < 4; ++i) { c.lo[i] = p->lo[i]; c.hi[i] = p->hi[i]; }
    return c;
}

extern "C" {

int sspp_ces_set_option(sspp_ces* p, int key, int64_t value) {
    sspp::clear_error();
    if (!p) return sspp::set_error(SSPP_E_INVAL, "null planner");
    if (key == SSPP_OPT_CES_FUSED) {
        p->fused = value ? 1 : 0;
        return SSPP_OK;
    }
    return sspp::set_error(SSPP_E_INVAL, "unknown option");
}

void sspp_ces_free(sspp_ces* p) {
    if (!p) return;
    if (p->job) sspp_job_free(p->job);
    for (void* q : {(void*)p->d_hdr, (void*)p->d_mean, (void*)p->d_sigma, (void*)p->d_lbest,
                    (void*)p->d_fixed, (void*)p->d_L, (void*)p->d_Cnf, (void*)p->d_Cwf,
                    (void*)p->d_cost, (void*)p->d_vias, (void*)p->d_status, (void*)p->d_elite,
                    (void*)p->d_LT, (void*)p->d_LH, (void*)p->d_rank, (void*)p->d_by_rank,
                    (void*)p->d_nsucc})
        if (q) (void)hipFree(q);
    if (p->h_stage) (void)hipHostFree(p->h_stage);
    delete p;
}

int sspp_ces_create(const sspp_scene* scene, const sspp_ces_config* cfg, int world, sspp_ces** out) {
    sspp::clear_error();
    if (!scene || !cfg || !out || !cfg->lo || !cfg->hi)
        return sspp::set_error(SSPP_E_INVAL, "sspp_ces_create: null argument");
    const int K = cfg->total_points - 2;
    if (K < 1 || K > kMaxVias)
        return sspp::set_error(SSPP_E_INVAL, "total_points must be in [3, 34] (1..32 via points)");
    if (cfg->samples < 0 || cfg->checks < 1) return sspp::set_error(SSPP_E_INVAL, "samples >= 0, checks >= 1");
    if (world < 1) return sspp::set_error(SSPP_E_INVAL, "world must be >= 1");
    // tsp_elites.h:15-19 partial_sorts the first max(1, int(n * frac)) of n candidates: frac > 1
    // would sort past the end (undefined behaviour in the reference), so it is rejected here
    if (!(cfg->elite_fraction >= 0.0 && cfg->elite_fraction <= 1.0))
        return sspp::set_error(SSPP_E_INVAL, "elite_fraction must be in [0, 1]");
    const long long maxslots = (long long)cfg->samples + 2;
    long long cap = (long long)((double)maxslots * cfg->elite_fraction);
    if (cap < 1) cap = 1;
    if (cap > kEliteCap)
        return sspp::set_error(SSPP_E_UNSUPPORTED, "(sample_count + 2) * elite_fraction exceeds 8192 elites");
    auto* p = new sspp_ces();
    p->cfg = *cfg;
    p->cfg.lo = p->cfg.hi = nullptr;
    p->K = K; p->world = world; p->cap = (int)cap;
    for (int i = 0; i < 4; ++i) { p->lo[i] = cfg->lo[i]; p->hi[i] = cfg->hi[i]; }
    p->spr = (int)((maxslots + world - 1) / world);
    p->nslots = p->spr * world;
    std::vector<double> zeros(4 * K, 0.0), start(4, 0.0);
    sspp_tsp_args a{};
    a.start = start.data(); a.end = start.data(); a.n_vias = K; a.check_points = cfg->checks;
    a.w_collision = cfg->w_collision; a.mean = zeros.data(); a.sigma = zeros.data();
    a.lo = p->lo; a.hi = p->hi; a.z_min = cfg->z_min; a.seed = cfg->seed;
    a.floor_z_min = cfg->floor_z_min; a.floor_margin = cfg->floor_margin; a.floor_scale = cfg->floor_scale;
    int rc = sspp_job_create_tsp(scene, &a, p->spr, &p->job);
    if (rc) { delete p; return rc; }
    const size_t ns = (size_t)p->nslots, kd = (size_t)4 * K;
    std::vector<double> LT(cap + 2), LH(cap + 2);
    for (long long m = 0; m <= cap + 1; ++m) {
        LT[m] = m ? std::log((double)m) : 0.0;            // log(i + 1.0), i = m - 1
        LH[m] = std::log((double)m + 0.5);                // log(k + 0.5)
    }
    hipError_t e;
    if ((e = hipMalloc((void**)&p->d_hdr, sizeof(CesHdr))) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_mean, sizeof(double) * kd)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_sigma, sizeof(double) * kd)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_lbest, sizeof(double) * kd)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_fixed, sizeof(double) * 2 * kd)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_L, sizeof(double) * ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_Cnf, sizeof(double) * ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_Cwf, sizeof(double) * ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_cost, sizeof(double) * ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_vias, sizeof(double) * ns * kd)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_status, ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_elite, sizeof(int) * cap)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_rank, sizeof(int) * ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_by_rank, sizeof(int) * ns)) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_nsucc, sizeof(int))) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_LT, sizeof(double) * LT.size())) != hipSuccess ||
        (e = hipMalloc((void**)&p->d_LH, sizeof(double) * LH.size())) != hipSuccess ||
        (e = hipMemcpy(p->d_LT, LT.data(), sizeof(double) * LT.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->d_LH, LH.data(), sizeof(double) * LH.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemset(p->d_hdr, 0, sizeof(CesHdr))) != hipSuccess ||
        (e = hipMemset(p->d_lbest, 0, sizeof(double) * kd)) != hipSuccess ||
        (e = hipMemset(p->d_mean, 0, sizeof(double) * kd)) != hipSuccess ||
        (e = hipMemset(p->d_sigma, 0, sizeof(double) * kd)) != hipSuccess ||
        (e = hipMemset(p->d_status, 0, ns)) != hipSuccess ||
        (e = hipMemset(p->d_rank, 0, sizeof(int) * ns)) != hipSuccess ||
        (e = hipMemset(p->d_by_rank, 0, sizeof(int) * ns)) != hipSuccess ||
        (e = hipMemset(p->d_nsucc, 0, sizeof(int))) != hipSuccess ||
        (p->stage_bytes = kStageHdr + sizeof(double) * (4 * ns + ns * kd + 3 * kd) + sizeof(int) * (size_t)cap + ns,
         (e = hipHostMalloc((void**)&p->h_stage, p->stage_bytes, hipHostMallocDefault)) != hipSuccess)) {
        rc = hip_err(e, "sspp_ces_create allocation");
        sspp_ces_free(p);
        return rc;
    }
    *out = p;
    return SSPP_OK;
}

int sspp_ces_get_info(const sspp_ces* p, sspp_ces_info* out) {
    if (!p || !out) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_get_info: null argument");
    out->n_vias = p->K;
    out->n_slots = p->nslots;
    out->slots_per_rank = p->spr;
    out->world = p->world;
    out->elite_capacity = p->cap;
    out->iteration = p->iter;
    return SSPP_OK;
}

int sspp_ces_begin(sspp_ces* p, const double* start, const double* end, int iterate, void* stream) {
    sspp::clear_error();
    if (!p || !start || !end) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_begin: null argument");
    for (int i = 0; i < 4; ++i) { p->start[i] = start[i]; p->end[i] = end[i]; }
    CesReset r{};
    if (!iterate) {
        // Planner::reset (tsp_planner.h:54-69): linear vias, z >= cfg.z_min, then
        // Distribution::reset (tsp_distribution.h:16-29): z >= dist.z_min, bounds, sigma clamps
        const int n = p->cfg.total_points;
        for (int i = 0; i < p->K; ++i) {
            const double t = (double)(i + 1) / (n - 1);
            for (int d = 0; d < 4; ++d) {
                double v = (1.0 - t) * start[d] + t * end[d];
                if (d == 2) v = v < p->cfg.z_min ? p->cfg.z_min : v;
                if (d == 2) v = v < p->cfg.dist_z_min ? p->cfg.dist_z_min : v;
                v = v < p->lo[d] ? p->lo[d] : (p->hi[d] < v ? p->hi[d] : v);
                r.mean0[4 * i + d] = v;
            }
        }
        double s = p->cfg.sigma0;
        s = s < p->cfg.stddev_min ? p->cfg.stddev_min : s;
        s = s > p->cfg.stddev_max ? p->cfg.stddev_max : s;
        s = s < p->cfg.sigma_floor ? p->cfg.sigma_floor : s;
        r.sigma0 = s;
    }
    note_stream(p, (hipStream_t)stream);
    p->staged_iter = -1;
    hipLaunchKernelGGL(k_ces_begin, dim3(1), dim3(128), 0, (hipStream_t)stream, ces_k(p), iterate ? 1 : 0,
                       r, p->d_hdr, p->d_mean, p->d_sigma, p->d_lbest, p->d_fixed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_err(e, "k_ces_begin launch");
    return SSPP_OK;
}

int sspp_ces_eval(sspp_ces* p, int rank, void* stream) {
    sspp::clear_error();
    if (!p || rank < 0 || rank >= p->world) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_eval: bad rank");
    sspp::TspCesEval ev{};
    ev.fixed = p->d_fixed; ev.nfixed = &p->d_hdr->nfixed;
    ev.mean = p->d_mean; ev.sigma = p->d_sigma;
    ev.slot0 = (long long)rank * p->spr;
    ev.samples = p->cfg.samples;
    ev.first_id = p->iter * (long long)p->cfg.samples;
    for (int i = 0; i < 4; ++i) { ev.start[i] = p->start[i]; ev.end[i] = p->end[i]; }
    const size_t o = (size_t)rank * p->spr;
    note_stream(p, (hipStream_t)stream);
    p->staged_iter = -1;
    return sspp::tsp_eval_ces(p->job, &ev, p->spr, p->d_L + o, p->d_Cnf + o, p->d_Cwf + o,
                              p->d_status + o, p->d_cost + o, p->d_vias + o * 4 * p->K, stream);
}

int sspp_ces_update(sspp_ces* p, void* stream) {
    sspp::clear_error();
    if (!p) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_update: null planner");
    const int nt = (p->nslots + kRankTile - 1) / kRankTile;
    hipStream_t st = (hipStream_t)stream;
    note_stream(p, st);
    const int fused = p->nslots <= kCesThreads && p->fused;
    if (!fused) {
        hipLaunchKernelGGL(k_ces_rank, dim3(nt, nt), dim3(kRankTile), 0, st, p->nslots, p->d_cost,
                           p->d_status, p->d_rank, p->d_nsucc);
        hipLaunchKernelGGL(k_ces_scatter, dim3(nt), dim3(256), 0, st, p->nslots, p->d_cost, p->d_status,
                           p->d_rank, p->d_by_rank);
    }
    // small lists: the update also fills sspp_ces_read's pinned staging (no staging launch)
    unsigned char* stage = fused ? p->h_stage : nullptr;
    hipLaunchKernelGGL(k_ces_update, dim3(1), dim3(kCesThreads), 0, st, ces_k(p), fused, p->d_status,
                       p->d_cost, p->d_by_rank, p->d_nsucc, p->d_vias, p->d_LT, p->d_LH, p->d_hdr, p->d_mean,
                       p->d_sigma, p->d_lbest, p->d_elite, p->d_L, p->d_Cnf, p->d_Cwf, stage);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_err(e, "k_ces_update launch");
    p->iter++;
    p->staged_iter = stage ? p->iter : -1;
    return SSPP_OK;
}

int sspp_ces_plan(sspp_ces* p, const double* start, const double* end, int iterate, int iterations,
                  void* stream) {
    if (!p || iterations < 1) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_plan: bad argument");
    if (p->world != 1) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_plan: multi-rank planners step eval/update themselves");
    for (int t = 0; t < iterations; ++t) {
        int rc = sspp_ces_begin(p, start, end, (t > 0 || iterate) ? 1 : 0, stream);
        if (rc) return rc;
        if ((rc = sspp_ces_eval(p, 0, stream))) return rc;
        if ((rc = sspp_ces_update(p, stream))) return rc;
    }
    return SSPP_OK;
}

// Several planners' iterations as one chain of batched launches: per iteration one
// k_ces_begin_group, one k_tsp_group over every goal's slots, then k_ces_rank_group /
// k_ces_scatter_group (lists above kCesThreads) and one k_ces_update_group — 3-5 launches for all
// goals instead of 3-5 per goal, and the goals' evaluations share the chip instead of following
// one another.  Each planner's state, buffers, seed and Philox ids are its own, so every result
// equals sspp_ces_plan on that planner alone (test_ces_plan_group_matches_single).  The planners
// must share the evaluation (scene, vias, checks, bounds, costs) and the CES configuration; a
// group that does not, or whose slot lists are small enough for the pair-split evaluation, runs
// goal by goal (sspp_ces_plan on each, same results).
int sspp_ces_plan_group(sspp_ces* const* ps, int G, const double* starts, const double* ends, int iterate,
                        int iterations, void* stream) {
    sspp::clear_error();
    if (!ps || !starts || !ends || G < 1 || iterations < 1)
        return sspp::set_error(SSPP_E_INVAL, "sspp_ces_plan_group: bad argument");
    const sspp_ces* p0 = ps[0];
    for (int g = 0; g < G; ++g)
        if (!ps[g] || ps[g]->world != 1)
            return sspp::set_error(SSPP_E_INVAL, "sspp_ces_plan_group: single-rank planners only");
    const CesK c0 = ces_k(p0);
    bool same = G <= kMaxCesGoals;
    for (int g = 1; g < G && same; ++g) {
        const CesK c = ces_k(ps[g]);
        same = std::memcmp(&c, &c0, sizeof c) == 0 && ps[g]->cfg.total_points == p0->cfg.total_points &&
               ps[g]->cfg.sigma0 == p0->cfg.sigma0 && ps[g]->fused == p0->fused;
        for (int h = 0; h < g && same; ++h) same = ps[h] != ps[g];
    }
    hipStream_t st = (hipStream_t)stream;
    auto one_by_one = [&]() {
        for (int g = 0; g < G; ++g) {
            int rc = sspp_ces_plan(ps[g], starts + 4 * g, ends + 4 * g, iterate, iterations, stream);
            if (rc) return rc;
        }
        return (int)SSPP_OK;
    };
    if (!same) return one_by_one();
    double s0 = p0->cfg.sigma0;  // the sigma clamps of sspp_ces_begin
    s0 = s0 < p0->cfg.stddev_min ? p0->cfg.stddev_min : s0;
    s0 = s0 > p0->cfg.stddev_max ? p0->cfg.stddev_max : s0;
    s0 = s0 < p0->cfg.sigma_floor ? p0->cfg.sigma_floor : s0;
    CesGroupDev gd{};
    std::vector<sspp_job*> jobs(G);
    std::vector<sspp::TspCesEval> evs(G);
    std::vector<sspp::TspCesOut> outs(G);
    for (int g = 0; g < G; ++g) {
        sspp_ces* p = ps[g];
        CesGoalDev& q = gd.g[g];
        q.h = p->d_hdr; q.mean = p->d_mean; q.sigma = p->d_sigma; q.lbest = p->d_lbest; q.fixed = p->d_fixed;
        q.status = p->d_status; q.cost = p->d_cost; q.vias = p->d_vias; q.L = p->d_L; q.Cnf = p->d_Cnf;
        q.Cwf = p->d_Cwf; q.rank = p->d_rank; q.by_rank = p->d_by_rank; q.nsucc = p->d_nsucc; q.elite = p->d_elite;
        for (int i = 0; i < 4; ++i) {
            q.start[i] = p->start[i] = starts[4 * g + i];
            q.end[i] = p->end[i] = ends[4 * g + i];
        }
        jobs[g] = p->job;
        sspp::TspCesEval& e = evs[g];
        e.fixed = p->d_fixed; e.nfixed = &p->d_hdr->nfixed; e.mean = p->d_mean; e.sigma = p->d_sigma;
        e.slot0 = 0; e.samples = p->cfg.samples;
        for (int i = 0; i < 4; ++i) { e.start[i] = p->start[i]; e.end[i] = p->end[i]; }
        outs[g] = sspp::TspCesOut{p->d_L, p->d_Cnf, p->d_Cwf, p->d_cost, p->d_vias, p->d_status};
    }
    const int n = p0->nslots;
    const int fused = n <= kCesThreads && p0->fused;
    const int nt = (n + kRankTile - 1) / kRankTile;
    for (int t = 0; t < iterations; ++t) {
        for (int g = 0; g < G; ++g) {
            sspp_ces* p = ps[g];
            note_stream(p, st);
            p->staged_iter = -1;
            evs[g].first_id = p->iter * (long long)p->cfg.samples;
            gd.g[g].stage = fused ? p->h_stage : nullptr;
        }
        hipLaunchKernelGGL(k_ces_begin_group, dim3(1, 1, G), dim3(128), 0, st, c0, (t > 0 || iterate) ? 1 : 0,
                           p0->cfg.total_points, s0, gd);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_err(e, "k_ces_begin_group launch");
        int rc = sspp::tsp_eval_ces_group(jobs.data(), evs.data(), outs.data(), G, n, stream);
        if (rc == SSPP_E_UNSUPPORTED && t == 0) {
            // the evaluation cannot be batched: this iteration's begin ran for every goal, so
            // finish it goal by goal, then the remaining iterations likewise
            sspp::clear_error();
            for (int g = 0; g < G; ++g) {
                if ((rc = sspp_ces_eval(ps[g], 0, stream)) || (rc = sspp_ces_update(ps[g], stream))) return rc;
                if (iterations > 1 && (rc = sspp_ces_plan(ps[g], starts + 4 * g, ends + 4 * g, 1, iterations - 1, stream)))
                    return rc;
            }
            return SSPP_OK;
        }
        if (rc) return rc;
        if (!fused) {
            hipLaunchKernelGGL(k_ces_rank_group, dim3(nt, nt, G), dim3(kRankTile), 0, st, n, gd);
            hipLaunchKernelGGL(k_ces_scatter_group, dim3(nt, 1, G), dim3(256), 0, st, n, gd);
        }
        hipLaunchKernelGGL(k_ces_update_group, dim3(1, 1, G), dim3(kCesThreads), 0, st, c0, fused, p0->d_LT,
                           p0->d_LH, gd);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_err(e, "k_ces_update_group launch");
        for (int g = 0; g < G; ++g) {
            ps[g]->iter++;
            ps[g]->staged_iter = fused ? ps[g]->iter : -1;
        }
    }
    return SSPP_OK;
}

int sspp_ces_pack(const sspp_ces* p, int rank, double* d_out, void* stream) {
    sspp::clear_error();
    if (!p || !d_out || rank < 0 || rank >= p->world) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_pack: bad argument");
    const size_t o = (size_t)rank * p->spr;
    const int KD = 4 * p->K;
    const long long tot = (long long)p->spr * (5 + KD);
    const int g = (int)std::min<long long>((tot + 255) / 256, 1024);
    hipLaunchKernelGGL(k_ces_pack, dim3(g), dim3(256), 0, (hipStream_t)stream, p->spr, KD, p->d_L + o,
                       p->d_Cnf + o, p->d_Cwf + o, p->d_cost + o, p->d_status + o, p->d_vias + o * KD, d_out);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SSPP_OK : hip_err(e, "k_ces_pack launch");
}

int sspp_ces_unpack(sspp_ces* p, const double* d_in, void* stream) {
    sspp::clear_error();
    if (!p || !d_in) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_unpack: bad argument");
    const int KD = 4 * p->K;
    const long long tot = (long long)p->nslots * (5 + KD);
    const int g = (int)std::min<long long>((tot + 255) / 256, 1024);
    note_stream(p, (hipStream_t)stream);
    p->staged_iter = -1;
    hipLaunchKernelGGL(k_ces_unpack, dim3(g), dim3(256), 0, (hipStream_t)stream, p->nslots, KD, d_in,
                       p->d_L, p->d_Cnf, p->d_Cwf, p->d_cost, p->d_status, p->d_vias);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SSPP_OK : hip_err(e, "k_ces_unpack launch");
}

int sspp_ces_get_buffers(const sspp_ces* p, sspp_ces_buffers* out) {
    if (!p || !out) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_get_buffers: null argument");
    out->L = p->d_L; out->C_nf = p->d_Cnf; out->C_wf = p->d_Cwf; out->cost = p->d_cost;
    out->status = p->d_status; out->vias = p->d_vias;
    out->mean = p->d_mean; out->sigma = p->d_sigma; out->last_best = p->d_lbest;
    out->elites = p->d_elite;
    return SSPP_OK;
}

int sspp_ces_read(sspp_ces* p, sspp_ces_state* st, double* L, double* Cnf, double* Cwf, double* cost,
                  uint8_t* status, double* vias, double* mean, double* sigma, double* last_best,
                  int32_t* elites) {
    sspp::clear_error();
    if (!p || !st) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_read: null argument");
    // one staging launch behind the planner's last operation (none when the last update staged
    // its iteration itself), one wait on that stream — preceded by a device-wide wait when the
    // operations since the previous read ran on more than one stream (the staging must see them
    // all, and the earlier streams may be gone by now: the device wait needs none of them)
    const int n = p->nslots, KD = 4 * p->K;
    hipError_t e = hipSuccess;
    if (p->mixed) {
        e = hipDeviceSynchronize();
        if (e != hipSuccess) return hip_err(e, "sspp_ces_read");
        p->mixed = false;
    }
    if (p->staged_iter != p->iter) {
        const long long tot = 4LL * n + (long long)n * KD + 3LL * KD + p->cap + n;
        const int g = (int)std::min<long long>((tot + 255) / 256, 256);
        hipLaunchKernelGGL(k_ces_stage, dim3(g), dim3(256), 0, p->last, n, KD, p->cap, p->d_hdr, p->d_L,
                           p->d_Cnf, p->d_Cwf, p->d_cost, p->d_vias, p->d_mean, p->d_sigma, p->d_lbest,
                           p->d_elite, p->d_status, p->h_stage);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(p->last);
    if (e != hipSuccess) return hip_err(e, "sspp_ces_read");
    // everything enqueued so far has completed: the next operation starts a new record, so a
    // read's stream differing from the next operation's does not count as mixed (which would
    // make the next read wait on the whole device, other planners' streams included)
    p->any_op = false;
    p->mixed = false;
    CesHdr h;
    std::memcpy(&h, p->h_stage, sizeof h);
    st->n_fixed = h.nfixed;
    st->n_candidates = h.nfixed + p->cfg.samples;
    st->n_success = h.nsucc;
    st->n_elite = h.nelite;
    st->has_best = h.has_best;
    st->best_slot = h.best_slot;
    st->best_cost = h.best_cost;
    st->iteration = p->iter;
    const size_t m = (size_t)st->n_candidates, kd = (size_t)KD;
    const double* sd = (const double*)(p->h_stage + kStageHdr);
    const size_t ov = 4 * (size_t)n, om = ov + (size_t)n * kd, oe = om + 3 * kd;
    const int32_t* si = (const int32_t*)(sd + oe);
    const uint8_t* sb = (const uint8_t*)(si + p->cap);
    struct { void* dst; const void* src; size_t bytes; } cp[] = {
        {L, sd, 8 * m}, {Cnf, sd + n, 8 * m}, {Cwf, sd + 2 * (size_t)n, 8 * m}, {cost, sd + 3 * (size_t)n, 8 * m},
        {status, sb, m}, {vias, sd + ov, 8 * m * kd}, {mean, sd + om, 8 * kd},
        {sigma, sd + om + kd, 8 * kd}, {last_best, sd + om + 2 * kd, 8 * kd},
        {elites, si, sizeof(int32_t) * (size_t)(h.nelite > 0 ? h.nelite : 0)}};
    for (auto& c : cp)
        if (c.dst && c.bytes) std::memcpy(c.dst, c.src, c.bytes);
    return SSPP_OK;
}

int sspp_ces_set_state(sspp_ces* p, const double* mean, const double* sigma, const double* last_best,
                       int has_best) {
    sspp::clear_error();
    if (!p) return sspp::set_error(SSPP_E_INVAL, "sspp_ces_set_state: null planner");
    p->staged_iter = -1;  // the staged copy no longer matches the device state
    const size_t kd = (size_t)4 * p->K;
    hipError_t e;
    if ((mean && (e = hipMemcpy(p->d_mean, mean, 8 * kd, hipMemcpyHostToDevice)) != hipSuccess) ||
        (sigma && (e = hipMemcpy(p->d_sigma, sigma, 8 * kd, hipMemcpyHostToDevice)) != hipSuccess) ||
        (last_best && (e = hipMemcpy(p->d_lbest, last_best, 8 * kd, hipMemcpyHostToDevice)) != hipSuccess))
        return hip_err(e, "sspp_ces_set_state copy");
    if (has_best >= 0) {
        CesHdr h;
        if ((e = hipMemcpy(&h, p->d_hdr, sizeof h, hipMemcpyDeviceToHost)) != hipSuccess ||
            (h.has_best = has_best, (e = hipMemcpy(p->d_hdr, &h, sizeof h, hipMemcpyHostToDevice)) != hipSuccess))
            return hip_err(e, "sspp_ces_set_state header");
    }
    return SSPP_OK;
}

}  // extern "C"
