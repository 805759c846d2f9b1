// sspp_kernels.hip — host side of the MI355X scorer: scenes, jobs, launches and the C ABI.
//
// The kernels are in sspp_kern.h; their instantiations are compiled per dof in sspp_inst.hip.
#include "sspp_kern.h"

#include <chrono>
#include <random>

using namespace sspk;

#ifndef SSPP_SINGLE_TU
namespace sspk {
SSPK_ENTRY_DECL(extern, 1, 2)
SSPK_ENTRY_DECL(extern, 1, 3)
SSPK_ENTRY_DECL(extern, 2, 2)
SSPK_ENTRY_DECL(extern, 2, 3)
SSPK_ENTRY_DECL(extern, 3, 2)
SSPK_ENTRY_DECL(extern, 3, 3)
SSPK_ENTRY_DECL(extern, 4, 2)
SSPK_ENTRY_DECL(extern, 4, 3)
SSPK_ENTRY_DECL(extern, 6, 2)
SSPK_ENTRY_DECL(extern, 6, 3)
SSPK_ENTRY_DECL(extern, 7, 2)
SSPK_ENTRY_DECL(extern, 7, 3)
SSPK_ENTRY_DECL(extern, 9, 2)
SSPK_ENTRY_DECL(extern, 9, 3)
SSPK_TSP_DECL(extern)
}  // namespace sspk
#endif

namespace sspk {
constexpr int kArgminThreads = 1024;
__global__ __launch_bounds__(kArgminThreads) void k_argmin(const BlockBest* __restrict__ part,
                                                           int nparts, sspp_best* out) {
    __shared__ double sc[kArgminThreads / 64];
    __shared__ long long si[kArgminThreads / 64], sn[kArgminThreads / 64], sl[kArgminThreads / 64];
    double bc = INFINITY;
    long long bi = -1, cnt = 0, lost = 0;  // lost: the records' `reserved` (lost survivors), summed
    for (int i = threadIdx.x; i < nparts; i += kArgminThreads) {
        const BlockBest b = part[i];
        cnt += b.count;
        lost += b.pad;
        if (better(b.cost, b.idx, bc, bi)) { bc = b.cost; bi = b.idx; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double oc = __shfl_xor(bc, off, 64);
        const long long oi = __shfl_xor(bi, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
        lost += __shfl_xor(lost, off, 64);
        if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sc[w] = bc; si[w] = bi; sn[w] = cnt; sl[w] = lost; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double c = sc[0];
        long long i = si[0], n = sn[0], l = sl[0];
        for (int k = 1; k < kArgminThreads / 64; ++k) {
            n += sn[k];
            l += sl[k];
            if (better(sc[k], si[k], c, i)) { c = sc[k]; i = si[k]; }
        }
        out->cost = i < 0 ? INFINITY : c;
        out->index = i;
        out->count = n;
        out->reserved = l;
    }
}

}  // namespace sspk

// =============================================================== host side: scene + jobs
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
        fill_f32(dg);
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
        fill_f32(dp);
        s->pairs.push_back(dp);
    }
    for (size_t i = 0; i < mover_bodies.size(); ++i) {
        DMover mv{};
        mv.qpos_adr = m->body_qpos_adr[mover_bodies[i]];
        for (int k = 0; k < 7; ++k) mv.qpos0[k] = m->qpos0[mv.qpos_adr + k];
        s->movers.push_back(mv);
    }
    // the pair visit order of the record-form pair loops (SceneT::visit): grouped by moving geom,
    // the reference's order within a group; only for tables a mask word can cover
    std::vector<DPair> visit;
    if (!s->pairs.empty() && s->pairs.size() <= 64) {
        std::vector<int> ix(s->pairs.size());
        for (size_t i = 0; i < ix.size(); ++i) ix[i] = (int)i;
        std::stable_sort(ix.begin(), ix.end(), [&](int x, int y) { return s->pairs[x].gm < s->pairs[y].gm; });
        for (int i : ix) {
            DPair q = s->pairs[i];
            q.pad = i;  // its record index
            visit.push_back(q);
        }
    }
    int rc;
    if ((rc = upload(&s->d_geoms, s->geoms.data(), s->geoms.size())) ||
        (rc = upload(&s->d_pairs, s->pairs.data(), s->pairs.size())) ||
        (rc = upload(&s->d_movers, s->movers.data(), s->movers.size())) ||
        (rc = upload(&s->d_visit, visit.data(), visit.size()))) {
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
    sspp::planner_cache_drop(s);
    if (s->d_geoms) (void)hipFree(s->d_geoms);
    if (s->d_pairs) (void)hipFree(s->d_pairs);
    if (s->d_movers) (void)hipFree(s->d_movers);
    if (s->d_visit) (void)hipFree(s->d_visit);
    delete s;
}

}  // extern "C"

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
// every prefix is spread evenly over the path.
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

// Hit order of a sampled job (sigma > 0).  checkCollision's answer is an OR over
// (waypoint, pair), so the order of both is free; k_sspp_c2f's phase 1 tests a prefix of the
// waypoint order and stops a candidate at its first touching pair, so the waypoints and pairs
// that settle the most sampled candidates should come first.  The orders only steer the scans,
// never their results.
//
// Waypoints: the GPU census (k_sspp_census) of kCensus candidates of the job's own distribution
// (an independent Philox seed) gives, per candidate, the collision waypoints in contact.  The
// first n1 waypoints (phase 1 tests them together) are the n1-set leaving the fewest candidates
// untouched: a greedy set improved by single swaps until no swap helps; then, greedily, the
// waypoint that settles the most candidates not yet settled (up to kPick in all), the rest in
// bisection order.
constexpr int kCensus = 2048, kPick = 12;
static void waypoints_from_census(const std::vector<uint64_t>& hits, int M, int W, int n1, std::vector<int>& wps) {
    const int nw = (W + 64) >> 6, npts = W + 1, mw = (M + 63) / 64;
    // per waypoint: the candidates in contact there, as bits
    std::vector<uint64_t> col((size_t)npts * mw, 0ull);
    for (int m = 0; m < M; ++m)
        for (int i = 0; i < npts; ++i)
            if ((hits[(size_t)m * nw + (i >> 6)] >> (i & 63)) & 1ull) col[(size_t)i * mw + (m >> 6)] |= 1ull << (m & 63);
    auto untouched = [&](const std::vector<int>& S) {
        int c = 0;
        for (int w = 0; w < mw; ++w) {
            uint64_t acc = 0ull;
            for (int i : S) acc |= col[(size_t)i * mw + w];
            const uint64_t valid = (w == mw - 1 && (M & 63)) ? ((1ull << (M & 63)) - 1ull) : ~0ull;
            c += __builtin_popcountll(~acc & valid);
        }
        return c;
    };
    n1 = std::max(1, std::min(n1, npts));
    std::vector<int> S;
    for (int r = 0; r < n1; ++r) {  // greedy
        int bi = -1, bc = M + 1;
        for (int i = 0; i < npts; ++i) {
            if (std::find(S.begin(), S.end(), i) != S.end()) continue;
            S.push_back(i);
            const int c = untouched(S);
            S.pop_back();
            if (c < bc) { bc = c; bi = i; }
        }
        S.push_back(bi);
    }
    int cur = untouched(S);
    for (int pass = 0; pass < 16; ++pass) {  // single swaps
        int bpos = -1, bi = -1, bc = cur;
        for (int pos = 0; pos < n1; ++pos) {
            const int keep = S[pos];
            for (int i = 0; i < npts; ++i) {
                if (std::find(S.begin(), S.end(), i) != S.end()) continue;
                S[pos] = i;
                const int c = untouched(S);
                if (c < bc) { bc = c; bpos = pos; bi = i; }
            }
            S[pos] = keep;
        }
        if (bpos < 0) break;
        S[bpos] = bi;
        cur = bc;
    }
    std::vector<int> order = S;
    while ((int)order.size() < kPick && (int)order.size() < npts) {  // greedy continuation
        int bi = -1, bc = untouched(order);
        for (int i = 0; i < npts; ++i) {
            if (std::find(order.begin(), order.end(), i) != order.end()) continue;
            order.push_back(i);
            const int c = untouched(order);
            order.pop_back();
            if (c < bc) { bc = c; bi = i; }
        }
        if (bi < 0) break;
        order.push_back(bi);
    }
    std::vector<char> taken(npts, 0);
    for (int i : order) taken[i] = 1;
    for (int w : wps) if (!taken[w]) order.push_back(w);
    wps.swap(order);
}

// Pairs: M host-sampled candidates of the job's distribution (host normals), the pairs each
// touches at the phase-1 waypoints `pick`; greedily the pair that settles the most candidates not
// yet settled, the rest in their previous order.
static void pairs_by_hits(const sspp_scene* sc, std::vector<DPair>& pairs, const double* knots, int nknots, int p,
                          const double* ctrl0, int D, double sigma, const double* limits, int W,
                          const std::vector<int>& pick) {
    const int np = (int)pairs.size(), n = nknots - p - 1, nm = (int)sc->movers.size();
    if (np < 2 || np > 64 || nm < 1 || nm > kMaxMovers || pick.empty()) return;
    constexpr int M = 256;
    std::mt19937_64 rng(0x5EEDull);
    std::normal_distribution<double> N01(0.0, 1.0);
    std::vector<uint64_t> cand(M, 0ull);
    std::vector<double> c((size_t)n * D);
    for (int m = 0; m < M; ++m) {
        for (size_t e = 0; e < c.size(); ++e) c[e] = ctrl0[e];
        for (int jj = p; jj < n - p; ++jj)
            for (int d = 0; d < D; ++d) c[(size_t)jj * D + d] += sigma * N01(rng) * limits[d];
        for (int w : pick) {
            const double u = (double)w / W;
            const int sp = span_of(u, p, knots, nknots);
            double N[kMaxP + 1];
            basis_funcs(u, p, sp, knots, N);
            double q[16] = {0};
            for (int d = 0; d < D && d < 16; ++d) {
                double acc = 0.0;
                for (int r = 0; r <= p; ++r) {
                    const int jj = sp - p + r;
                    if (jj >= 0 && jj < n) acc += N[r] * c[(size_t)jj * D + d];
                }
                q[d] = acc;
            }
            double mp[kMaxMovers][3], mR[kMaxMovers][9];
            for (int mv = 0; mv < nm; ++mv) {
                double qp[7];
                for (int k = 0; k < 7; ++k) qp[k] = (7 * mv + k < D) ? q[7 * mv + k] : sc->movers[mv].qpos0[k];
                normalize4(qp + 3);
                quat2mat(qp + 3, mR[mv]);
                for (int k = 0; k < 3; ++k) mp[mv][k] = qp[k];
            }
            for (int k = 0; k < np; ++k) {
                if ((cand[m] >> k) & 1ull) continue;
                const DPair& pr = pairs[k];
                const DGeom& G = sc->geoms[pr.gm];
                const int mv = G.mover > 0 ? G.mover : 0;
                double gp[3], gm[9], t3[3], op[3], om[9];
                matvec3(mR[mv], G.pos, t3);
                for (int d = 0; d < 3; ++d) gp[d] = mp[mv][d] + t3[d];
                if (G.relrot) matmul3(mR[mv], G.mat, gm);
                else for (int e = 0; e < 9; ++e) gm[e] = mR[mv][e];
                if (pr.omover >= 0) {
                    matvec3(mR[pr.omover], pr.opos, t3);
                    for (int d = 0; d < 3; ++d) op[d] = mp[pr.omover][d] + t3[d];
                    matmul3(mR[pr.omover], pr.omat, om);
                } else {
                    for (int d = 0; d < 3; ++d) op[d] = pr.opos[d];
                    for (int e = 0; e < 9; ++e) om[e] = pr.omat[e];
                }
                if (G.rbound > 0.0 && pr.orbound > 0.0) {  // the bounding-sphere test
                    const double dx = op[0] - gp[0], dy = op[1] - gp[1], dz = op[2] - gp[2];
                    const double thr = G.rbound + pr.orbound + pr.margin;
                    if (dx * dx + dy * dy + dz * dz > thr * thr) continue;
                }
                int nd = 0;
                const bool gfirst = (G.type < pr.otype) || (G.type == pr.otype && G.orig < pr.oorig);
                const int nc = gfirst ? collide<false>(G.type, gp, gm, G.size, pr.otype, op, om, pr.osize, pr.margin, &nd)
                                      : collide<false>(pr.otype, op, om, pr.osize, G.type, gp, gm, G.size, pr.margin, &nd);
                if (nc > 0) cand[m] |= 1ull << k;
            }
        }
    }
    std::vector<char> used(np, 0), settled(M, 0);
    std::vector<DPair> out;
    for (;;) {
        int best = -1, bc = 0;
        for (int k = 0; k < np; ++k) {
            if (used[k]) continue;
            int cnt = 0;
            for (int m = 0; m < M; ++m) cnt += !settled[m] && ((cand[m] >> k) & 1ull);
            if (cnt > bc) { bc = cnt; best = k; }
        }
        if (best < 0) break;
        used[best] = 1;
        out.push_back(pairs[best]);
        for (int m = 0; m < M; ++m) if ((cand[m] >> best) & 1ull) settled[m] = 1;
    }
    for (int k = 0; k < np; ++k) if (!used[k]) out.push_back(pairs[k]);
    pairs.swap(out);
}

// Pairs a SAMPLED candidate can reach (job-level broadphase, exact).  sampleWithNoise moves
// control point (j, d), j in [p, n - p), by (sigma z) limits(d) with |z| <= 8.5722 (FP64
// Box-Muller: u1 >= 2^-53) or 5.7683 (FP32 quads: u1 >= 2^-24); every other control point is the
// initial spline's.  A B-spline lies in the convex hull of its control points, so every waypoint
// of every candidate puts the mover root inside the AABB of the initial control points grown by
// those bounds, and a pair pair_may_touch rejects for that box (the moving geom's reach covers
// any rotation) has no contact for any candidate of the job: it is dropped from the sample-mode
// pair table (scored caller splines, sspp_job_score_ctrl, keep the full table).
static std::vector<DPair> reachable_pairs(const sspp_scene* sc, const std::vector<DPair>& in,
                                          const double* init_ctrl, int n, int D, int p, double sigma,
                                          const double* limits, int sampler) {
    const double zmax = (sampler ? 5.8 : 8.6) * (1.0 + 1e-9);
    const int nm = (int)sc->movers.size();
    double lo[kMaxMovers][3], hi[kMaxMovers][3];
    for (int m = 0; m < nm && m < kMaxMovers; ++m)
        for (int d = 0; d < 3; ++d) {
            const int col = 7 * m + d;
            if (col >= D) { lo[m][d] = hi[m][d] = sc->movers[m].qpos0[d]; continue; }
            double a = init_ctrl[col], b = a;
            for (int jj = 0; jj < n; ++jj) {
                const double v = init_ctrl[jj * D + col];
                const double r = (jj >= p && jj < n - p) ? std::fabs(sigma) * zmax * std::fabs(limits[col]) : 0.0;
                a = std::min(a, v - r);
                b = std::max(b, v + r);
            }
            lo[m][d] = a - 1e-9;
            hi[m][d] = b + 1e-9;
        }
    std::vector<DPair> out;
    for (const DPair& pr : in) {
        const DGeom& G = sc->geoms[pr.gm];
        const int m = (nm > 1 && G.mover == 1) ? 1 : 0;
        if (pair_may_touch(pr, G, lo[m], hi[m])) out.push_back(pr);
    }
    return out;
}

static void table_flags(const sspp_scene* sc, const std::vector<DPair>& t, int* np, int* cb, int* og) {
    *np = (int)t.size();
    *cb = 0;
    *og = 1;
    for (const DPair& pr : t) {
        const int tg = sc->geoms[pr.gm].type;
        *cb |= (tg == 5 && pr.otype == 6) || (tg == 6 && pr.otype == 5);
        *og &= pr.gm == t[0].gm;
    }
}

// Basis rows for a list of parameters (same A2.1/A2.2 code as the device header).
// d_tab32 (optional): the same rows rounded to FP32 (k_sspp_c2f's filtered scan)
static int upload_basis(const std::vector<double>& us, int p, const double* knots, int nknots,
                        double** d_tab, int** d_span, float** d_tab32 = nullptr) {
    std::vector<double> tab(us.size() * (p + 1));
    std::vector<int> sp(us.size());
    for (size_t i = 0; i < us.size(); ++i) {
        sp[i] = span_of(us[i], p, knots, nknots);
        basis_funcs(us[i], p, sp[i], knots, &tab[i * (p + 1)]);
    }
    int rc = upload(d_tab, tab.data(), tab.size());
    if (rc) return rc;
    if (d_tab32) {
        std::vector<float> t32(tab.begin(), tab.end());
        if ((rc = upload(d_tab32, t32.data(), t32.size()))) return rc;
    }
    return upload(d_span, sp.data(), sp.size());
}

// the throughput shape: 2-wave workgroups of 32 candidates x 4 phase-1 lanes (DESIGN.md §5:
// against one-wave workgroups of 16, a survivor's remaining waypoints spread over 128 lanes)
constexpr int kThroughputNT = 128, kThroughputG1 = 4;

// both pair tables to the device, synchronously (job creation, option changes)
static int upload_pairs_sync(sspp_job* j) {
    const sspp_scene* sc = j->scene;
    const size_t cap = sizeof(DPair) * std::max<size_t>(1, sc->pairs.size());
    if (!j->d_pairs) HIPCHK(hipMalloc((void**)&j->d_pairs, cap));
    if (!j->d_pairs_s) HIPCHK(hipMalloc((void**)&j->d_pairs_s, cap));
    HIPCHK(hipMemcpy(j->d_pairs, j->h_pairs.data(), sizeof(DPair) * j->h_pairs.size(), hipMemcpyHostToDevice));
    if (!j->h_pairs_s.empty())
        HIPCHK(hipMemcpy(j->d_pairs_s, j->h_pairs_s.data(), sizeof(DPair) * j->h_pairs_s.size(), hipMemcpyHostToDevice));
    return SSPP_OK;
}

// the hit census (k_sspp_census) of M candidates into d (hit bits [M][ceil((W + 1) / 64)]), on
// stream st; pairs: the sampled table to scan (nullptr: the job's)
static hipError_t launch_census_d(sspp_job* j, int M, unsigned long long* d, const DPair* pairs, hipStream_t st) {
    const unsigned long long seed = j->seed ^ 0xC3A5C85C97CB3127ull;  // independent of the job's candidates
    switch (j->D) {
#ifndef SSPP_DEV_ONLY
        case 1: return entry_census<1>(j, M, seed, d, pairs, st);
        case 2: return entry_census<2>(j, M, seed, d, pairs, st);
        case 3: return entry_census<3>(j, M, seed, d, pairs, st);
        case 4: return entry_census<4>(j, M, seed, d, pairs, st);
        case 6: return entry_census<6>(j, M, seed, d, pairs, st);
        case 9: return entry_census<9>(j, M, seed, d, pairs, st);
#endif
        case 7: return entry_census<7>(j, M, seed, d, pairs, st);
    }
    return hipErrorInvalidValue;
}

// the census, synchronously: hit bits to the host
static int run_census(sspp_job* j, int M, std::vector<uint64_t>& hits) {
    const int nw = (j->W + 64) >> 6;
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc((void**)&d, sizeof(unsigned long long) * (size_t)M * nw));
    hipError_t e = launch_census_d(j, M, d, nullptr, nullptr);
    hits.assign((size_t)M * nw, 0ull);
    if (e == hipSuccess) e = hipMemcpy(hits.data(), d, sizeof(uint64_t) * hits.size(), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "k_sspp_census");
    return SSPP_OK;
}

// The census scans every collision waypoint of kCensus candidates: above this many waypoints the
// pre-pass would cost more than it saves, and the job keeps the gap / bisection order
constexpr int kCensusMaxPts = 4097;

// The job's scan orders for its initial spline / sigma / limits: the pair table ordered by the
// mean-path gap (pairs_for_job), refined with the collision-waypoint order by the hit-order
// pre-pass (order 2: sampled jobs at creation), and its sample-mode subset (reachable_pairs).
// create: the waypoint order and both tables are (re)uploaded synchronously; otherwise the pair
// tables are queued on `stream` from the pinned staging at byte offset `pin_off` (the caller
// sized it for both) and the waypoint order stays.
static int set_job_tables(sspp_job* j, const double* init_ctrl, double sigma, const double* limits, int order,
                          bool create, void* stream, size_t pin_off = 0) {
    const sspp_scene* sc = j->scene;
    std::vector<int> wps = c2f_order(j->W);
    if (sc && !sc->pairs.empty()) {
        j->h_pairs = order == 0 ? sc->pairs : pairs_for_job(sc, j->h_knots.data(), j->nknots, j->p, init_ctrl, j->D);
        j->h_pairs_s = reachable_pairs(sc, j->h_pairs, init_ctrl, j->n, j->D, j->p, sigma, limits, j->sampler);
        table_flags(sc, j->h_pairs, &j->np_full, &j->cb_full, &j->og_full);
        table_flags(sc, j->h_pairs_s, &j->np_samp, &j->cb_samp, &j->og_samp);
        if (order == 2 && create && !j->h_pairs_s.empty() && j->W + 1 <= kCensusMaxPts) {
            // the census scans the sampled table in gap order; then both orders, and the
            // sampled table again (reachable_pairs keeps the order it is given)
            const auto t0 = std::chrono::steady_clock::now();
            int rc = upload_pairs_sync(j);
            if (rc) return rc;
            std::vector<uint64_t> hits;
            if ((rc = run_census(j, kCensus, hits))) return rc;
            waypoints_from_census(hits, kCensus, j->W, kThroughputG1, wps);
            const std::vector<int> pick(wps.begin(), wps.begin() + std::min<size_t>(wps.size(), kThroughputG1));
            pairs_by_hits(sc, j->h_pairs, j->h_knots.data(), j->nknots, j->p, init_ctrl, j->D, sigma, limits, j->W,
                          pick);
            j->h_pairs_s = reachable_pairs(sc, j->h_pairs, init_ctrl, j->n, j->D, j->p, sigma, limits, j->sampler);
            table_flags(sc, j->h_pairs, &j->np_full, &j->cb_full, &j->og_full);
            table_flags(sc, j->h_pairs_s, &j->np_samp, &j->cb_samp, &j->og_samp);
            j->prepass_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
    }
    j->pair_order = order;
    if (create) {
        j->wp_order = order == 2 ? 2 : 0;
        j->h_wps = wps;
        std::vector<double> uo;
        for (int i : wps) uo.push_back((double)i / j->W);
        if (j->d_otab) { (void)hipFree(j->d_otab); j->d_otab = nullptr; }
        if (j->d_otab32) { (void)hipFree(j->d_otab32); j->d_otab32 = nullptr; }
        if (j->d_ospan) { (void)hipFree(j->d_ospan); j->d_ospan = nullptr; }
        int rc = upload_basis(uo, j->p, j->h_knots.data(), j->nknots, &j->d_otab, &j->d_ospan, &j->d_otab32);
        if (rc) return rc;
    }
    if (!sc || sc->pairs.empty()) return SSPP_OK;
    const size_t bytes = sizeof(DPair) * j->h_pairs.size(), bytes_s = sizeof(DPair) * j->h_pairs_s.size();
    if (create) return upload_pairs_sync(j);
    if (pin_off + bytes + bytes_s > j->h_pin_bytes) return sspp::set_error(SSPP_E_NOMEM, "pair staging too small");
    hipStream_t st = (hipStream_t)stream;
    unsigned char* pa = j->h_pin + pin_off;
    std::memcpy(pa, j->h_pairs.data(), bytes);
    std::memcpy(pa + bytes, j->h_pairs_s.data(), bytes_s);
    HIPCHK(hipMemcpyAsync(j->d_pairs, pa, bytes, hipMemcpyHostToDevice, st));
    if (bytes_s) HIPCHK(hipMemcpyAsync(j->d_pairs_s, pa + bytes, bytes_s, hipMemcpyHostToDevice, st));
    return SSPP_OK;
}

// k_sspp_c2f dynamic LDS bytes for cpb candidates of nrd own doubles each
static size_t c2f_lds(const sspp_job* j, int cpb, int nrd) {
    const int nm = j->nm < 1 ? 1 : j->nm;
    const int rbox = std::max(6 * nm, lanes_for(j->W - 1) / 64 + 1);
    return sizeof(double) * ((size_t)j->n * j->D + (size_t)cpb * (nrd + rbox) + j->D) +
           sizeof(unsigned long long) * cpb + sizeof(int) * (3 * cpb + 1) +
           sizeof(float) * ((size_t)j->n * j->D + (size_t)cpb * nrd);  // the FP32 copies
}

// The FP32 filter's certified margin for a pair table (sspp_filter.h): FP32's error
// on a separation grows with the pair's extent (centre distance and box extents are bounded by
// the two bounding radii plus the margin for every pair that passes the sphere test), about 6e-5 m
// per metre of extent; eps = 2e-4 m per metre, at least 2e-4.  0 (filter off) past 64 pairs or
// for pairs larger than 8 m, where the certified range would not be worth it.
constexpr double kF32EpsPerMetre = 2e-4;
constexpr float kF32PosLimit = 8.0f;
static double f32_eps(const sspp_scene* sc, const std::vector<DPair>& t) {
    if (!sc || t.empty() || t.size() > 64) return 0.0;
    double S = 1.0;
    for (const DPair& pr : t) {
        const DGeom& G = sc->geoms[pr.gm];
        // the moving geom's offset from its mover's root scales the FP32 pose error like an extent
        double gofs = 0.0, far = 0.0;
        for (int k = 0; k < 3; ++k) gofs += G.pos[k] * G.pos[k];
        gofs = std::sqrt(gofs);
        const double ext = G.rbound + pr.orbound + pr.margin + gofs;
        for (int k = 0; k < 3; ++k) far = std::max(far, std::fabs(pr.opos[k]));
        if (!(ext <= 8.0) || !(far <= 2.0 * kF32PosLimit) || G.rbound <= 0.0) return 0.0;
        S = std::max(S, ext);
    }
    return kF32EpsPerMetre * S;
}

// The asynchronous pre-pass (sspp::job_create_sspp_async): the census on the job's own stream
// (scanning its own copy of the sampled table), its hit bits into pinned memory, then a host
// thread orders the waypoints and pairs exactly as the synchronous creation does.  The thread
// touches only its copies and the job's pre_* result fields, published by prepass_state = 2.
static int prepass_start(sspp_job* j, const double* init_ctrl, double sigma, const double* limits) {
    const sspp_scene* sc = j->scene;
    if (!sc || j->h_pairs_s.empty() || j->W + 1 > kCensusMaxPts) return SSPP_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const int M = kCensus, nw = (j->W + 64) >> 6;
    const size_t nh = (size_t)M * nw;
    j->pre_stream = (hipStream_t)sspp::shared_stream(1);  // shared by every job's pre-pass, not owned
    if (!j->pre_stream) return sspp::set_error(SSPP_E_HIP, "hipStreamCreate (shared pre-pass stream)");
    HIPCHK(hipEventCreateWithFlags(&j->pre_ev, hipEventDisableTiming));
    HIPCHK(hipMalloc((void**)&j->d_hits, sizeof(unsigned long long) * nh));
    HIPCHK(hipHostMalloc((void**)&j->h_hits, sizeof(unsigned long long) * nh, hipHostMallocDefault));
    HIPCHK(hipMalloc((void**)&j->d_census_pairs, sizeof(DPair) * j->h_pairs_s.size()));
    HIPCHK(hipMemcpy(j->d_census_pairs, j->h_pairs_s.data(), sizeof(DPair) * j->h_pairs_s.size(), hipMemcpyHostToDevice));
    hipError_t e = launch_census_d(j, M, j->d_hits, j->d_census_pairs, j->pre_stream);
    if (e == hipSuccess) e = hipMemcpyAsync(j->h_hits, j->d_hits, sizeof(unsigned long long) * nh, hipMemcpyDeviceToHost, j->pre_stream);
    if (e == hipSuccess) e = hipEventRecord(j->pre_ev, j->pre_stream);
    if (e != hipSuccess) return hip_fail(e, "k_sspp_census (asynchronous pre-pass)");
    struct Copies {
        std::vector<double> knots, init, limits;
        std::vector<DPair> pairs;
        double sigma;
        int gen;
    };
    Copies c{j->h_knots, std::vector<double>(init_ctrl, init_ctrl + (size_t)j->n * j->D),
             std::vector<double>(limits, limits + j->D), j->h_pairs, sigma, j->tables_gen};
    j->prepass_state.store(1, std::memory_order_relaxed);
    j->prepass_thread = std::thread([j, sc, c = std::move(c), t0, M, nh]() mutable {
        if (hipEventSynchronize(j->pre_ev) != hipSuccess) {
            j->prepass_state.store(3, std::memory_order_release);
            return;
        }
        std::vector<uint64_t> hits(j->h_hits, j->h_hits + nh);
        std::vector<int> wps = c2f_order(j->W);
        waypoints_from_census(hits, M, j->W, kThroughputG1, wps);
        const std::vector<int> pick(wps.begin(), wps.begin() + std::min<size_t>(wps.size(), kThroughputG1));
        pairs_by_hits(sc, c.pairs, c.knots.data(), j->nknots, j->p, c.init.data(), j->D, c.sigma, c.limits.data(), j->W,
                      pick);
        j->pre_pairs_s = reachable_pairs(sc, c.pairs, c.init.data(), j->n, j->D, j->p, c.sigma, c.limits.data(), j->sampler);
        j->pre_pairs = std::move(c.pairs);
        j->pre_wps = std::move(wps);
        j->pre_gen = c.gen;
        j->pre_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        j->prepass_state.store(2, std::memory_order_release);
    });
    return SSPP_OK;
}

// Swap in the pre-pass's orders, once it has landed (called before each launch; never waits).  The
// waypoint order suits any values; the pair tables are the creation's reachable subset, so they are
// taken only when no update has re-derived the tables since.  Replaced device tables are retired,
// not freed: launches on other streams may still read them.
static void prepass_apply(sspp_job* j) {
    if (j->prepass_state.load(std::memory_order_acquire) != 2) return;
    j->prepass_thread.join();
    j->prepass_state.store(3, std::memory_order_relaxed);
    std::vector<double> uo;
    for (int i : j->pre_wps) uo.push_back((double)i / j->W);
    double* ot = nullptr;
    float* ot32 = nullptr;
    int* os = nullptr;
    if (upload_basis(uo, j->p, j->h_knots.data(), j->nknots, &ot, &os, &ot32) == SSPP_OK) {
        j->retired.insert(j->retired.end(), {(void*)j->d_otab, (void*)j->d_otab32, (void*)j->d_ospan});
        j->d_otab = ot; j->d_otab32 = ot32; j->d_ospan = os;
        j->h_wps = j->pre_wps;
        j->wp_order = 2;
    } else {
        sspp::clear_error();
        for (void* q : {(void*)ot, (void*)ot32, (void*)os}) if (q) (void)hipFree(q);
    }
    if (j->pre_gen == j->tables_gen && j->scene) {
        const size_t cap = sizeof(DPair) * std::max<size_t>(1, j->scene->pairs.size());
        DPair *dp = nullptr, *dps = nullptr;
        if (hipMalloc((void**)&dp, cap) == hipSuccess && hipMalloc((void**)&dps, cap) == hipSuccess &&
            hipMemcpy(dp, j->pre_pairs.data(), sizeof(DPair) * j->pre_pairs.size(), hipMemcpyHostToDevice) == hipSuccess &&
            (j->pre_pairs_s.empty() ||
             hipMemcpy(dps, j->pre_pairs_s.data(), sizeof(DPair) * j->pre_pairs_s.size(), hipMemcpyHostToDevice) == hipSuccess)) {
            j->retired.insert(j->retired.end(), {(void*)j->d_pairs, (void*)j->d_pairs_s});
            j->d_pairs = dp; j->d_pairs_s = dps;
            j->h_pairs = j->pre_pairs; j->h_pairs_s = j->pre_pairs_s;
            table_flags(j->scene, j->h_pairs, &j->np_full, &j->cb_full, &j->og_full);
            table_flags(j->scene, j->h_pairs_s, &j->np_samp, &j->cb_samp, &j->og_samp);
            j->pair_order = 2;
        } else {
            if (dp) (void)hipFree(dp);
            if (dps) (void)hipFree(dps);
        }
    }
    j->prepass_ms = j->pre_ms;
}

// wait for a running pre-pass and drop its result (option changes, job free)
static void prepass_drop(sspp_job* j) {
    if (j->prepass_thread.joinable()) j->prepass_thread.join();
    j->prepass_state.store(3, std::memory_order_relaxed);
}

static int job_create_sspp_impl(const sspp_scene* scene, const sspp_sspp_args* a, int64_t max_batch,
                                sspp_job** out, bool async_prepass);

extern "C" int sspp_job_create_sspp(const sspp_scene* scene, const sspp_sspp_args* a, int64_t max_batch,
                         sspp_job** out) {
    return job_create_sspp_impl(scene, a, max_batch, out, false);
}

int sspp::job_create_sspp_async(const sspp_scene* scene, const sspp_sspp_args* a, int64_t max_batch, sspp_job** out) {
    return job_create_sspp_impl(scene, a, max_batch, out, true);
}

static int job_create_sspp_impl(const sspp_scene* scene, const sspp_sspp_args* a, int64_t max_batch,
                                sspp_job** out, bool async_prepass) {
    sspp::clear_error();
    const auto t_create = std::chrono::steady_clock::now();
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
    j->sampler = a->sampler ? 1 : 0;
    j->h_knots.assign(a->knots, a->knots + j->nknots);
    j->nm = scene ? (int)scene->movers.size() : 1;
    if (j->nm < 1) j->nm = 1;
    j->lpc = lanes_for(W - 1);
    // the worst-case launch footprint (caller splines: n x D doubles per candidate, plus the
    // shared initial spline, hull boxes and flags) must fit the latency shape's 4 candidates in
    // 64 KiB of LDS, or a later sspp_job_score_ctrl could not launch
    if (c2f_lds(j, 4, n * D) > 64 * 1024) {
        delete j;
        return sspp::set_error(SSPP_E_UNSUPPORTED, "problem too large for LDS (n_ctrl x dof)");
    }
    int rc;
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
    j->h_stage.assign(a->init_ctrl, a->init_ctrl + (size_t)n * D);
    j->h_stage.insert(j->h_stage.end(), a->limits, a->limits + D);
    // hit order only for jobs that sample (sigma > 0): a scoring job's candidates are the caller's
    const int order = a->sigma != 0.0 ? 2 : 1;
    if ((rc = set_job_tables(j, a->init_ctrl, a->sigma, a->limits, async_prepass ? 1 : order, true, nullptr)) ||
        (async_prepass && order == 2 && (rc = prepass_start(j, a->init_ctrl, a->sigma, a->limits)))) {
        sspp_job_free(j);
        return rc;
    }
    // one BlockBest per workgroup and step (grown per launch when a shape needs more)
    const int64_t nrec = std::max<int64_t>(64, (max_batch + 3) / 4);
    j->part_cap = nrec;
    if (hipMalloc((void**)&j->d_part, sizeof(BlockBest) * nrec) != hipSuccess ||
        hipMalloc((void**)&j->d_sync, sizeof(ArgminSync) * kMaxSteps) != hipSuccess ||
        hipMemset(j->d_sync, 0, sizeof(ArgminSync) * kMaxSteps) != hipSuccess) {
        sspp_job_free(j);
        return sspp::set_error(SSPP_E_NOMEM, "hipMalloc block partials");
    }
    j->create_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_create).count();
    *out = j;
    return SSPP_OK;
}

// k_sspp_c2f launch shape (NT threads, G1 phase-1 lanes per candidate, 64 / G1 candidates per
// wave), measured on MI355X: launches of many candidates are throughput-bound ->
// 2-wave workgroups of 32 candidates x 4 lanes; a launch of a few thousand (one plan() batch)
// is latency-bound -> 4-wave workgroups of 4 candidates x 64 lanes: a whole wave per candidate in
// phase 1, a survivor's remaining waypoints over 256 lanes in phase 2.  Forced shapes
// (sspp_job_set_option) are for tests and tuning.
static void c2f_shape(const sspp_job* j, int64_t cands, int* nt, int* g1) {
    const bool lat = cands < 16384;
    *nt = j->opt_nt ? j->opt_nt : (lat ? 256 : kThroughputNT);
    *g1 = j->opt_g1 ? j->opt_g1 : (lat ? 64 : kThroughputG1);
}


// Split launches from this many candidates per launch (the throughput shape's range): below it
// a launch is one plan() batch, whose workgroups are few enough to finish their own survivors
constexpr int64_t kSplitMinCands = 16384;

// the survivor queue of split launches: header (counters re-armed by each launch's last
// workgroup), ready words, the survivors' rows and the argmin list, for `cands` slots of `nrd`
// own doubles each
static int survq_reserve(sspp_job* j, int64_t cands, int nrd) {
    if (!j->d_sq_hdr) {
        SurvQ h{};
        for (int s = 0; s < kMaxSteps; ++s) h.bestbits[s] = 0x7FF0000000000000ull;  // +inf
        HIPCHK(hipMalloc((void**)&j->d_sq_hdr, sizeof(SurvQ)));
        HIPCHK(hipMemcpy(j->d_sq_hdr, &h, sizeof(SurvQ), hipMemcpyHostToDevice));
    }
    if (cands <= j->sq_cap && nrd == j->sq_nrd) return SSPP_OK;
    HIPCHK(hipDeviceSynchronize());  // earlier launches may still use the old buffers
    for (void* p : {(void*)j->d_sq_rec, (void*)j->d_sq_ctrl, (void*)j->d_sq_ctrl32, (void*)j->d_sq_res,
                    (void*)j->d_sq_orphan})
        if (p) (void)hipFree(p);
    j->d_sq_rec = nullptr; j->d_sq_ctrl = nullptr; j->d_sq_ctrl32 = nullptr; j->d_sq_res = nullptr;
    j->d_sq_orphan = nullptr;
    j->sq_cap = 0;
    const size_t n = (size_t)cands, nr = (size_t)std::max(1, nrd);
    HIPCHK(hipMalloc((void**)&j->d_sq_rec, sizeof(unsigned long long) * n));
    HIPCHK(hipMemset(j->d_sq_rec, 0, sizeof(unsigned long long) * n));  // ready words: not ready
    HIPCHK(hipMalloc((void**)&j->d_sq_ctrl, sizeof(double) * n * nr));
    HIPCHK(hipMalloc((void**)&j->d_sq_ctrl32, sizeof(float) * n * nr));
    HIPCHK(hipMalloc((void**)&j->d_sq_res, sizeof(SurvBest) * n));
    // handed-over tickets: one per workgroup at most, and a launch has at most `cands` workgroups
    HIPCHK(hipMalloc((void**)&j->d_sq_orphan, sizeof(unsigned) * n));
    j->sq_cap = cands;
    j->sq_nrd = nrd;
    return SSPP_OK;
}

static int run_sspp(sspp_job* j, const double* d_ctrl, int64_t first_id, int64_t B, double* d_arc,
                    uint8_t* d_feasible, double* d_ctrl_out, sspp_best* d_best, void* stream,
                    int steps = 1, int64_t step_stride = 0) {
    sspp::clear_error();
    if (!j || j->kind != 0) return sspp::set_error(SSPP_E_INVAL, "not a SamplingPathPlanner job");
    if (B < 1 || B > j->max_batch) return sspp::set_error(SSPP_E_INVAL, "batch size out of range");
    if (!d_arc || !d_feasible) return sspp::set_error(SSPP_E_INVAL, "null output");
    if (steps < 1 || steps > kMaxSteps || (steps > 1 && d_ctrl))
        return sspp::set_error(SSPP_E_INVAL, "steps per launch: 1..64 (sampled candidates)");
    hipStream_t st = (hipStream_t)stream;
    if (j->prepass_state.load(std::memory_order_relaxed) == 2) prepass_apply(j);
    int nt, g1;
    c2f_shape(j, (int64_t)steps * B, &nt, &g1);
    const int n = j->n, D = j->D, p = j->p;
    const int r0 = d_ctrl ? 0 : std::min(p, n), r1 = d_ctrl ? n : std::max(r0, n - p);
    const int nrd = (r1 - r0) * D;
    int cpw = 64 / g1, cpb = (nt / 64) * cpw;
    // k_sspp_c2f compacts survivors, lists phase-3 candidates and reduces the block argmin with
    // one wave (tid < 64): a forced shape holding more than 64 candidates per workgroup is refused
    if (cpb > 64)
        return sspp::set_error(SSPP_E_INVAL, "launch shape " + std::to_string(nt) + "x" + std::to_string(g1) +
                                                 " holds more than 64 candidates per workgroup");
    size_t lds = c2f_lds(j, cpb, nrd);
    if (lds > 64 * 1024 && !j->opt_nt) {  // large splines: the latency shape's 4 candidates
        nt = 256; g1 = 64; cpw = 1; cpb = 4;
        lds = c2f_lds(j, cpb, nrd);
    }
    if (lds > 64 * 1024) return sspp::set_error(SSPP_E_UNSUPPORTED, "problem too large for LDS");
    const int nblk = (int)((B + cpb - 1) / cpb);
    if ((int64_t)nblk * steps > j->part_cap) {  // one BlockBest per workgroup and step
        (void)hipDeviceSynchronize();
        if (j->d_part) (void)hipFree(j->d_part);
        j->d_part = nullptr;
        j->part_cap = 0;
        if (hipMalloc((void**)&j->d_part, sizeof(BlockBest) * (size_t)nblk * steps) != hipSuccess)
            return sspp::set_error(SSPP_E_NOMEM, "hipMalloc block partials");
        j->part_cap = (int64_t)nblk * steps;
    }
    SsppC2F c{};
    c.sc = kscene_job(j, d_ctrl == nullptr);
    c.has_scene = j->scene != nullptr && (c.sc.npairs > 0 || c.sc.static_block);
    c.sampler = j->sampler;
    c.p = p; c.n = n; c.W = j->W; c.sigma = j->sigma; c.seed = j->seed;
    c.first_id = first_id; c.B = B;
    c.g1 = g1; c.cpw = cpw; c.cpb = cpb; c.npts = j->W + 1; c.n1 = std::min(g1, j->W + 1);
    c.lpc = lanes_for(j->W - 1);
    c.nblk_step = nblk;
    c.step_stride = step_stride;
    c.arc_all = j->arc_all;
    c.r0 = r0; c.r1 = r1;
    c.nt = nt; c.lds = (int)lds;
    c.ctrl_feas = j->ctrl_feas;
    const double feps = j->f32 && c.has_scene ? f32_eps(j->scene, d_ctrl ? j->h_pairs : j->h_pairs_s) : 0.0;
    c.f32 = feps > 0.0 ? 1 : 0;
    c.feps = (float)feps;
    c.fplim = kF32PosLimit;
    j->last_nt = nt; j->last_g1 = g1; j->last_f32 = c.f32;
    // split launch (the survivor queue, SurvQ): multi-step throughput launches of sampled
    // candidates with collision, one output row per candidate; launch_c2f_nt
    // splits only a launch that is one resident round (c2f_one_round)
    c.nsteps = steps;
    // (a split launch's arrival counters hold up to 65535 workgroups per shard in their low half)
    c.split = j->opt_split && (int64_t)steps * B >= kSplitMinCands && !d_ctrl && !d_ctrl_out && !j->arc_all &&
              (int64_t)nblk * steps < 65536 &&
              c.has_scene && c.sc.npairs > 0 && !c.sc.static_block && j->nm == 1 && c.sc.onegeom && !c.sc.cylbox &&
              cpb >= 3;  // the consumers' control words live in s_surv (cpb + 1 ints)
    SurvPtrs q{};
    int split_used = 0;
    if (c.split) {
        // shard s holds the survivors of workgroups b = s (mod kSurvShards), cpb at most each
        const int nb_all = nblk * steps;
        const int shard_cap = ((nb_all + kSurvShards - 1) / kSurvShards) * cpb;
        int rc = survq_reserve(j, (int64_t)shard_cap * kSurvShards, nrd);
        if (rc) return rc;
        q = SurvPtrs{j->d_sq_hdr, j->d_sq_rec, j->d_sq_ctrl, j->d_sq_ctrl32, j->d_sq_res, j->d_sq_orphan,
#ifdef SSPP_DEBUG_PROGRESS
                     j->dbg_beacon,
#endif
                     j->sq_cap, shard_cap};
        c.linger = (unsigned long long)j->opt_linger_us * 100ull;  // the 100 MHz wall clock
        c.drop_orphans = j->opt_split_drop;
        // the last workgroup's per-step minimum bits, ids and counts reuse the LDS from offset 0
        c.lds = std::max(c.lds, (int)(20 * kMaxSteps + 16));
    }
    SsppPtrs o{d_ctrl, d_ctrl_out, d_arc, d_feasible, d_best, q, &split_used};
    const int nb = nblk * steps;
    hipError_t e = hipErrorInvalidValue;
    switch (j->D) {
#ifndef SSPP_DEV_ONLY
        case 1: e = entry_c2f<1>(c, j, o, nb, st); break;
        case 2: e = entry_c2f<2>(c, j, o, nb, st); break;
        case 3: e = entry_c2f<3>(c, j, o, nb, st); break;
        case 4: e = entry_c2f<4>(c, j, o, nb, st); break;
        case 6: e = entry_c2f<6>(c, j, o, nb, st); break;
        case 9: e = entry_c2f<9>(c, j, o, nb, st); break;
#endif
        case 7: e = entry_c2f<7>(c, j, o, nb, st); break;
    }
    j->last_split = split_used;
    if (e != hipSuccess) return hip_fail(e, "k_sspp_c2f launch");
    return SSPP_OK;
}

extern "C" int sspp_job_sample_score(sspp_job* j, int64_t first_id, int64_t B, double* d_arc,
                          uint8_t* d_feasible, double* d_ctrl_out, sspp_best* d_best, void* stream) {
    return run_sspp(j, nullptr, first_id, B, d_arc, d_feasible, d_ctrl_out, d_best, stream);
}

// Re-target a SamplingPathPlanner job to another plan() call with the same knots, dof and
// check_points (the drop-in planner caches one job per shape): the initial control points,
// sigma, limits and seed change; the pair tables are re-ordered for the new mean path (gap
// order: a re-plan stays on the microsecond host path, so the hit-order pre-pass of job
// creation is not repeated, and the waypoint order stays the creation's).  Uploads are
// asynchronous on `stream` from job-owned host copies (valid until the next update).
extern "C" int sspp_job_update_sspp(sspp_job* j, const double* init_ctrl, double sigma,
                                    const double* limits, uint64_t seed, void* stream) {
    sspp::clear_error();
    if (!j || j->kind != 0 || !init_ctrl || !limits) return sspp::set_error(SSPP_E_INVAL, "sspp_job_update_sspp: bad argument");
    const size_t nd = (size_t)j->n * j->D;
    hipStream_t st = (hipStream_t)stream;
    j->seed = seed;  // a kernel argument: nothing to upload
    // the device tables depend only on (init_ctrl, sigma, limits): an update that repeats the
    // values the device holds (a planning loop re-planning the same query) uploads nothing
    if (j->h_stage.size() == nd + (size_t)j->D && j->sigma == sigma &&
        std::memcmp(j->h_stage.data(), init_ctrl, sizeof(double) * nd) == 0 &&
        std::memcmp(j->h_stage.data() + nd, limits, sizeof(double) * j->D) == 0)
        return SSPP_OK;
    const bool pairs = j->d_pairs && j->scene;
    const size_t vbytes = sizeof(double) * (nd + j->D);
    const size_t need = vbytes + (pairs ? 2 * sizeof(DPair) * j->scene->pairs.size() : 0);
    // the pinned staging is the source of the previous update's copies until they complete
    if (j->upd_pending) {
        HIPCHK(hipEventSynchronize(j->upd_ev));
        j->upd_pending = false;
    }
    if (need > j->h_pin_bytes) {
        if (j->h_pin) HIPCHK(hipHostFree(j->h_pin));
        j->h_pin = nullptr;
        j->h_pin_bytes = 0;
        HIPCHK(hipHostMalloc((void**)&j->h_pin, need, hipHostMallocDefault));
        j->h_pin_bytes = need;
    }
    if (!j->upd_ev) HIPCHK(hipEventCreateWithFlags(&j->upd_ev, hipEventDisableTiming));
    j->h_stage.assign(init_ctrl, init_ctrl + nd);
    j->h_stage.insert(j->h_stage.end(), limits, limits + j->D);
    j->sigma = sigma;
    std::memcpy(j->h_pin, j->h_stage.data(), vbytes);
    const double* pv = (const double*)j->h_pin;
    HIPCHK(hipMemcpyAsync(j->d_init, pv, sizeof(double) * nd, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(j->d_limits, pv + nd, sizeof(double) * j->D, hipMemcpyHostToDevice, st));
    if (pairs) {
        ++j->tables_gen;  // a pre-pass still running ordered the previous values' tables
        const int rc = set_job_tables(j, init_ctrl, sigma, limits, j->pair_order == 0 ? 0 : 1, false, stream, vbytes);
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(j->upd_ev, st));
    j->upd_pending = true;
    return SSPP_OK;
}

extern "C" int sspp_job_score_ctrl(sspp_job* j, const double* d_ctrl, int64_t first_id, int64_t B,
                        double* d_arc, uint8_t* d_feasible, sspp_best* d_best, void* stream) {
    if (!d_ctrl) return sspp::set_error(SSPP_E_INVAL, "null control points");
    return run_sspp(j, d_ctrl, first_id, B, d_arc, d_feasible, nullptr, d_best, stream);
}

// Explicit launch options of a job (tests and tuning; nothing is read from the environment).
extern "C" int sspp_job_set_option(sspp_job* j, int key, int64_t value) {
    sspp::clear_error();
    if (!j) return sspp::set_error(SSPP_E_INVAL, "null job");
    switch (key) {
        case SSPP_OPT_SHAPE_NT:
            if (j->kind != 0 || !(value == 0 || value == 64 || value == 128 || value == 256))
                return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_SHAPE_NT: 0, 64, 128 or 256");
            j->opt_nt = (int)value;
            return SSPP_OK;
        case SSPP_OPT_SHAPE_G1:
            if (j->kind != 0 || value < 0 || value > 64)
                return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_SHAPE_G1: 0 (per launch) or 1..64");
            j->opt_g1 = (int)value;
            return SSPP_OK;
        case SSPP_OPT_ORDER: {
            if (j->kind != 0 || value < 0 || value > 2) return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_ORDER: 0, 1 or 2");
            prepass_drop(j);
            HIPCHK(hipDeviceSynchronize());  // earlier launches may still read the tables
            const size_t nd = (size_t)j->n * j->D;
            return set_job_tables(j, j->h_stage.data(), j->sigma, j->h_stage.data() + nd, (int)value, true, nullptr);
        }
        case SSPP_OPT_TSP_FORM:
            if (j->kind != 1 || value < -1 || value > 4) return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_TSP_FORM: -1..4");
            j->tsp_form = (int)value;
            return SSPP_OK;
        case SSPP_OPT_TSP_GENERIC:
            if (j->kind != 1) return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_TSP_GENERIC: TaskSpacePlanner jobs only");
            j->tsp_generic = value ? 1 : 0;
            return SSPP_OK;
        case SSPP_OPT_F32:
            if (j->kind != 0 || value < 0 || value > 1) return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_F32: 0 or 1");
            j->f32 = (int)value;
            return SSPP_OK;
        case SSPP_OPT_SPLIT:
            if (j->kind != 0 || value < 0 || value > 1) return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_SPLIT: 0 or 1");
            j->opt_split = (int)value;
            return SSPP_OK;
        case SSPP_OPT_SPLIT_LINGER_US:
            if (j->kind != 0 || value < 0 || value > 1000000)
                return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_SPLIT_LINGER_US: 0..1000000");
            j->opt_linger_us = (int)value;
            return SSPP_OK;
        case SSPP_OPT_SPLIT_DROP:
            if (j->kind != 0 || value < 0 || value > 1) return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_SPLIT_DROP: 0 or 1");
            j->opt_split_drop = (int)value;
            return SSPP_OK;
#ifdef SSPP_DEBUG_PROGRESS
        case 900:  // debugging builds: the split launch's progress beacons ([grid][4] words, mapped host memory)
            j->dbg_beacon = (unsigned*)(uintptr_t)value;
            return SSPP_OK;
#endif
        case SSPP_OPT_TSP_REP:
            if (j->kind != 1 || value < -1 || value == 0 || value > 16)
                return sspp::set_error(SSPP_E_INVAL, "SSPP_OPT_TSP_REP: -1 or 1..16");
            j->tsp_rep = (int)value;
            return SSPP_OK;
    }
    return sspp::set_error(SSPP_E_INVAL, "unknown or read-only option");
}

extern "C" int sspp_job_get_option(const sspp_job* j, int key, int64_t* value) {
    if (!j || !value) return sspp::set_error(SSPP_E_INVAL, "null argument");
    switch (key) {
        case SSPP_OPT_SHAPE_NT: *value = j->opt_nt; return SSPP_OK;
        case SSPP_OPT_SHAPE_G1: *value = j->opt_g1; return SSPP_OK;
        case SSPP_OPT_ORDER: *value = j->pair_order; return SSPP_OK;
        case SSPP_OPT_TSP_FORM: *value = j->kind == 1 ? j->last_form : -1; return SSPP_OK;
        case SSPP_OPT_TSP_GENERIC: *value = j->tsp_generic; return SSPP_OK;
        case SSPP_OPT_SAMPLER: *value = j->sampler; return SSPP_OK;
        case SSPP_OPT_LAST_NT: *value = j->last_nt; return SSPP_OK;
        case SSPP_OPT_LAST_G1: *value = j->last_g1; return SSPP_OK;
        case SSPP_OPT_WP_ORDER: *value = j->wp_order; return SSPP_OK;
        case SSPP_OPT_PREPASS_US: *value = (int64_t)(j->prepass_ms * 1e3); return SSPP_OK;
        case SSPP_OPT_NPAIRS: *value = j->np_samp; return SSPP_OK;
        case SSPP_OPT_CYLBOX: *value = j->cb_samp; return SSPP_OK;
        case SSPP_OPT_F32: *value = j->f32; return SSPP_OK;
        case SSPP_OPT_LAST_F32: *value = j->last_f32; return SSPP_OK;
        case SSPP_OPT_CREATE_US: *value = (int64_t)(j->create_ms * 1e3); return SSPP_OK;
        case SSPP_OPT_SPLIT: *value = j->opt_split; return SSPP_OK;
        case SSPP_OPT_LAST_SPLIT: *value = j->last_split; return SSPP_OK;
        case SSPP_OPT_SPLIT_LINGER_US: *value = j->opt_linger_us; return SSPP_OK;
        case SSPP_OPT_SPLIT_DROP: *value = j->opt_split_drop; return SSPP_OK;
        case SSPP_OPT_SPLIT_HANDOFFS:
        case SSPP_OPT_SPLIT_LOST: {  // synchronous read of the queue header (tests, diagnostics)
            *value = 0;
            if (!j->d_sq_hdr) return SSPP_OK;
            SurvQ h;
            HIPCHK(hipDeviceSynchronize());
            HIPCHK(hipMemcpy(&h, j->d_sq_hdr, sizeof(SurvQ), hipMemcpyDeviceToHost));
            *value = (int64_t)(key == SSPP_OPT_SPLIT_HANDOFFS ? h.handoffs : h.lost_total);
            return SSPP_OK;
        }
        case SSPP_OPT_TSP_REP: *value = j->kind == 1 ? j->last_rep : 0; return SSPP_OK;
        case SSPP_OPT_PREPASS_STATE: *value = j->prepass_state.load(std::memory_order_acquire); return SSPP_OK;
    }
    return sspp::set_error(SSPP_E_INVAL, "unknown option");
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
    std::vector<double> u(n), knots(n + 3), Minv((size_t)2 * n * n + n);  // QR program
    for (int i = 0; i < n; ++i) u[i] = (double)i / (n - 1);
    if (sspp::qr_program(u.data(), n, 2, knots.data(), Minv.data()) != 0) {
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
    // one record per workgroup: k_tsp's blocks, or one per candidate for k_tsp_pp
    const int64_t nrec = std::max<int64_t>(nblk, std::min<int64_t>(max_batch, kTspPpMaxBatch));
    j->part_cap = nrec;
    if (hipMalloc((void**)&j->d_part, sizeof(BlockBest) * nrec) != hipSuccess ||
        hipMalloc((void**)&j->d_sync, sizeof(ArgminSync)) != hipSuccess ||
        hipMemset(j->d_sync, 0, sizeof(ArgminSync)) != hipSuccess) {
        sspp_job_free(j);
        return sspp::set_error(SSPP_E_NOMEM, "hipMalloc block partials");
    }
    *out = j;
    return SSPP_OK;
}

// default sub-batches per k_tsp workgroup (form 3): enough to bring the grid down to about one
// resident round of 4-wave workgroups (1024 on 256 CUs), at most 8.  Stacking (16384 candidates,
// 2 per sub-batch): 8 — 91.8 / 107.0 / 117.3 / 123.2 M cand/s at 1 / 2 / 4 / 8 (profiles/r05u_*)
static int tsp_auto_rep(const sspp_job* j, int64_t B) {
    const int64_t r = B / ((int64_t)j->cpb * 1024);
    return (int)std::max<int64_t>(1, std::min<int64_t>(8, r));
}

// sub-batches per workgroup for a k_tsp launch of form `mode` (1 where the form runs one)
static int tsp_rep_for(const sspp_job* j, const TspK& k, int mode, int64_t B) {
    if ((mode != 3 && mode != 4) || !((SSPP_TSP_REP_FORMS >> mode) & 1)) return 1;
    int rep = j->tsp_rep > 0 ? j->tsp_rep : tsp_auto_rep(j, B);
    const size_t extra = mode == 3 ? tsp_def_lds(k.sc.npairs) : tsp_def2_lds(k.sc.npairs);
    while (rep > 1 && tsp_base_lds(j->cpb, j->n, rep) + extra > 64 * 1024) --rep;
    return rep;
}

// the launch's TspK for job j (run_tsp, tsp_eval_ces_group)
static TspK tsp_k(const sspp_job* j, int64_t first_id, int64_t B) {
    TspK k{};
    k.sc = kscene(j->scene, true, j->tsp_generic != 0);
    k.n = j->n; k.K = j->K; k.cp = j->cp;
    for (int i = 0; i < 4; ++i) { k.start[i] = j->start[i]; k.end[i] = j->end[i]; k.lo[i] = j->lo[i]; k.hi[i] = j->hi[i]; }
    k.z_min = j->z_min; k.seed = j->seed; k.first_id = first_id; k.B = B;
    k.w_col = j->w_col; k.floor_z_min = j->floor_z_min; k.floor_margin = j->floor_margin;
    k.floor_scale = j->floor_scale;
    k.lpc = j->lpc; k.cpb = j->cpb;
    return k;
}

// k_tsp's deferred-polygon forms (modes 3 / 4) where they apply, else the inline form (0); the
// pair-split forms (1 / 2) are run_tsp's choice for small batches
static int tsp_large_mode(const sspp_job* j, const TspK& k) {
    const int pp_opt = j->tsp_form;
    bool has_bb = false;
    for (const DPair& pr : j->scene->pairs) has_bb |= j->scene->geoms[pr.gm].type == 6 && pr.otype == 6;
    const bool def_ok = j->cp <= j->lpc && k.sc.npairs >= 1 && k.sc.npairs <= kDefPairs && has_bb &&
                        j->lds + tsp_def_lds(k.sc.npairs) <= 64 * 1024;
    if (def_ok && (pp_opt < 0 || pp_opt == 3)) return 3;
    const bool def2_ok = j->cp <= j->lpc && k.sc.npairs >= 1 && k.sc.npairs <= 64 && has_bb &&
                         j->lds + tsp_def2_lds(k.sc.npairs) <= 64 * 1024;
    if (def2_ok && (pp_opt < 0 || pp_opt == 4)) return 4;
    return 0;
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
    TspK k = tsp_k(j, first_id, B);
    const double* mean = j->d_mean;
    const double* sigma = j->d_sigma;
    if (ces) {
        if (d_vias) return sspp::set_error(SSPP_E_INVAL, "CES slot mode samples its own via sets");
        k.ces = 1; k.fixed = ces->fixed; k.nfixed = ces->nfixed;
        k.slot0 = ces->slot0; k.samples = ces->samples;
        mean = ces->mean; sigma = ces->sigma;
        for (int i = 0; i < 4; ++i) { k.start[i] = ces->start[i]; k.end[i] = ces->end[i]; }
    }
    // small batches (the anytime CES loop) take the pair-split kernel: one workgroup per
    // candidate, the scene's pairs spread over 8 waves (same outputs, bit for bit)
    // and, with more than 8 pairs, ceil(npairs / 8) workgroups per candidate (k_tsp_pp2).
    // The form is an explicit job option (SSPP_OPT_TSP_FORM: 0 k_tsp, 1 the single-workgroup
    // split, 2 the multi-workgroup split where it applies; -1 = by batch size)
    const int pp_opt = j->tsp_form;
    const bool pp_ok = j->cp <= 64 && k.sc.npairs <= 64 && B <= j->part_cap;
    const bool pp = pp_ok && (pp_opt < 0 ? B <= kTspPpMaxBatch : (pp_opt == 1 || pp_opt == 2));
    const int npg = (k.sc.npairs + 7) / 8;
    int mode = pp ? 1 : 0;
    if (pp && npg > 1 && pp_opt != 1 && B <= kTspPpMaxBatch) {
        if (!j->d_pp_arrive) {
            const int64_t cap = std::min<int64_t>(j->max_batch, kTspPpMaxBatch);
            if (hipMalloc((void**)&j->d_pp_nd, sizeof(unsigned) * 4096 * (size_t)cap) != hipSuccess ||
                hipMalloc((void**)&j->d_pp_term, sizeof(double) * 4096 * (size_t)cap) != hipSuccess ||
                hipMalloc((void**)&j->d_pp_arrive, sizeof(unsigned) * (size_t)cap) != hipSuccess ||
                hipMemset(j->d_pp_arrive, 0, sizeof(unsigned) * (size_t)cap) != hipSuccess)
                return sspp::set_error(SSPP_E_NOMEM, "hipMalloc k_tsp_pp2 records");
            j->pp_cap = cap;
        }
        if (B <= j->pp_cap) {
            mode = 2;
            k.rec_nd = j->d_pp_nd; k.rec_term = j->d_pp_term; k.arrive = j->d_pp_arrive; k.npg = npg;
        }
    }
    // the deferred-polygon form of k_tsp (mode 3): one waypoint per lane, few pairs, some of them
    // box-box (the polygons it defers); the default for such batches above the pair-split sizes.
    // (A form in rounds for many pairs — the gripper's 48 — measured more registers than the
    // inline narrowphase: the polygons of divergent pairs need the pair data in VGPRs.)  The
    // lane-local deferred polygons (mode 4): one waypoint per lane, up to 64 pairs, some of them
    // box-box; the default where mode 3 does not apply (the gripper's 48 pairs)
    if (mode == 0) mode = tsp_large_mode(j, k);
    // k_tsp forms: rep sub-batches per workgroup (SSPP_OPT_TSP_REP; -1: REP_AUTO below)
    k.rep = tsp_rep_for(j, k, mode, B);
    j->last_rep = k.rep;
    const int cpr = j->cpb * k.rep;
    const int nblk = mode == 2 ? (int)B * npg : mode == 1 ? (int)B : (int)((B + cpr - 1) / cpr);
    j->last_form = mode;
    hipStream_t st = (hipStream_t)stream;
    hipError_t e0 = entry_tsp<0>(k, j, nblk, mean, sigma, d_vias, d_vias_out, d_L, d_Cnf, d_Cwf, d_cost, d_status,
                                 d_best, st, mode);
    if (e0 != hipSuccess) return hip_fail(e0, "k_tsp launch");
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "k_tsp launch");
    return SSPP_OK;
}

void sspp::job_set_ctrl_feasible_only(sspp_job* j, int on) {
    if (j) j->ctrl_feas = on ? 1 : 0;
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

// Multi-goal CES evaluation (ces.hip sspp_ces_plan_group): one k_tsp_group launch over every goal's
// slots [0, n).  The goals' jobs must describe the same evaluation (scene, spline, checks, bounds,
// costs) and differ only in start / end, seed, distribution and buffers; SSPP_E_UNSUPPORTED when
// they do not, or when run_tsp would pick a pair-split form for n slots (the caller then
// evaluates goal by goal).
int sspp::tsp_eval_ces_group(sspp_job* const* jobs, const TspCesEval* evs, const TspCesOut* outs, int G,
                             int64_t n, void* stream) {
    sspp::clear_error();
    if (!jobs || !evs || !outs || G < 1 || n < 1) return sspp::set_error(SSPP_E_INVAL, "tsp_eval_ces_group: bad argument");
    if (G > kMaxGoals) return sspp::set_error(SSPP_E_UNSUPPORTED, "more goals than one launch holds");
    const sspp_job* j0 = jobs[0];
    for (int g = 0; g < G; ++g) {
        const sspp_job* j = jobs[g];
        if (!j || j->kind != 1 || n > j->max_batch) return sspp::set_error(SSPP_E_INVAL, "tsp_eval_ces_group: bad job");
        bool same = j->scene == j0->scene && j->n == j0->n && j->K == j0->K && j->cp == j0->cp &&
                    j->lpc == j0->lpc && j->cpb == j0->cpb && j->lds == j0->lds && j->z_min == j0->z_min &&
                    j->w_col == j0->w_col && j->floor_z_min == j0->floor_z_min &&
                    j->floor_margin == j0->floor_margin && j->floor_scale == j0->floor_scale &&
                    j->tsp_generic == j0->tsp_generic && j->tsp_form == j0->tsp_form &&
                    j->d_tab && j->h_knots == j0->h_knots && evs[g].samples == evs[0].samples &&
                    evs[g].slot0 == 0;
        for (int i = 0; i < 4; ++i) same = same && j->lo[i] == j0->lo[i] && j->hi[i] == j0->hi[i];
        if (!same) return sspp::set_error(SSPP_E_UNSUPPORTED, "goals differ beyond start / end / seed");
        const TspCesEval& e = evs[g];
        const TspCesOut& o = outs[g];
        if (!e.fixed || !e.nfixed || !e.mean || !e.sigma || !o.L || !o.Cnf || !o.Cwf || !o.cost || !o.status || !o.vias)
            return sspp::set_error(SSPP_E_INVAL, "tsp_eval_ces_group: null argument");
    }
    TspK k = tsp_k(j0, 0, n);
    k.ces = 1; k.slot0 = 0; k.samples = evs[0].samples;
    const bool pp_ok = j0->cp <= 64 && k.sc.npairs <= 64 && n <= j0->part_cap;
    const int pp_opt = j0->tsp_form;
    if (pp_ok && (pp_opt < 0 ? n <= kTspPpMaxBatch : (pp_opt == 1 || pp_opt == 2)))
        return sspp::set_error(SSPP_E_UNSUPPORTED, "pair-split batch size: goal by goal");
    const int mode = tsp_large_mode(j0, k);
    k.rep = tsp_rep_for(j0, k, mode, n * G);
    TspGoals goals{};
    goals.n = G;
    goals.nblk = (int)((n + (int64_t)j0->cpb * k.rep - 1) / ((int64_t)j0->cpb * k.rep));
    for (int g = 0; g < G; ++g) {
        const TspCesEval& e = evs[g];
        const TspCesOut& o = outs[g];
        TspGoal& q = goals.g[g];
        for (int i = 0; i < 4; ++i) { q.start[i] = e.start[i]; q.end[i] = e.end[i]; }
        q.seed = jobs[g]->seed; q.first_id = e.first_id;
        q.fixed = e.fixed; q.nfixed = e.nfixed; q.mean = e.mean; q.sigma = e.sigma;
        q.vias_out = o.vias; q.oL = o.L; q.oCnf = o.Cnf; q.oCwf = o.Cwf; q.ocost = o.cost; q.ostatus = o.status;
        jobs[g]->last_form = mode;
        jobs[g]->last_rep = k.rep;
    }
    hipError_t e = entry_tsp_group<0>(k, goals, j0, goals.nblk * G, (hipStream_t)stream, mode);
    if (e != hipSuccess) return hip_fail(e, "k_tsp_group launch");
    return SSPP_OK;
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

extern "C" int sspp_job_info(const sspp_job* j, int* lpc, int* cpb_out, int* threads, size_t* lds) {
    if (!j) return sspp::set_error(SSPP_E_INVAL, "null job");
    if (j->kind == 0) {  // the last k_sspp_c2f launch's shape (before any launch: the throughput shape)
        const int nt = j->last_nt ? j->last_nt : kThroughputNT, g1 = j->last_g1 ? j->last_g1 : kThroughputG1;
        const int cpb = (nt / 64) * (64 / g1);
        if (lpc) *lpc = g1;
        if (cpb_out) *cpb_out = cpb;
        if (threads) *threads = nt;
        if (lds) *lds = c2f_lds(j, cpb, std::max(0, j->n - 2 * j->p) * j->D);
        return SSPP_OK;
    }
    if (lpc) *lpc = j->lpc;
    if (cpb_out) *cpb_out = j->cpb;
    if (threads) *threads = kBlock;
    if (lds) *lds = j->lds;
    return SSPP_OK;
}

extern "C" void sspp_job_free(sspp_job* j) {
    if (!j) return;
    prepass_drop(j);
    if (j->pre_stream) (void)hipStreamSynchronize(j->pre_stream);
    for (void* q : {(void*)j->d_sq_hdr, (void*)j->d_sq_rec, (void*)j->d_sq_ctrl, (void*)j->d_sq_ctrl32,
                    (void*)j->d_sq_res, (void*)j->d_sq_orphan})
        if (q) (void)hipFree(q);
    for (void* q : j->retired) if (q) (void)hipFree(q);
    for (void* q : {(void*)j->d_hits, (void*)j->d_census_pairs}) if (q) (void)hipFree(q);
    if (j->h_hits) (void)hipHostFree(j->h_hits);
    if (j->pre_ev) (void)hipEventDestroy(j->pre_ev);

    for (double* p : {j->d_knots, j->d_tab, j->d_init, j->d_limits, j->d_Minv, j->d_mean, j->d_sigma})
        if (p) (void)hipFree(p);
    if (j->d_span) (void)hipFree(j->d_span);
    if (j->d_otab) (void)hipFree(j->d_otab);
    if (j->d_otab32) (void)hipFree(j->d_otab32);
    if (j->d_pairs) (void)hipFree(j->d_pairs);
    if (j->d_pairs_s) (void)hipFree(j->d_pairs_s);
    if (j->d_ospan) (void)hipFree(j->d_ospan);
    if (j->d_part) (void)hipFree(j->d_part);
    if (j->d_sync) (void)hipFree(j->d_sync);
    for (void* q : {(void*)j->d_pp_nd, (void*)j->d_pp_term, (void*)j->d_pp_arrive})
        if (q) (void)hipFree(q);
    if (j->upd_ev) {
        (void)hipEventSynchronize(j->upd_ev);
        (void)hipEventDestroy(j->upd_ev);
    }
    if (j->h_pin) (void)hipHostFree(j->h_pin);
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
    long long bi = -1, cnt = 0, lost = 0;  // lost: the records' `reserved`, summed (a shortfall stays visible)
    for (int r = threadIdx.x; r < R; r += 64) {
        const BlockBest b = parts[(long long)r * G + g];
        cnt += b.count;
        lost += b.pad;
        if (better(b.cost, b.idx, bc, bi)) { bc = b.cost; bi = b.idx; }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double oc = __shfl_xor(bc, off, 64);
        const long long oi = __shfl_xor(bi, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
        lost += __shfl_xor(lost, off, 64);
        if (better(oc, oi, bc, bi)) { bc = oc; bi = oi; }
    }
    if (threadIdx.x == 0) {
        out[g].cost = bi < 0 ? INFINITY : bc;
        out[g].index = bi;
        out[g].count = cnt;
        out[g].reserved = lost;
    }
}
}  // namespace

static int steps_check(sspp_job* const* jobs, int nbranch, void* const* streams, int64_t B, int steps_per_launch,
                       double* const* d_arc, uint8_t* const* d_feasible) {
    if (!jobs || !streams || !d_arc || !d_feasible || nbranch < 1 || B < 1)
        return sspp::set_error(SSPP_E_INVAL, "sspp steps: bad argument");
    for (int b = 0; b < nbranch; ++b) {
        if (!jobs[b] || jobs[b]->kind != 0 || !d_arc[b] || !d_feasible[b])
            return sspp::set_error(SSPP_E_INVAL, "sspp steps: bad branch");
        for (int c = 0; c < b; ++c)
            if (jobs[c] == jobs[b]) return sspp::set_error(SSPP_E_INVAL, "branches need distinct jobs");
    }
    if (steps_per_launch < 1 || steps_per_launch > kMaxSteps)
        return sspp::set_error(SSPP_E_INVAL, "steps_per_launch must be in [1, 64]");
    return SSPP_OK;
}

static int steps_run(sspp_job* const* jobs, int nbranch, void* const* streams, int64_t B, int S, int nsteps,
                     int64_t first_id, int64_t step_stride, double* const* d_arc, uint8_t* const* d_feasible,
                     sspp_best* d_best) {
    for (int i = 0, l = 0; i < nsteps; i += S, ++l) {
        const int b = l % nbranch, s = std::min(S, nsteps - i);
        const int rc = run_sspp(jobs[b], nullptr, first_id + (int64_t)i * step_stride, B, d_arc[b],
                                d_feasible[b], nullptr, d_best ? d_best + i : nullptr, streams[b],
                                s, step_stride);
        if (rc != SSPP_OK) return rc;
    }
    return SSPP_OK;
}

extern "C" int sspp_steps_enqueue_sspp(sspp_job* const* jobs, int nbranch, void* const* streams,
                                       int64_t B, int nsteps, int steps_per_launch, int64_t first_id,
                                       int64_t step_stride, double* const* d_arc,
                                       uint8_t* const* d_feasible, sspp_best* d_best) {
    sspp::clear_error();
    int rc = steps_check(jobs, nbranch, streams, B, steps_per_launch, d_arc, d_feasible);
    if (rc) return rc;
    if (nsteps < 0) return sspp::set_error(SSPP_E_INVAL, "sspp_steps_enqueue_sspp: nsteps < 0");
    return steps_run(jobs, nbranch, streams, B, steps_per_launch, nsteps, first_id, step_stride, d_arc,
                     d_feasible, d_best);
}

// the same executor as a handle: its branches checked and copied once, then each call passes only
// the steps to run (a planning loop's per-call host work: one small argument list)
struct sspp_steps {
    std::vector<sspp_job*> jobs;
    std::vector<void*> streams;
    std::vector<double*> arc;
    std::vector<uint8_t*> feas;
    int64_t B = 0;
    int spl = 1;
};

extern "C" int sspp_steps_create_sspp(sspp_job* const* jobs, int nbranch, void* const* streams, int64_t B,
                                      int steps_per_launch, double* const* d_arc, uint8_t* const* d_feasible,
                                      sspp_steps** out) {
    sspp::clear_error();
    if (!out) return sspp::set_error(SSPP_E_INVAL, "sspp_steps_create_sspp: null output");
    int rc = steps_check(jobs, nbranch, streams, B, steps_per_launch, d_arc, d_feasible);
    if (rc) return rc;
    auto* ex = new sspp_steps();
    ex->jobs.assign(jobs, jobs + nbranch);
    ex->streams.assign(streams, streams + nbranch);
    ex->arc.assign(d_arc, d_arc + nbranch);
    ex->feas.assign(d_feasible, d_feasible + nbranch);
    ex->B = B;
    ex->spl = steps_per_launch;
    *out = ex;
    return SSPP_OK;
}

extern "C" int sspp_steps_run(sspp_steps* ex, int nsteps, int64_t first_id, int64_t step_stride, sspp_best* d_best) {
    if (!ex || nsteps < 0) {
        sspp::clear_error();
        return sspp::set_error(SSPP_E_INVAL, "sspp_steps_run: bad argument");
    }
    return steps_run(ex->jobs.data(), (int)ex->jobs.size(), ex->streams.data(), ex->B, ex->spl, nsteps, first_id,
                     step_stride, ex->arc.data(), ex->feas.data(), d_best);
}

extern "C" void sspp_steps_free(sspp_steps* ex) { delete ex; }

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

#ifdef SSPP_TSP_STATS
extern "C" int sspp_debug_tsp_stats(unsigned long long* out, int reset) {
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tsp_stats), sizeof(unsigned long long) * 16);
    if (reset) {
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tsp_stats), z, sizeof z);
    }
    return 0;
}
#endif
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
extern "C" int sspp_debug_wg_phases(unsigned long long* out, int n) {  // 8 per workgroup
    hipDeviceSynchronize();
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_ph), sizeof(unsigned long long) * (size_t)n);
    return 0;
}
extern "C" int sspp_debug_p2_times(unsigned long long* out, int n) {  // [8 * 4095]: the split epilogue
    hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_p2_t), sizeof(unsigned long long) * (size_t)n);
    return 0;
}
extern "C" int sspp_debug_p2_waves(unsigned long long* out, int n) {  // 8 per split-queue slot
    hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_p2_w), sizeof(unsigned long long) * (size_t)n);
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


