// planner.hip — the cached drop-in SamplingPathPlanner behind `_sspp.SamplingPathPlannerN`.
//
// Reference: the planner object of include/sspp.h:20-245, bound at src/sspp_bindings.cpp:24-50.
// The reference keeps its MuJoCo model and one mjData per OpenMP thread for the planner's
// lifetime (initializeDataCopies, include/sspp.h:235-244); here the planner keeps, per object:
// a HIP stream, the job of the last plan() shape (its basis tables, pair table and argmin
// counters stay on the device), the candidate buffers, and pinned host memory that the
// scoring kernel writes its outputs into.  A plan() call is therefore
//   initializePath (host, µs) -> sspp_job_update_sspp (async copies; none when the query
//   repeats) -> k_sspp_c2f (sample + score + fused argmin; arc / feasible / the argmin record
//   and the control points of the feasible candidates only, straight into pinned host memory)
//   -> stream sync -> the feasible rows gathered on the host in candidate order
// with no allocation, no device-wide synchronisation, no second launch and no copy of
// infeasible candidates' control points (plan() returns only the feasible splines,
// include/sspp.h:215-216).
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "model.h"

namespace {

int hipck(hipError_t e, const char* what) {
    if (e == hipSuccess) return SSPP_OK;
    return sspp::set_error(SSPP_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
struct Dev {
    T* p = nullptr;
    size_t n = 0;
    ~Dev() { if (p) (void)hipFree(p); }
    int reserve(size_t count) {
        if (count <= n) return SSPP_OK;
        if (p) (void)hipFree(p);
        p = nullptr; n = 0;
        hipError_t e = hipMalloc((void**)&p, sizeof(T) * (count ? count : 1));
        if (e != hipSuccess) return sspp::set_error(SSPP_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        n = count;
        return SSPP_OK;
    }
};

template <class T>
struct Pinned {
    T* p = nullptr;
    T* d = nullptr;  // its device address (mapped), looked up once per allocation
    size_t n = 0;
    ~Pinned() { if (p) (void)hipHostFree(p); }
    int reserve(size_t count) {
        if (count <= n) return SSPP_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr; d = nullptr; n = 0;
        hipError_t e = hipHostMalloc((void**)&p, sizeof(T) * (count ? count : 1),
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return sspp::set_error(SSPP_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        n = count;
        return SSPP_OK;
    }
    T* dev() {
        if (!d && p) {
            void* q = nullptr;
            if (hipHostGetDevicePointer(&q, p, 0) == hipSuccess) d = (T*)q;
        }
        return d;
    }
};

struct JobRef {
    sspp_job* j = nullptr;
    ~JobRef() { reset(); }
    void reset() { if (j) sspp_job_free(j); j = nullptr; }
};

}  // namespace

struct sspp_planner {
    const sspp_scene* scene = nullptr;
    int D = 0;
    hipStream_t stream = nullptr;  // sspp::shared_stream(0), not owned
    // plan(): job of the last shape
    JobRef plan_job;
    int plan_n = 0, plan_W = 0;
    int64_t plan_cap = 0;
    Dev<double> d_arc, d_ctrl;
    Dev<unsigned char> d_feas;
    Dev<sspp_best> d_best;
    Pinned<double> h_arc, h_ctrl;      // plan(): the scoring kernel's outputs (mapped)
    Pinned<unsigned char> h_feas;
    Pinned<sspp_best> h_best;
    // score(): job keyed on (knots, n, W, collision)
    JobRef score_job;
    std::vector<double> score_knots;
    int score_W = 0, score_coll = -1;
    int64_t score_cap = 0;
    Pinned<double> h_in;
    Pinned<double> h_sarc;
    Pinned<unsigned char> h_sfeas;
    Pinned<sspp_best> h_sbest;
    Dev<double> d_in;
    ~sspp_planner() {
        if (stream) (void)hipStreamSynchronize(stream);  // this planner's work on the shared stream
        plan_job.reset();
        score_job.reset();
    }
};

extern "C" int sspp_planner_create(const sspp_scene* scene, int dof, sspp_planner** out) {
    sspp::clear_error();
    if (!out || dof < 1 || dof > 16) return sspp::set_error(SSPP_E_INVAL, "sspp_planner_create: bad argument");
    hipStream_t st = (hipStream_t)sspp::shared_stream(0);
    if (!st) return sspp::set_error(SSPP_E_HIP, "hipStreamCreate (shared planner stream)");
    auto* p = new sspp_planner();
    p->scene = scene;
    p->D = dof;
    p->stream = st;
    *out = p;
    return SSPP_OK;
}

// One stream for every planner's plan() and one for every job's pre-pass, for the process: a
// planner used to create its own stream, and the first fresh planner after the process's first
// three streams paid 5.7 ms for a new hardware queue in its first plan().
// plan() synchronises the stream it enqueued on, so planners used from one host thread never wait
// for each other; planners driven from several host threads share the GPU queue in order.
void* sspp::shared_stream(int which) {
    static std::mutex mu;
    static hipStream_t st[2] = {nullptr, nullptr};
    if (which < 0 || which > 1) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    if (!st[which] && hipStreamCreateWithFlags(&st[which], hipStreamNonBlocking) != hipSuccess) st[which] = nullptr;
    return (void*)st[which];
}

extern "C" void sspp_planner_free(sspp_planner* p) { delete p; }

extern "C" int sspp_planner_get_option(const sspp_planner* p, int key, int64_t* value) {
    sspp::clear_error();
    if (!p || !value) return sspp::set_error(SSPP_E_INVAL, "sspp_planner_get_option: null argument");
    if (!p->plan_job.j) return sspp::set_error(SSPP_E_INVAL, "sspp_planner_get_option: no plan() yet");
    return sspp_job_get_option(p->plan_job.j, key, value);
}

// plan()'s common front: initializePath on the host, then the job of this shape created (first
// call / new shape / larger batch) or re-targeted asynchronously, then one scoring launch on the
// planner's stream.  pinned_out: arc / feasible / best and the feasible candidates' control
// points go straight to the mapped pinned buffers (plan()); otherwise to device memory, the
// control points of every candidate only with all_ctrl (sspp_plan_sspp).
static int plan_enqueue(sspp_planner* p, const double* start, const double* end, double sigma,
                        const double* limits, int sample_count, int check_points, int init_points,
                        uint64_t seed, int64_t first_id, double* knots_out, bool pinned_out,
                        bool all_ctrl = false) {
    const int n = init_points, D = p->D, deg = 3;
    if (sample_count < 1) return sspp::set_error(SSPP_E_INVAL, "sample_count must be >= 1");
    if (n < deg + 1) return sspp::set_error(SSPP_E_INVAL, "init_points must be >= 4 for a cubic spline");
    if (check_points < 2) return sspp::set_error(SSPP_E_INVAL, "check_points must be >= 2");
    // initializePath (include/sspp.h:82-97): linear via points at t_i = i / (n - 1)
    std::vector<double> u((size_t)n), pts((size_t)n * D), ctrl0((size_t)n * D);
    for (int i = 0; i < n; ++i) {
        const double t = (double)i / (n - 1);
        u[i] = t;
        for (int d = 0; d < D; ++d) pts[(size_t)i * D + d] = (1 - t) * start[d] + t * end[d];
    }
    if (sspp::interpolate(pts.data(), n, D, deg, u.data(), knots_out, ctrl0.data()) != 0)
        return sspp::set_error(SSPP_E_INVAL, "initializePath: interpolation failed");
    int rc;
    const size_t nd = (size_t)n * D;
    const int64_t B = sample_count;
    if (!p->plan_job.j || p->plan_n != n || p->plan_W != check_points || B > p->plan_cap) {
        p->plan_job.reset();
        sspp_sspp_args a{};
        a.knots = knots_out; a.degree = deg; a.init_ctrl = ctrl0.data(); a.n_ctrl = n; a.dof = D;
        a.sigma = sigma; a.limits = limits; a.check_points = check_points; a.seed = seed;
        // the hit-order pre-pass runs off this call's path (first plan() latency)
        if ((rc = sspp::job_create_sspp_async(p->scene, &a, B, &p->plan_job.j))) return rc;
        p->plan_n = n; p->plan_W = check_points; p->plan_cap = B;
        if ((rc = p->d_arc.reserve(B)) || (rc = p->d_feas.reserve(B)) || (rc = p->d_best.reserve(1)) ||
            (rc = p->d_ctrl.reserve(B * nd)) || (rc = p->h_arc.reserve(B)) || (rc = p->h_feas.reserve(B)) ||
            (rc = p->h_best.reserve(1)) || (rc = p->h_ctrl.reserve(B * nd))) {
            p->plan_job.reset();
            return rc;
        }
    } else if ((rc = sspp_job_update_sspp(p->plan_job.j, ctrl0.data(), sigma, limits, seed, p->stream))) {
        return rc;
    }
    // pinned_out: outputs straight into the mapped pinned buffers, control points of the
    // feasible candidates only; otherwise every candidate's outputs to device memory
    sspp::job_set_ctrl_feasible_only(p->plan_job.j, pinned_out ? 1 : 0);
    if (!pinned_out)
        return sspp_job_sample_score(p->plan_job.j, first_id, B, p->d_arc.p, p->d_feas.p,
                                     all_ctrl ? p->d_ctrl.p : nullptr, p->d_best.p, p->stream);
    // no device argmin here: findBestPath runs over the feasible rows in the host gather
    // (sspp_planner_plan), which saves the kernel's cross-workgroup argmin hand-off
    double* ha = p->h_arc.dev();
    unsigned char* hf = p->h_feas.dev();
    double* hc = p->h_ctrl.dev();
    if (!ha || !hf || !hc) return sspp::set_error(SSPP_E_HIP, "hipHostGetDevicePointer failed");
    return sspp_job_sample_score(p->plan_job.j, first_id, B, ha, hf, hc, nullptr, p->stream);
}

extern "C" int sspp_planner_plan(sspp_planner* p, const double* start, const double* end, double sigma,
                                 const double* limits, int sample_count, int check_points,
                                 int init_points, uint64_t seed, int64_t first_id, double* knots_out,
                                 int64_t* n_feasible, int64_t* feasible_ids, double* feasible_arc,
                                 double* feasible_ctrl, sspp_best* best_out) {
    sspp::clear_error();
    if (!p || !start || !end || !limits || !knots_out || !n_feasible || !best_out)
        return sspp::set_error(SSPP_E_INVAL, "sspp_planner_plan: null argument");
    int rc;
    if ((rc = plan_enqueue(p, start, end, sigma, limits, sample_count, check_points, init_points, seed,
                           first_id, knots_out, true)) ||
        (rc = hipck(hipStreamSynchronize(p->stream), "plan")))
        return rc;
    // the feasible candidates in candidate order (findBestPath's input, include/sspp.h:215-216)
    // and findBestPath itself (include/sspp.h:171-192): a path is taken when its arc length is
    // below the running minimum, which starts at +inf (an infinite or NaN arc is never taken);
    // ties to the lowest id (the first in candidate order) — the device argmin's (cost, id) order
    const size_t nd = (size_t)init_points * p->D;
    const unsigned char* f = p->h_feas.p;
    long long cnt = 0;
    double bc = INFINITY;
    int64_t bi = -1;
    for (int64_t i = 0; i < sample_count; ++i) {
        if (f[i] != 1) continue;
        const double a = p->h_arc.p[i];
        if (a < bc) { bc = a; bi = first_id + i; }
        if (feasible_ids) feasible_ids[cnt] = first_id + i;
        if (feasible_arc) feasible_arc[cnt] = a;
        if (feasible_ctrl) std::memcpy(feasible_ctrl + cnt * nd, p->h_ctrl.p + i * nd, sizeof(double) * nd);
        ++cnt;
    }
    *n_feasible = cnt;
    best_out->cost = bi < 0 ? INFINITY : bc;
    best_out->index = bi;
    best_out->count = cnt;
    best_out->reserved = 0;
    return SSPP_OK;
}

// ---- sspp_plan_sspp: the blocking all-candidates form of plan() on a cached planner per
// (scene, dof).  The cache lives for the process; sspp_scene_free drops a scene's planners.
namespace {
struct PlannerCache {
    std::mutex mu;  // one plan at a time through the cache (a planner is not re-entrant)
    struct Entry { const sspp_scene* scene; int D; sspp_planner* p; };
    std::vector<Entry> entries;
};
PlannerCache& planner_cache() {
    static PlannerCache* c = new PlannerCache();  // never destroyed: no teardown-order hazards
    return *c;
}
}  // namespace

void sspp::planner_cache_drop(const sspp_scene* scene) {
    PlannerCache& c = planner_cache();
    std::lock_guard<std::mutex> g(c.mu);
    for (size_t i = 0; i < c.entries.size();) {
        if (c.entries[i].scene == scene) {
            sspp_planner_free(c.entries[i].p);
            c.entries.erase(c.entries.begin() + i);
        } else {
            ++i;
        }
    }
}

extern "C" int sspp_plan_sspp(const sspp_scene* scene, int dof, const double* start,
                              const double* end, double sigma, const double* limits,
                              int sample_count, int check_points, int init_points, uint64_t seed,
                              double* knots_out, double* ctrl_out, uint8_t* feasible_out,
                              double* arc_out, sspp_best* best_out) {
    sspp::clear_error();
    if (!start || !end || !limits || !knots_out || !feasible_out || !arc_out || !best_out)
        return sspp::set_error(SSPP_E_INVAL, "sspp_plan_sspp: null argument");
    PlannerCache& c = planner_cache();
    std::lock_guard<std::mutex> g(c.mu);
    sspp_planner* p = nullptr;
    for (auto& e : c.entries)
        if (e.scene == scene && e.D == dof) p = e.p;
    int rc;
    if (!p) {
        if ((rc = sspp_planner_create(scene, dof, &p))) return rc;
        c.entries.push_back({scene, dof, p});
    }
    if ((rc = plan_enqueue(p, start, end, sigma, limits, sample_count, check_points, init_points, seed, 0,
                           knots_out, false, ctrl_out != nullptr)))
        return rc;
    // every candidate's outputs through the pinned staging (async copies, one stream sync)
    const int64_t B = sample_count;
    const size_t nd = (size_t)init_points * dof;
    if ((rc = p->h_sarc.reserve(B)) || (rc = p->h_sfeas.reserve(B)) || (rc = p->h_sbest.reserve(1)))
        return rc;
    if ((rc = hipck(hipMemcpyAsync(p->h_sarc.p, p->d_arc.p, sizeof(double) * B, hipMemcpyDeviceToHost, p->stream), "copy arc")) ||
        (rc = hipck(hipMemcpyAsync(p->h_sfeas.p, p->d_feas.p, (size_t)B, hipMemcpyDeviceToHost, p->stream), "copy feasible")) ||
        (rc = hipck(hipMemcpyAsync(p->h_sbest.p, p->d_best.p, sizeof(sspp_best), hipMemcpyDeviceToHost, p->stream), "copy best")) ||
        (ctrl_out && (rc = hipck(hipMemcpyAsync(p->h_ctrl.p, p->d_ctrl.p, sizeof(double) * B * nd,
                                                hipMemcpyDeviceToHost, p->stream), "copy ctrl"))) ||
        (rc = hipck(hipStreamSynchronize(p->stream), "plan")))
        return rc;
    std::memcpy(arc_out, p->h_sarc.p, sizeof(double) * B);
    std::memcpy(feasible_out, p->h_sfeas.p, (size_t)B);
    *best_out = *p->h_sbest.p;
    if ((rc = sspp_best_check(best_out, 1))) return rc;
    if (ctrl_out) std::memcpy(ctrl_out, p->h_ctrl.p, sizeof(double) * B * nd);
    return SSPP_OK;
}

extern "C" int sspp_planner_score(sspp_planner* p, const double* knots, int degree, const double* ctrl,
                                  int64_t B, int n, int W, int with_collision, double* arc_out,
                                  uint8_t* feasible_out, sspp_best* best_out) {
    sspp::clear_error();
    if (!p || !knots || !ctrl || B < 1 || n < degree + 1) return sspp::set_error(SSPP_E_INVAL, "sspp_planner_score: bad argument");
    const int D = p->D;
    const size_t nd = (size_t)n * D;
    const int nk = n + degree + 1;
    const int coll = with_collision && p->scene ? 1 : 0;
    int rc;
    const bool same = p->score_job.j && p->score_W == W && p->score_coll == coll && B <= p->score_cap &&
                      (int)p->score_knots.size() == nk &&
                      std::memcmp(p->score_knots.data(), knots, sizeof(double) * nk) == 0;
    if (!same) {
        p->score_job.reset();
        std::vector<double> ones((size_t)D, 1.0);
        sspp_sspp_args a{};
        a.knots = knots; a.degree = degree; a.init_ctrl = ctrl; a.n_ctrl = n; a.dof = D;
        a.sigma = 0.0; a.limits = ones.data(); a.check_points = W; a.seed = 0;
        if ((rc = sspp_job_create_sspp(coll ? p->scene : nullptr, &a, B, &p->score_job.j))) return rc;
        p->score_knots.assign(knots, knots + nk);
        p->score_W = W; p->score_coll = coll; p->score_cap = B;
        if ((rc = p->d_in.reserve(B * nd)) || (rc = p->h_in.reserve(B * nd)) || (rc = p->h_sarc.reserve(B)) ||
            (rc = p->h_sfeas.reserve(B)) || (rc = p->h_sbest.reserve(1)) || (rc = p->d_arc.reserve(B)) ||
            (rc = p->d_feas.reserve(B)) || (rc = p->d_best.reserve(1))) {
            p->score_job.reset();
            return rc;
        }
    }
    std::memcpy(p->h_in.p, ctrl, sizeof(double) * B * nd);
    if ((rc = hipck(hipMemcpyAsync(p->d_in.p, p->h_in.p, sizeof(double) * B * nd, hipMemcpyHostToDevice,
                                   p->stream), "copy splines")))
        return rc;
    if ((rc = sspp_job_score_ctrl(p->score_job.j, p->d_in.p, 0, B, p->d_arc.p, p->d_feas.p, p->d_best.p,
                                  p->stream)))
        return rc;
    if ((rc = hipck(hipMemcpyAsync(p->h_sarc.p, p->d_arc.p, sizeof(double) * B, hipMemcpyDeviceToHost, p->stream), "copy arc")) ||
        (rc = hipck(hipMemcpyAsync(p->h_sfeas.p, p->d_feas.p, (size_t)B, hipMemcpyDeviceToHost, p->stream), "copy feasible")) ||
        (rc = hipck(hipMemcpyAsync(p->h_sbest.p, p->d_best.p, sizeof(sspp_best), hipMemcpyDeviceToHost, p->stream), "copy best")) ||
        (rc = hipck(hipStreamSynchronize(p->stream), "score")))
        return rc;
    if (arc_out) std::memcpy(arc_out, p->h_sarc.p, sizeof(double) * B);
    if (feasible_out) std::memcpy(feasible_out, p->h_sfeas.p, (size_t)B);
    if (best_out) {
        *best_out = *p->h_sbest.p;
        if ((rc = sspp_best_check(best_out, 1))) return rc;
    }
    return SSPP_OK;
}
