// sspp_hostapi.cpp — host-synchronous conveniences over the job API (host buffers in/out).
//
// One-shot scoring / sampling of host splines (tests and the oracle comparisons); the blocking
// plan() form, sspp_plan_sspp, lives in planner.hip on a cached sspp_planner.  The candidate
// work still runs entirely in the HIP kernels; this file only stages buffers.
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <string>
#include <vector>

#include "model.h"

namespace {

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    int alloc(size_t bytes) {
        hipError_t e = hipMalloc(&p, bytes ? bytes : 8);
        if (e != hipSuccess)
            return sspp::set_error(SSPP_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        return SSPP_OK;
    }
};

int hipck(hipError_t e, const char* what) {
    if (e == hipSuccess) return SSPP_OK;
    return sspp::set_error(SSPP_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct JobGuard {
    sspp_job* j = nullptr;
    ~JobGuard() { if (j) sspp_job_free(j); }
};

// run a SamplingPathPlanner job on host buffers; ctrl_in (host) optional
int run_job_host(const sspp_scene* scene, const double* knots, int degree, const double* init_ctrl,
                 int n, int D, double sigma, const double* limits, int W, uint64_t seed,
                 int64_t first_id, int64_t B, const double* ctrl_in, double* ctrl_out,
                 double* arc_out, uint8_t* feasible_out, sspp_best* best_out) {
    sspp_sspp_args a{};
    std::vector<double> ones((size_t)D, 1.0);
    a.knots = knots; a.degree = degree; a.init_ctrl = init_ctrl; a.n_ctrl = n; a.dof = D;
    a.sigma = sigma; a.limits = limits ? limits : ones.data(); a.check_points = W; a.seed = seed;
    JobGuard jg;
    int rc = sspp_job_create_sspp(scene, &a, B, &jg.j);
    if (rc) return rc;
    const size_t nd = (size_t)n * D;
    DevBuf d_arc, d_feas, d_best, d_ctrl;
    if ((rc = d_arc.alloc(sizeof(double) * B)) || (rc = d_feas.alloc((size_t)B)) ||
        (rc = d_best.alloc(sizeof(sspp_best))))
        return rc;
    if (ctrl_in || ctrl_out) {
        if ((rc = d_ctrl.alloc(sizeof(double) * nd * B))) return rc;
    }
    if (ctrl_in) {
        if ((rc = hipck(hipMemcpy(d_ctrl.p, ctrl_in, sizeof(double) * nd * B, hipMemcpyHostToDevice), "copy ctrl")))
            return rc;
        rc = sspp_job_score_ctrl(jg.j, (const double*)d_ctrl.p, first_id, B, (double*)d_arc.p,
                                 (uint8_t*)d_feas.p, (sspp_best*)d_best.p, nullptr);
    } else {
        rc = sspp_job_sample_score(jg.j, first_id, B, (double*)d_arc.p, (uint8_t*)d_feas.p,
                                   ctrl_out ? (double*)d_ctrl.p : nullptr, (sspp_best*)d_best.p, nullptr);
    }
    if (rc) return rc;
    if ((rc = hipck(hipDeviceSynchronize(), "kernel"))) return rc;
    if (arc_out && (rc = hipck(hipMemcpy(arc_out, d_arc.p, sizeof(double) * B, hipMemcpyDeviceToHost), "copy arc")))
        return rc;
    if (feasible_out && (rc = hipck(hipMemcpy(feasible_out, d_feas.p, (size_t)B, hipMemcpyDeviceToHost), "copy feasible")))
        return rc;
    if (best_out && ((rc = hipck(hipMemcpy(best_out, d_best.p, sizeof(sspp_best), hipMemcpyDeviceToHost), "copy best")) ||
                     (rc = sspp_best_check(best_out, 1))))
        return rc;
    if (ctrl_out && !ctrl_in &&
        (rc = hipck(hipMemcpy(ctrl_out, d_ctrl.p, sizeof(double) * nd * B, hipMemcpyDeviceToHost), "copy ctrl")))
        return rc;
    return SSPP_OK;
}

}  // namespace

extern "C" int sspp_score_ctrl_host(const sspp_scene* scene, const double* knots, int degree,
                                    const double* ctrl, int64_t B, int n, int D, int W,
                                    double* arc_out, uint8_t* feasible_out, sspp_best* best_out) {
    sspp::clear_error();
    if (!knots || !ctrl || B < 1) return sspp::set_error(SSPP_E_INVAL, "sspp_score_ctrl_host: bad argument");
    return run_job_host(scene, knots, degree, ctrl, n, D, 0.0, nullptr, W, 0, 0, B, ctrl, nullptr,
                        arc_out, feasible_out, best_out);
}

extern "C" int sspp_sample_ctrl_host(const double* knots, int degree, const double* init_ctrl,
                                     int n, int D, double sigma, const double* limits,
                                     uint64_t seed, int64_t first_id, int64_t B, double* ctrl_out) {
    sspp::clear_error();
    if (!knots || !init_ctrl || !limits || !ctrl_out || B < 1)
        return sspp::set_error(SSPP_E_INVAL, "sspp_sample_ctrl_host: bad argument");
    return run_job_host(nullptr, knots, degree, init_ctrl, n, D, sigma, limits, 2, seed, first_id,
                        B, nullptr, ctrl_out, nullptr, nullptr, nullptr);
}
