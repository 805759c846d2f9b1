// sspp_hostapi.cpp — host-synchronous conveniences over the job API (host buffers in/out).
//
// These back the pybind11 drop-in (`from sspp import _sspp`): the reference's plan() is a
// blocking call on host data (include/sspp.h:194-225, bound at src/sspp_bindings.cpp:43-50).
// The candidate work still runs entirely in the HIP kernels; this file only stages buffers.
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
    if (best_out && (rc = hipck(hipMemcpy(best_out, d_best.p, sizeof(sspp_best), hipMemcpyDeviceToHost), "copy best")))
        return rc;
    if (ctrl_out && !ctrl_in &&
        (rc = hipck(hipMemcpy(ctrl_out, d_ctrl.p, sizeof(double) * nd * B, hipMemcpyDeviceToHost), "copy ctrl")))
        return rc;
    return SSPP_OK;
}

}  // namespace

extern "C" int sspp_plan_sspp(const sspp_scene* scene, int dof, const double* start,
                              const double* end, double sigma, const double* limits,
                              int sample_count, int check_points, int init_points, uint64_t seed,
                              double* knots_out, double* ctrl_out, uint8_t* feasible_out,
                              double* arc_out, sspp_best* best_out) {
    sspp::clear_error();
    if (!start || !end || !limits || !knots_out || !feasible_out || !arc_out || !best_out)
        return sspp::set_error(SSPP_E_INVAL, "sspp_plan_sspp: null argument");
    if (sample_count < 1) return sspp::set_error(SSPP_E_INVAL, "sample_count must be >= 1");
    const int n = init_points, p = 3;
    if (n < p + 1) return sspp::set_error(SSPP_E_INVAL, "init_points must be >= 4 for a cubic spline");
    // initializePath (include/sspp.h:82-97): linear via points at t_i = i/(n-1)
    std::vector<double> u((size_t)n), pts((size_t)n * dof), ctrl0((size_t)n * dof);
    for (int i = 0; i < n; ++i) {
        double t = (double)i / (n - 1);
        u[i] = t;
        for (int d = 0; d < dof; ++d) pts[(size_t)i * dof + d] = (1 - t) * start[d] + t * end[d];
    }
    if (sspp::interpolate(pts.data(), n, dof, p, u.data(), knots_out, ctrl0.data()) != 0)
        return sspp::set_error(SSPP_E_INVAL, "initializePath: interpolation failed");
    return run_job_host(scene, knots_out, p, ctrl0.data(), n, dof, sigma, limits, check_points,
                        seed, 0, sample_count, nullptr, ctrl_out, arc_out, feasible_out, best_out);
}

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
