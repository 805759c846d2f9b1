// model.h — host-side scene model (MuJoCo-like flat arrays) and shared host helpers.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/sspp_hip.h"

struct sspp_model {
    std::string path;
    std::vector<std::string> body_names, geom_names;
    std::vector<int32_t> body_parent, body_jnt_type, body_qpos_adr;
    std::vector<double> body_pos, body_quat;
    std::vector<int32_t> geom_type, geom_body, geom_contype, geom_conaffinity;
    std::vector<double> geom_size, geom_pos, geom_quat, geom_margin;
    std::vector<int32_t> exclude;
    std::vector<double> qpos0;
    int nbody() const { return (int)body_parent.size(); }
    int ngeom() const { return (int)geom_type.size(); }
};

namespace sspp {
// thread-local error message plumbing (sspp_last_error)
int set_error(int code, const std::string& msg);
void clear_error();

// MJCF -> model (mjcf.cpp)
int load_mjcf(const std::string& path, sspp_model& out);

// spline helpers (spline_host.cpp) — Eigen Splines semantics
void knot_averaging(const double* u, int n, int p, double* knots);
int span_of(double u, int p, const double* knots, int nknots);
void basis_funcs(double u, int p, const double* knots, int nknots, double* N);
int interpolate(const double* pts, int n, int D, int p, const double* u, double* knots,
                double* ctrl);
// Householder QR "program" of the collocation matrix for fixed parameters u (PathModel::fromVias
// precompute): [n][n] reflectors | [n] |v|^2 | [n][n] R; qr_apply replays it on B [n][D]
int qr_program(const double* u, int n, int p, double* knots, double* prog);
void qr_apply(const double* prog, int n, double* B, int D);

// CES slot-mode evaluation of a TaskSpacePlanner job (sspp_kernels.hip; used by ces.hip)
struct TspCesEval {
    const double* fixed;   // device [2][K][4]: mean set, forwarded best
    const int* nfixed;     // device: fixed slots in this iteration's list (1 or 2)
    const double* mean;    // device [K][4] sampling distribution
    const double* sigma;   // device [K][4]
    long long slot0;       // first slot evaluated by this call
    long long samples;     // random samples in the list
    long long first_id;    // Philox id of sample 0
    double start[4], end[4];
};
int tsp_eval_ces(sspp_job* j, const TspCesEval* e, int64_t n, double* d_L, double* d_Cnf,
                 double* d_Cwf, uint8_t* d_status, double* d_cost, double* d_vias_out,
                 void* stream);
// several goals' CES evaluations in one k_tsp_group launch (ces.hip sspp_ces_plan_group)
struct TspCesOut {
    double *L, *Cnf, *Cwf, *cost, *vias;
    uint8_t* status;
};
int tsp_eval_ces_group(sspp_job* const* jobs, const TspCesEval* evs, const TspCesOut* outs, int G, int64_t n,
                       void* stream);
// sspp_job_create_sspp with the hit-order pre-pass off the caller's path: the job starts in gap /
// bisection order and swaps in the hit order at the first launch after the pre-pass lands (the
// drop-in planner's first plan(), planner.hip; results are identical in every order)
int job_create_sspp_async(const sspp_scene* scene, const sspp_sspp_args* a, int64_t max_batch, sspp_job** out);
// k_sspp_c2f writes ctrl_out rows only for feasible candidates (drop-in planner, planner.hip)
void job_set_ctrl_feasible_only(sspp_job* j, int on);
// sspp_plan_sspp's cached planners (planner.hip): dropped when their scene is freed
void planner_cache_drop(const sspp_scene* scene);
// Process-wide HIP streams (created on first use, never destroyed): 0 = every drop-in planner's
// plan() stream, 1 = every job's asynchronous hit-order pre-pass.  A new stream can cost a new
// hardware queue (5.7 ms measured for a fresh planner's stream, the first in a process to need
// one: profiles/r06j_bench_dropin.json), so planners and pre-passes share these two
void* shared_stream(int which);  // a hipStream_t
}  // namespace sspp
