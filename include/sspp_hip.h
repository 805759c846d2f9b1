/*
 * sspp_hip.h — C ABI of the MI355X-native sampled-spline candidate scorer.
 *
 * This is the drop-in boundary underneath `from sspp import _sspp` (the pybind11 module
 * in sspp_amd/csrc/sspp_pybind.cpp) and any other FFI (ctypes stub in INTEGRATION.md).
 * Plain C types only: no torch, no Eigen, no MuJoCo.  All functions return an int status
 * (SSPP_OK = 0, negative on error) and set a thread-local message (sspp_last_error()).
 *
 * Each entry point names the reference interface it replaces (paths under the reference
 * repository Geryyy/sspp @ 2025-09-12):
 *
 *   sspp_model_load_mjcf     <- SamplingPathPlanner(const std::string&)  include/sspp.h:44-63
 *                               (mj_loadXML; restricted to free joints + plane/sphere/box/cylinder)
 *   sspp_model_body_point    <- Utility::get_body_point                  include/utility.h:228-259
 *   sspp_scene_create        <- SamplingPathPlanner::initializeDataCopies include/sspp.h:235-244
 *                               / tsp::CollisionWorld                     include/sspp/tsp_collision_world.h:12-41
 *   sspp_interpolate         <- SamplingPathPlanner::initializePath      include/sspp.h:82-97
 *                               (Eigen SplineFitting::Interpolate) and PathModel::fromVias
 *                               include/sspp/tsp_path_model.h:32-43
 *   sspp_spline_eval         <- SamplingPathPlanner::evaluate             include/sspp.h:99-107
 *   sspp_job_create_sspp     <- SamplingPathPlanner::plan (set-up part)   include/sspp.h:194-200
 *   sspp_job_sample_score    <- plan's candidate loop                     include/sspp.h:203-219
 *                               = sampleWithNoise (114-130) + checkCollision (132-150)
 *                               + computeArcLength (152-169) + findBestPath (171-192)
 *   sspp_job_score_ctrl      <- checkCollision + computeArcLength + findBestPath on
 *                               caller-supplied splines (sspp_bindings.cpp:36-41)
 *   sspp_job_create_tsp      <- tsp::Planner (evaluation config)          include/sspp/tsp_planner.h:31-51
 *   sspp_job_tsp_sample_score<- Planner::plan eval loop + best pick       include/sspp/tsp_planner.h:89-138
 *                               = Sampler::sample_set (tsp_sampler.h:40-51) + PathModel::fromVias
 *                               + Evaluator::eval_one_pass (tsp_evaluator.h:18-32)
 *   sspp_job_tsp_score_vias  <- the same on caller-supplied via sets
 *   sspp_ces_create          <- tsp::Planner(model, body, cfg, lo, hi, z_min)  tsp_planner.h:33-51
 *                               via tsp::TaskSpacePlanner's ctor                include/sspp/tsp.h:12-55
 *   sspp_ces_begin           <- Planner::plan prologue: reset() / initLinear   tsp_planner.h:54-75
 *                               + seed list (mean set, forwarded best)          tsp_planner.h:78-93
 *   sspp_ces_eval            <- Planner::plan evaluation loop                  tsp_planner.h:95-119
 *   sspp_ces_update          <- EliteSelector::select/weights                  tsp_elites.h:13-32
 *                               + Distribution::update/adapt                    tsp_distribution.h:31-83
 *                               + best pick / last_best_ forwarding             tsp_planner.h:121-142
 *   sspp_ces_plan            <- TaskSpacePlanner::plan(start, end, iterate)    include/sspp/tsp.h:58-60
 *                               (repeated `iterations` times, no host round trip)
 *   sspp_ces_read            <- successes()/failures()/sampled_sets()/mean()/sigma() getters
 *                               tsp_planner.h:151-158, tsp.h:63-78
 *
 * Device pointers: every `d_` argument is device memory (hipMalloc / torch.cuda); the job
 * run functions issue only asynchronous work on `stream` (hipStream_t passed as void*; NULL =
 * default stream), allocate nothing and never synchronise, so they can be captured into a
 * hipGraph.  Host pointers are read during the call only.
 */
#ifndef SSPP_HIP_H
#define SSPP_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SSPP_OK 0
#define SSPP_E_INVAL (-1)
#define SSPP_E_HIP (-2)
#define SSPP_E_SCENE (-3)
#define SSPP_E_NOMEM (-4)
#define SSPP_E_UNSUPPORTED (-5)
#define SSPP_E_IO (-6)
#define SSPP_E_INCOMPLETE (-7) /* a result record reports lost work (sspp_best::reserved != 0) */

/* MuJoCo mjtGeom codes for the supported primitives */
#define SSPP_GEOM_PLANE 0
#define SSPP_GEOM_SPHERE 2
#define SSPP_GEOM_CAPSULE 3
#define SSPP_GEOM_CYLINDER 5
#define SSPP_GEOM_BOX 6
#define SSPP_GEOM_MESH 7

#define SSPP_MODE_QPOS 0 /* SamplingPathPlanner: q (D values) -> qpos[0:D] */
#define SSPP_MODE_BODY 1 /* TaskSpacePlanner: (x,y,z,yaw) -> free body     */

typedef struct sspp_model sspp_model;
typedef struct sspp_scene sspp_scene;
typedef struct sspp_job sspp_job;

/* Flat, read-only view of a parsed model (MuJoCo-like arrays; body 0 = world). */
typedef struct sspp_model_view {
    int nbody;
    const int32_t* body_parent;
    const int32_t* body_jnt_type; /* -1 none, 0 free */
    const int32_t* body_qpos_adr;
    const double* body_pos;       /* [nbody][3] */
    const double* body_quat;      /* [nbody][4] normalised */
    int ngeom;
    const int32_t* geom_type;
    const int32_t* geom_body;
    const int32_t* geom_contype;
    const int32_t* geom_conaffinity;
    const double* geom_size;      /* [ngeom][3] */
    const double* geom_pos;       /* [ngeom][3] */
    const double* geom_quat;      /* [ngeom][4] */
    const double* geom_margin;
    int nexclude;
    const int32_t* exclude;       /* [nexclude][2] */
    int nq;
    const double* qpos0;
} sspp_model_view;

/* Result of one batch: global argmin over feasible candidates (lowest id on ties). */
typedef struct sspp_best {
    double cost;      /* +inf when no candidate is feasible */
    int64_t index;    /* global candidate id, -1 when none */
    int64_t count;    /* number of feasible candidates in the batch */
    int64_t reserved; /* candidates the launch could not finish: 0.  A split launch
                         (SSPP_OPT_SPLIT) counts its finished survivors against the reserved
                         queue slots and writes any shortfall here; the reductions below sum
                         it; every consumer of a record (sspp_best_check, sspp_best_reduce,
                         the planners, the Python layer) refuses a non-zero value with
                         SSPP_E_INCOMPLETE, because the step's outputs are then incomplete  */
} sspp_best;

typedef struct sspp_scene_info {
    int n_moving_geoms;
    int n_static_geoms;
    int n_pairs;            /* moving pairs evaluated per waypoint */
    int n_static_pairs;     /* env-env pairs (evaluated once at creation) */
    int static_contacts;    /* contacts among env-env pairs at qpos0 */
    int n_movers;
    double static_cost;     /* Collision.h cost of env-env contacts (per waypoint) */
} sspp_scene_info;

typedef struct sspp_sspp_args {
    const double* knots;    /* host [n + degree + 1] */
    int degree;
    const double* init_ctrl;/* host [n][dof] */
    int n_ctrl;
    int dof;
    double sigma;
    const double* limits;   /* host [dof] */
    int check_points;       /* W: collision at i/W, i=0..W; arc on W points */
    uint64_t seed;
    int arc_all;            /* 0 (reference): arc length only for collision-free candidates
                               (findBestPath, include/sspp.h:171-192), +inf for the others;
                               1: arc length for every candidate                         */
    int sampler;            /* 0 (default): FP64 Box-Muller normals, as the reference's
                               std::normal_distribution<double> (include/sspp.h:116,125);
                               1: opt-in FP32 Box-Muller quads (faster, |z| <= 5.77)     */
} sspp_sspp_args;

typedef struct sspp_tsp_args {
    const double* start;    /* host [4] (x, y, z, yaw) */
    const double* end;      /* host [4] */
    int n_vias;             /* K (total_points - 2) */
    int check_points;       /* cp */
    double w_collision;
    const double* mean;     /* host [K][4] sampling mean (Distribution::mean_vias) */
    const double* sigma;    /* host [K][4] */
    const double* lo;       /* host [4] Sampler limits_min */
    const double* hi;       /* host [4] Sampler limits_max */
    double z_min;           /* PlannerConfig::z_min (sample_set clamp) */
    uint64_t seed;
    double floor_z_min, floor_margin, floor_scale; /* Evaluator (0, 0.01, 10) */
} sspp_tsp_args;

const char* sspp_last_error(void);
int sspp_version(void);
/* Source revision the library was built from (16 hex digits of sspp_amd/_stamp.py's hash of
 * sspp_amd/csrc/ + this header); the Python layer refuses a profiling variant whose revision
 * differs from the tree it runs in.  No reference counterpart (build hygiene only). */
const char* sspp_build_id(void);
int sspp_device_count(int* n);

/* ---- model ---- */
int sspp_model_load_mjcf(const char* xml_path, sspp_model** out);
int sspp_model_view_get(const sspp_model* m, sspp_model_view* out);
int sspp_model_body_id(const sspp_model* m, const char* name);
int sspp_model_geom_id(const sspp_model* m, const char* name);
int sspp_model_body_point(const sspp_model* m, const char* name, double out_xyzyaw[4]);
void sspp_model_free(sspp_model* m);

/* ---- scene (model + moving set, device-resident tables) ---- */
int sspp_scene_create(const sspp_model* m, int mode, int arg /* dof or body id */,
                      int count_static_contacts, sspp_scene** out);
int sspp_scene_get_info(const sspp_scene* s, sspp_scene_info* out);
void sspp_scene_free(sspp_scene* s);

/* ---- splines (host) ---- */
int sspp_interpolate(const double* pts /* [n][D] */, int n, int D, int degree,
                     const double* u /* [n] */, double* knots_out /* [n+degree+1] */,
                     double* ctrl_out /* [n][D] */);
int sspp_spline_eval(const double* knots, int n_knots, int degree, const double* ctrl /* [n][D] */,
                     int D, double u, double* out /* [D] */);

/* ---- SamplingPathPlanner job ---- */
int sspp_job_create_sspp(const sspp_scene* scene /* NULL = no collision */,
                         const sspp_sspp_args* args, int64_t max_batch, sspp_job** out);
int sspp_job_sample_score(sspp_job* job, int64_t first_id, int64_t B, double* d_arc,
                          uint8_t* d_feasible, double* d_ctrl_out /* nullable [B][n][D] */,
                          sspp_best* d_best, void* stream);
int sspp_job_score_ctrl(sspp_job* job, const double* d_ctrl /* [B][n][D] */, int64_t first_id,
                        int64_t B, double* d_arc, uint8_t* d_feasible, sspp_best* d_best,
                        void* stream);

/* ---- TaskSpacePlanner job ---- */
int sspp_job_create_tsp(const sspp_scene* scene, const sspp_tsp_args* args, int64_t max_batch,
                        sspp_job** out);
int sspp_job_tsp_sample_score(sspp_job* job, int64_t first_id, int64_t B, double* d_L,
                              double* d_Cnf, double* d_Cwf, uint8_t* d_status, double* d_cost,
                              double* d_vias_out /* nullable [B][K][4] */, sspp_best* d_best,
                              void* stream);
int sspp_job_tsp_score_vias(sspp_job* job, const double* d_vias /* [B][K][4] */,
                            int64_t first_id, int64_t B, double* d_L, double* d_Cnf,
                            double* d_Cwf, uint8_t* d_status, double* d_cost, sspp_best* d_best,
                            void* stream);
/* SamplingPathPlanner jobs: the last (or, before any launch, the throughput) k_sspp_c2f shape —
 * lanes_per_candidate = phase-1 lanes G1; TaskSpacePlanner jobs: k_tsp's lanes per candidate */
int sspp_job_info(const sspp_job* job, int* lanes_per_candidate, int* candidates_per_block,
                  int* block_threads, size_t* lds_bytes);
void sspp_job_free(sspp_job* job);

/* Explicit job options (tests and tuning; the library reads no environment variables).
 * Nothing here changes a result: every option selects among bit-identical evaluation orders or
 * kernel forms.  sspp_job_get_option also reads back the effective configuration.          */
#define SSPP_OPT_SHAPE_NT 1     /* k_sspp_c2f threads per workgroup: 64, 128 or 256; 0 = per launch */
#define SSPP_OPT_SHAPE_G1 2     /* phase-1 lanes per candidate 1..64; 0 = per launch.  A launch
                                   whose (NT / 64) * (64 / G1) exceeds 64 candidates per workgroup
                                   (e.g. 128 x 1, 256 x 2) fails with SSPP_E_INVAL            */
#define SSPP_OPT_ORDER 3        /* scan order: 0 scene / bisection, 1 mean-path gap (pairs),
                                   2 hit order (waypoints + pairs, host pre-pass; the default of
                                   sampled jobs, sigma > 0); setting it rebuilds the tables
                                   (synchronous)                                               */
#define SSPP_OPT_TSP_FORM 4     /* TaskSpacePlanner: -1 by batch size, 0 k_tsp, 1 k_tsp_pp,
                                   2 k_tsp_pp2, 3 k_tsp with box-box polygons deferred to the
                                   workgroup (<= 8 pairs), 4 deferred to the end of each lane's
                                   pair loop (<= 64 pairs); get: the last launch's form        */
#define SSPP_OPT_TSP_GENERIC 5  /* TaskSpacePlanner: 1 = generic box-box / cylinder-box code even
                                   where every pair is upright                                 */
#define SSPP_OPT_SAMPLER 6      /* get: the job's sampler (sspp_sspp_args::sampler)             */
#define SSPP_OPT_LAST_NT 7      /* get: threads per workgroup of the last k_sspp_c2f launch     */
#define SSPP_OPT_LAST_G1 8      /* get: phase-1 lanes per candidate of that launch              */
#define SSPP_OPT_WP_ORDER 9     /* get: collision-waypoint order (0 bisection, 2 hit order)     */
#define SSPP_OPT_PREPASS_US 10  /* get: host microseconds of the creation's hit-order pre-pass  */
#define SSPP_OPT_NPAIRS 11      /* get: pairs in the sampled-candidate table                    */
#define SSPP_OPT_CYLBOX 12      /* get: that table has cylinder-box pairs (k_sspp_c2f settles them) */
#define SSPP_OPT_F32 13         /* k_sspp_c2f's FP32-filtered scan: 1 (default) on, 0 all-FP64.
                                   The filter only settles what FP64 settles the same way, so the
                                   results are identical either way               */
#define SSPP_OPT_LAST_F32 14    /* get: the last k_sspp_c2f launch ran the filtered scan         */
#define SSPP_OPT_CREATE_US 15   /* get: host microseconds of the job's creation                  */
#define SSPP_OPT_PREPASS_STATE 16 /* get: asynchronous hit-order pre-pass (the drop-in planner's
                                   jobs): 0 none, 1 running, 2 landed, 3 applied / dropped      */
#define SSPP_OPT_SPLIT 17       /* multi-step launches of >= 16384 sampled candidates that fit one
                                   resident round (single-geom movers, no cylinder-box pairs): 1
                                   (default) k_sspp_c2f's workgroups queue their phase-1 survivors
                                   and finish queued survivors, whoever sampled them; 0 each
                                   workgroup finishes its own.  Results identical either way      */
#define SSPP_OPT_LAST_SPLIT 18  /* get: the last launch was split                                */
#define SSPP_OPT_SPLIT_LINGER_US 20 /* split launches: microseconds a ticket waits for a slot that is
                                   not reserved yet before it hands the slot to the launch's last
                                   workgroup (default 10000; 0 = at once: tests).  Results
                                   identical for every value                                     */
#define SSPP_OPT_SPLIT_DROP 21  /* tests only: 1 = the last workgroup drops handed-over slots
                                   instead of finishing them, so the lost-work check must fire  */
#define SSPP_OPT_SPLIT_HANDOFFS 22 /* get (synchronous): slots handed to last workgroups so far */
#define SSPP_OPT_SPLIT_LOST 23  /* get (synchronous): survivors lost so far (0 unless DROP)     */
#define SSPP_OPT_TSP_REP 19     /* TaskSpacePlanner k_tsp form 3: sub-batches of candidates
                                   per workgroup (one prologue for all of them), 1..16, -1 by batch
                                   size; get: the last k_tsp launch's                            */
int sspp_job_set_option(sspp_job* job, int key, int64_t value);
int sspp_job_get_option(const sspp_job* job, int key, int64_t* value);

/* ---- TaskSpacePlanner CES iteration on the device (tsp::Planner::plan) ----
 * An iteration's candidate list is [mean set, forwarded best (iterate && last_best), samples]
 * (n_fixed + samples slots; ranks own slots_per_rank consecutive slots each).  All state
 * (distribution, last best, per-slot results) stays on the device; sspp_ces_read copies it
 * out synchronously.  Random samples of iteration t use Philox ids t * samples + [0, samples). */
typedef struct sspp_ces sspp_ces;
typedef struct sspp_ces_config {
    int samples;            /* PlannerConfig::samples (sample_count)                      */
    int checks;             /* check_points                                              */
    int total_points;       /* init_points (start + K vias + end), 3..34                 */
    double w_collision, elite_fraction, inc, dec;
    double sigma_floor, var_beta, mean_lr, stddev_min, stddev_max;
    double z_min;           /* PlannerConfig::z_min: seed / sample z clamp               */
    double dist_z_min;      /* Distribution::z_min — TaskSpacePlanner passes stddev_initial
                               here (tsp.h:53 -> tsp_planner.h:45)             */
    double sigma0;          /* Planner::sigma0_ = 0.3 (tsp_planner.h:177)                 */
    const double* lo;       /* host [4] limits_min (Sampler + Distribution bounds)       */
    const double* hi;       /* host [4] limits_max                                       */
    double floor_z_min, floor_margin, floor_scale; /* Evaluator (0, 0.01, 10)  */
    uint64_t seed;
} sspp_ces_config;
typedef struct sspp_ces_info {
    int n_vias, n_slots, slots_per_rank, world, elite_capacity;
    int64_t iteration;
} sspp_ces_info;
typedef struct sspp_ces_state {
    int n_fixed;            /* 1 (mean set) or 2 (+ forwarded best) in the last list     */
    int n_candidates;       /* n_fixed + samples                                          */
    int n_success, n_elite, has_best;
    int64_t best_slot;      /* slot of the last update's best, -1 if no success          */
    double best_cost;
    int64_t iteration;      /* completed updates                                          */
} sspp_ces_state;
typedef struct sspp_ces_buffers {   /* device pointers, n_slots entries (vias: [n_slots][K][4]) */
    double *L, *C_nf, *C_wf, *cost;
    uint8_t* status;        /* 1 = SolverStatus::Converged (C_nf == 0.0)                  */
    double* vias;
    double *mean, *sigma, *last_best;  /* [K][4] */
    int32_t* elites;        /* slots of the last update's elites, best first             */
} sspp_ces_buffers;
int sspp_ces_create(const sspp_scene* scene /* SSPP_MODE_BODY */, const sspp_ces_config* cfg,
                    int world, sspp_ces** out);
int sspp_ces_get_info(const sspp_ces* ces, sspp_ces_info* out);
int sspp_ces_begin(sspp_ces* ces, const double* start /* [4] */, const double* end /* [4] */,
                   int iterate, void* stream);
int sspp_ces_eval(sspp_ces* ces, int rank, void* stream);  /* this rank's slots */
int sspp_ces_update(sspp_ces* ces, void* stream);           /* needs every slot's results */
int sspp_ces_plan(sspp_ces* ces, const double* start, const double* end, int iterate,
                  int iterations, void* stream);            /* world == 1 */
/* multi-goal: iterations x sspp_ces_plan of G <= 16 single-rank planners (starts / ends: [G][4])
 * as one chain of batched launches on `stream` (one k_tsp_group evaluation per iteration over
 * every goal's slots).  Each planner's results equal sspp_ces_plan on it alone.  Planners that
 * differ in scene, vias, checks, bounds or CES configuration run one by one.  No reference
 * counterpart: BASELINE configs[4] is build-defined.                      */
int sspp_ces_plan_group(sspp_ces* const* ces, int G, const double* starts, const double* ends, int iterate,
                        int iterations, void* stream);
int sspp_ces_get_buffers(const sspp_ces* ces, sspp_ces_buffers* out);
/* multi-rank exchange: this rank's slots_per_rank slots as packed f64 records
 * [L, C_nf, C_wf, cost, status, vias(4K)] (5 + 4K doubles each) into d_out; unpack scatters
 * the all-gathered records of every rank (n_slots records) into the planner's arrays.     */
int sspp_ces_pack(const sspp_ces* ces, int rank, double* d_out, void* stream);
int sspp_ces_unpack(sspp_ces* ces, const double* d_in, void* stream);
int sspp_ces_read(sspp_ces* ces, sspp_ces_state* state, double* L, double* C_nf, double* C_wf,
                  double* cost, uint8_t* status, double* vias, double* mean, double* sigma,
                  double* last_best, int32_t* elites);     /* synchronous; outputs nullable */
int sspp_ces_set_state(sspp_ces* ces, const double* mean, const double* sigma,
                       const double* last_best, int has_best /* -1 = keep */);
/* SSPP_OPT_CES_FUSED: 1 (default) small slot lists rank their successes inside k_ces_update
 * (3 launches per iteration), 0 the rank / scatter kernels (5 launches); bit-identical.     */
#define SSPP_OPT_CES_FUSED 101
int sspp_ces_set_option(sspp_ces* ces, int key, int64_t value);
void sspp_ces_free(sspp_ces* ces);

/* Re-target a SamplingPathPlanner job (same knots, dof, check_points) to new initial control
 * points / sigma / limits / seed: asynchronous uploads on `stream` (the job keeps the host
 * staging alive until its next update).  Used by the cached drop-in planner below.         */
int sspp_job_update_sspp(sspp_job* job, const double* init_ctrl /* [n][D] */, double sigma,
                         const double* limits /* [D] */, uint64_t seed, void* stream);

/* ---- drop-in planner: SamplingPathPlanner<N> state kept on the device across calls ----
 * One object per `_sspp.SamplingPathPlannerN` (src/sspp_bindings.cpp:24-50): it owns a HIP
 * stream, the job of the last plan() shape (init_points, check_points, capacity) and the
 * device / pinned buffers, so a plan() call is: initializePath on the host, an asynchronous
 * job update (skipped when the query repeats), one scoring launch that writes arc lengths,
 * feasibility, the argmin record and the feasible candidates' control points straight into
 * mapped pinned host memory, one stream synchronisation, and a host gather of the feasible
 * rows in candidate order.  Not re-entrant per object (as the reference's planner).
 *   sspp_planner_plan  <- SamplingPathPlanner::plan (include/sspp.h:194-225): writes
 *     knots [init_points+4], *n_feasible, feasible ids (first_id + index) / arc / ctrl
 *     [n_feasible][n][D] (caller buffers sized for sample_count) and the argmin record.
 *   sspp_planner_score <- checkCollision / computeArcLength / findBestPath on host splines
 *     sharing one knot vector (include/sspp.h:132-192); with_collision = 0: arc length only. */
typedef struct sspp_planner sspp_planner;
int sspp_planner_create(const sspp_scene* scene, int dof, sspp_planner** out);
int sspp_planner_plan(sspp_planner* p, const double* start, const double* end, double sigma,
                      const double* limits, int sample_count, int check_points, int init_points,
                      uint64_t seed, int64_t first_id, double* knots_out, int64_t* n_feasible,
                      int64_t* feasible_ids, double* feasible_arc, double* feasible_ctrl,
                      sspp_best* best_out);
int sspp_planner_score(sspp_planner* p, const double* knots, int degree,
                       const double* ctrl /* [B][n][D] */, int64_t B, int n, int W, int with_collision,
                       double* arc_out, uint8_t* feasible_out, sspp_best* best_out);
void sspp_planner_free(sspp_planner* p);
/* sspp_job_get_option on the planner's plan() job (its effective configuration; tests) */
int sspp_planner_get_option(const sspp_planner* p, int key, int64_t* value);

/* ---- step executor: a planning loop's back-to-back batches in one call ----
 * Enqueues nsteps independent SamplingPathPlanner steps (each = one plan() batch of B
 * candidates: sampleWithNoise + checkCollision + computeArcLength + findBestPath,
 * include/sspp.h:194-225).  Step i scores candidate ids [first_id + i * step_stride, ... + B)
 * and writes its own argmin record to d_best[i] (nullable).  Steps are grouped
 * steps_per_launch (1..64) to a kernel launch — each step keeps its own workgroups, outputs and
 * argmin — and launch l goes to branch l % nbranch: jobs[b] (distinct jobs: each owns its argmin
 * counters), streams[b], scratch outputs d_arc[b] / d_feasible[b] of steps_per_launch * B
 * entries.  Asynchronous.                                                                  */
int sspp_steps_enqueue_sspp(sspp_job* const* jobs, int nbranch, void* const* streams, int64_t B,
                            int nsteps, int steps_per_launch, int64_t first_id,
                            int64_t step_stride, double* const* d_arc, uint8_t* const* d_feasible,
                            sspp_best* d_best);
/* The same executor as a handle (a planning loop's per-call arguments are only the steps):
 * sspp_steps_create_sspp checks and copies the branches once; sspp_steps_run(ex, nsteps, first_id,
 * step_stride, d_best) enqueues like sspp_steps_enqueue_sspp; the jobs, streams and buffers must
 * outlive the handle.                                                                      */
typedef struct sspp_steps sspp_steps;
int sspp_steps_create_sspp(sspp_job* const* jobs, int nbranch, void* const* streams, int64_t B,
                           int steps_per_launch, double* const* d_arc, uint8_t* const* d_feasible,
                           sspp_steps** out);
int sspp_steps_run(sspp_steps* ex, int nsteps, int64_t first_id, int64_t step_stride, sspp_best* d_best);
void sspp_steps_free(sspp_steps* ex);

/* ---- multi-GPU helpers: reduce gathered per-rank results (lowest cost, lowest id) ---- */
int sspp_best_reduce(const sspp_best* parts, int n, sspp_best* out);          /* host */
/* SSPP_OK, or SSPP_E_INCOMPLETE when any of the n records reports lost work (reserved != 0) */
int sspp_best_check(const sspp_best* recs, int n);                            /* host */
int sspp_best_reduce_device(const sspp_best* d_parts, int n, sspp_best* d_out,
                            void* stream);                                    /* device, async */
/* G steps gathered from R ranks: d_parts [R][G] -> d_out [G] (device, async)              */
int sspp_best_reduce_steps(const sspp_best* d_parts, int R, int G, sspp_best* d_out,
                           void* stream);

/* ---- host-synchronous conveniences (host buffers in/out; used by the _sspp drop-in) ----
 * sspp_plan_sspp  <- SamplingPathPlanner::plan (include/sspp.h:194-225) in one call:
 *   initializePath (linear vias, degree 3, init_points) + sample_count candidates scored on the
 *   GPU.  Outputs: knots [init_points+4], ctrl [sample_count][init_points][dof] (nullable),
 *   feasible [sample_count], arc [sample_count], best.  Runs on a process-wide sspp_planner
 *   cached per (scene, dof) — job, buffers and stream reused, async copies into pinned memory
 *   and one stream synchronisation per call; calls are serialised by a mutex;
 *   sspp_scene_free releases the scene's cached planners.                                */
int sspp_plan_sspp(const sspp_scene* scene, int dof, const double* start, const double* end,
                   double sigma, const double* limits, int sample_count, int check_points,
                   int init_points, uint64_t seed, double* knots_out, double* ctrl_out,
                   uint8_t* feasible_out, double* arc_out, sspp_best* best_out);
/* checkCollision / computeArcLength / findBestPath on host splines sharing one knot vector:
 * scene NULL = arc length only (everything feasible).                                    */
int sspp_score_ctrl_host(const sspp_scene* scene, const double* knots, int degree,
                         const double* ctrl /* [B][n][D] */, int64_t B, int n, int D, int W,
                         double* arc_out, uint8_t* feasible_out, sspp_best* best_out);
/* sampleWithNoise (include/sspp.h:114-130) for candidate ids [first_id, first_id + B). */
int sspp_sample_ctrl_host(const double* knots, int degree, const double* init_ctrl, int n, int D,
                          double sigma, const double* limits, uint64_t seed, int64_t first_id,
                          int64_t B, double* ctrl_out /* [B][n][D] */);

#ifdef __cplusplus
}
#endif
#endif
