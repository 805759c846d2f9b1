/*
 * sspp_oracle.h — CPU restatement of Geryyy/sspp's candidate-scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (sspp_amd/, sspp/, include/)
 * links, imports or calls this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * What it restates (reference paths relative to /root/reference):
 *   include/sspp.h:82-97     SamplingPathPlanner::initializePath   (Eigen SplineFitting::Interpolate)
 *   include/sspp.h:114-130   sampleWithNoise                      (RNG replaced by Philox)
 *   include/sspp.h:132-150   checkCollision                       (mj_forward + ncon>0, restated)
 *   include/sspp.h:152-169   computeArcLength
 *   include/sspp.h:171-192   findBestPath                         (lowest index on ties)
 *   include/Collision.h:84-103  collision_point_cost
 *   include/utility.h:149-206   mj_set_point / yaw_to_quat
 *   include/sspp/tsp_path_model.h:32-43  PathModel::fromVias
 *   include/sspp/tsp_evaluator.h:10-32   floorPenalty / eval_one_pass
 *   include/sspp/tsp_sampler.h:12-51     Sampler::sample / sample_set (RNG replaced by Philox)
 *   sspp/BSplines.py:11-62   B / bspline / knot_vector (Cox–de Boor, Python reference)
 *
 * Third-party arithmetic restated (absent from /root/reference, versions unpinned there):
 *   Eigen3 unsupported/Eigen/Splines: KnotAveraging, Spline::Span (Piegl–Tiller A2.1),
 *     Spline::BasisFunctions (A2.2), Spline::operator(), SplineFitting::Interpolate
 *     (collocation matrix + HouseholderQR solve).
 *   MuJoCo mj_kinematics (free joint -> body tree -> geom frames, mju_normalize4,
 *     mju_mulQuat, mju_quat2Mat), mj_collision pair filter (contype/conaffinity,
 *     weld bodies, parent filter, <exclude>), bounding-sphere broadphase with margin,
 *     and primitive narrowphase (semantics defined in DESIGN.md §Collision semantics).
 *   Parity with Eigen and MuJoCo themselves is UNPINNED (neither is available offline);
 *   the spline part is pinned by the reference's own BSplines.py golden vectors and
 *   closed-form known answers, the collision part by hand-computed known answers.
 */
#ifndef SSPP_ORACLE_H
#define SSPP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_GEOM_PLANE = 0, OR_GEOM_SPHERE = 2, OR_GEOM_CAPSULE = 3, OR_GEOM_CYLINDER = 5, OR_GEOM_BOX = 6 };
enum { OR_JNT_NONE = -1, OR_JNT_FREE = 0 };

/* Flat model (MuJoCo-like).  Body 0 is the world body.  body_parent[i] < i. */
typedef struct or_model {
    int nbody;
    const int32_t* body_parent;
    const int32_t* body_jnt_type;   /* OR_JNT_NONE or OR_JNT_FREE */
    const int32_t* body_qpos_adr;   /* for free joints */
    const double*  body_pos;        /* [nbody][3] relative to parent */
    const double*  body_quat;       /* [nbody][4] relative to parent (normalised) */
    int ngeom;
    const int32_t* geom_type;
    const int32_t* geom_body;
    const int32_t* geom_contype;
    const int32_t* geom_conaffinity;
    const double*  geom_size;       /* [ngeom][3] */
    const double*  geom_pos;        /* [ngeom][3] in body frame */
    const double*  geom_quat;       /* [ngeom][4] in body frame */
    const double*  geom_margin;     /* [ngeom] */
    int nexclude;
    const int32_t* exclude;         /* [nexclude][2] body ids */
    int nq;
    const double*  qpos0;           /* [nq] */
} or_model;

typedef struct or_scene or_scene;

/* mode: 0 = sspp window (q -> qpos[0:dof]), 1 = free body point (x,y,z,yaw) */
or_scene* or_scene_create(const or_model* m, int mode, int arg /* dof or body id */);
void      or_scene_destroy(or_scene* s);
int       or_scene_npairs(const or_scene* s, int* n_moving, int* n_static);

/* ---- splines (Eigen semantics) ---- */
void   or_knot_averaging(const double* u, int n, int p, double* knots /* n+p+1 */);
int    or_span(double u, int p, const double* knots, int nknots);
void   or_basis(double u, int p, const double* knots, int nknots, double* N /* p+1 */);
void   or_spline_eval(const double* knots, int nknots, int p, const double* ctrl /* [n][D] */,
                      int D, double u, double* out);
int    or_interpolate(const double* pts /* [n][D] */, int n, int D, int p, const double* u,
                      double* knots, double* ctrl);
/* ---- Python BSplines.py semantics ---- */
void   or_py_knot_vector(int n, int k, double* t /* n+k+1 */);
double or_py_B(double theta, int k, int i, const double* t);
void   or_py_bspline(double theta, const double* t, int nt, const double* c /* [n][D] */, int D,
                     int k, double* out);

/* ---- counter-based RNG (replaces std::default_random_engine) ---- */
void   or_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void   or_normal_quad(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream, double z[4]);
void   or_normal_pair(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream,
                      double* z0, double* z1);
void   or_normal_pair_libm(uint64_t seed, uint64_t cand, uint32_t idx, uint32_t stream,
                           double* z0, double* z1);
/* sampleWithNoise for candidates [first, first+B): ctrl_out [B][n][D]; sampler 0 = FP64 pairs
   (default), 1 = FP32 quads (opt-in) */
void   or_sample_sspp(const double* init_ctrl, int n, int D, int p, double sigma,
                      const double* limits, uint64_t seed, int64_t first, int64_t B,
                      double* ctrl_out, int sampler);
/* Sampler::sample_set: vias_out [B][K][4] */
void   or_sample_tsp(const double* mean /* [K][4] */, const double* sigma /* [K][4] */, int K,
                     const double* lo, const double* hi, double z_min, uint64_t seed,
                     int64_t first, int64_t B, double* vias_out);

/* ---- collision / FK ---- */
/* q: dof values (mode 0) or (x,y,z,yaw) (mode 1).  Returns contact count (all pairs
   that are counted in this mode); deep_cost receives the Collision.h cost. */
int    or_point_contacts(const or_scene* s, const double* q, int count_static,
                         double* deep_cost, int* n_deep);
/* analysis hook: per-pair contact counts at q (counts/g1/g2 [npair]); returns npair */
int    or_point_pair_contacts(const or_scene* s, const double* q, int* counts, int* g1, int* g2);
/* geom world poses after FK for q (test hook). xpos [ngeom][3], xmat [ngeom][9] */
void   or_fk_geoms(const or_scene* s, const double* q, double* xpos, double* xmat);

/* ---- canonical reduction order shared with the GPU kernels ---- */
double or_canon_sum(const double* x, int n, int lanes);
int    or_lanes_for(int items);

/* ---- SamplingPathPlanner scoring ---- */
int    or_sspp_score(const or_scene* s /* NULL = no collision */, const double* knots, int nknots,
                     int p, const double* ctrl /* [B][n][D] */, int n, int D, int64_t B, int W,
                     int count_static, int sequential_sum, int nthreads,
                     int arc_all /* 0: +inf for colliding candidates (findBestPath) */,
                     double* arc_out, uint8_t* feasible_out);
int64_t or_argmin(const double* cost, const uint8_t* feasible, int64_t B, double* best_cost);

/* ---- TaskSpacePlanner scoring ---- */
int    or_tsp_score(const or_scene* s, const double* start, const double* end,
                    const double* vias /* [B][K][4] */, int K, int64_t B, int cp,
                    double w_collision, int sequential_sum, int nthreads,
                    double* L, double* Cnf, double* Cwf, uint8_t* status, double* cost);
int64_t or_tsp_best(const double* cost, const uint8_t* status, int64_t B, double* best_cost);

/* ---- TaskSpacePlanner CES update (tsp_planner.h:121-142, tsp_elites.h, tsp_distribution.h) ---- */
typedef struct or_ces_cfg {
    int K;
    double frac, inc, dec, sigma_floor, var_beta, mean_lr, sd_min, sd_max, dist_z_min;
    double lo[4], hi[4];
    int sequential;   /* 1: reference summation order; 0: GPU canonical wave order */
} or_ces_cfg;
/* in/out: mean, sigma, last_best [K][4], has_best; out: elites (slots, best first), n_elite,
   best_slot (-1 if no success).  Returns the number of successes. */
int    or_ces_update(const or_ces_cfg* c, const double* cost, const uint8_t* status,
                     const double* vias /* [n][K][4] */, int64_t n, double* mean, double* sigma,
                     double* last_best, int* has_best, int32_t* elites, int* n_elite,
                     int64_t* best_slot);

#ifdef __cplusplus
}
#endif
#endif
