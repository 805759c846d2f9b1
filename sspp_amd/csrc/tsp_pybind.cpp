// tsp_pybind.cpp — the `_tsp` Python extension: tsp::TaskSpacePlanner on the MI355X.
//
// The reference's own `_tsp` binding (src/tsp_bindings.cpp) no longer compiles against its
// headers, so this module mirrors the C++ adapter it should expose,
// include/sspp/tsp.h:7-106 (constructor arguments, plan(start, end, iterate), getters), and the
// types of include/sspp/tsp_types.h (Point, Spline = Eigen::Spline<double, 4, 2>, ViaSet,
// SolverStatus, PathCandidate).  The CES iteration itself (seeds, evaluation, elites,
// distribution update, best forwarding) runs on the device through the C ABI (sspp_ces_*);
// this file only marshals arguments and builds the returned objects.
//
// Deliberate differences: the constructor takes an MJCF path instead of an
// mjModel*; candidates come from Philox streams (attribute `seed`); successes are returned in
// slot order (mean set, forwarded best, samples); `plan_iterations` runs several plan()
// iterations back to back without returning to Python.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <array>
#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "sspp_hip.h"

namespace py = pybind11;

namespace {

void ck(int rc, const char* what) {
    if (rc < 0) {
        std::string msg = std::string(what) + ": " + sspp_last_error();
        if (rc == SSPP_E_INVAL) throw py::value_error(msg);
        throw std::runtime_error(msg);
    }
}

using Point = std::array<double, 4>;
using ViaSet = std::vector<Point>;

enum class SolverStatus { Converged, Failed, BelowFloor, MaxIter, Unknown };

const char* status_str(SolverStatus s) {
    switch (s) {
        case SolverStatus::Converged: return "Converged";
        case SolverStatus::Failed: return "Failed";
        case SolverStatus::BelowFloor: return "BelowFloor";
        case SolverStatus::MaxIter: return "MaxIter";
        default: return "Unknown";
    }
}

Point point_of(py::array_t<double, py::array::forcecast> a, const char* name) {
    py::array_t<double> c = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(a);
    if (!c || c.size() != 4)
        throw py::value_error(std::string(name) + ": expected 4 values (x, y, z, yaw)");
    return {c.data()[0], c.data()[1], c.data()[2], c.data()[3]};
}

py::array_t<double> arr(const Point& p) {
    py::array_t<double> a(4);
    for (int i = 0; i < 4; ++i) a.mutable_data()[i] = p[i];
    return a;
}

// tsp::Spline: degree-2, 4-DoF; ctrls() is (4, n) like Eigen's ControlPointVectorType
struct Spline {
    std::vector<double> knots;  // n + 3
    std::vector<double> ctrl;   // [4][n] (row = dof)
    int n() const { return (int)(ctrl.size() / 4); }
    Point eval(double u) const {
        if (ctrl.empty()) throw std::runtime_error("evaluate on an empty spline");
        const int nn = n();
        std::vector<double> c((size_t)nn * 4);
        for (int d = 0; d < 4; ++d)
            for (int j = 0; j < nn; ++j) c[(size_t)j * 4 + d] = ctrl[(size_t)d * nn + j];
        Point out;
        ck(sspp_spline_eval(knots.data(), (int)knots.size(), 2, c.data(), 4, u, out.data()), "evaluate");
        return out;
    }
};

// PathModel::fromVias / initLinear (tsp_path_model.h:21-43): interpolate [start, vias, end]
// at u_i = i / (total_points - 1) with degree 2
Spline spline_through(const std::vector<Point>& pts) {
    const int n = (int)pts.size();
    if (n < 3) throw py::value_error("a degree-2 path needs at least 3 points (start, via, end)");
    std::vector<double> u(n), P((size_t)n * 4), knots(n + 3), ctrl((size_t)n * 4);
    for (int i = 0; i < n; ++i) {
        u[i] = (double)i / (n - 1);
        for (int d = 0; d < 4; ++d) P[(size_t)i * 4 + d] = pts[i][d];
    }
    ck(sspp_interpolate(P.data(), n, 4, 2, u.data(), knots.data(), ctrl.data()), "fromVias");
    Spline s;
    s.knots = knots;
    s.ctrl.resize((size_t)4 * n);
    for (int d = 0; d < 4; ++d)
        for (int j = 0; j < n; ++j) s.ctrl[(size_t)d * n + j] = ctrl[(size_t)j * 4 + d];
    return s;
}

struct GradientStep {  // tsp_types.h:18-23 (unused by the CES-only planner)
    Point x{0, 0, 0, 0};
    double f = 0.0;
};

struct PathCandidate {  // tsp_types.h:25-34
    ViaSet via;
    py::object refined = py::none();
    std::vector<GradientStep> steps;
    SolverStatus status = SolverStatus::Failed;
    double L = -1.0, C_nf = -1.0, C_wf = -1.0;
};

class TaskSpacePlanner {
public:
    TaskSpacePlanner(const std::string& xml, const std::string& body_name, double stddev_initial,
                     double stddev_min, double stddev_max, double inc, double dec,
                     double elite_fraction, int sample_count, int check_points, int /*gd_iterations*/,
                     int init_points, double collision_weight, double z_min,
                     py::array_t<double, py::array::forcecast> limits_min,
                     py::array_t<double, py::array::forcecast> limits_max, bool /*enable_gd*/,
                     double sigma_floor, double var_ema_beta, double mean_lr, double /*max_step_norm*/,
                     double /*floor_margin*/, double /*floor_penalty_scale*/, uint64_t seed)
        : lo_(point_of(limits_min, "limits_min")), hi_(point_of(limits_max, "limits_max")),
          total_points_(init_points), samples_(sample_count) {
        sspp_model* m = nullptr;
        if (sspp_model_load_mjcf(xml.c_str(), &m) < 0)
            throw std::runtime_error(std::string("Failed to load MuJoCo model from XML: ") + sspp_last_error());
        model_.reset(m);
        const int body = sspp_model_body_id(m, body_name.c_str());
        if (body < 0) throw std::runtime_error("Body not found: " + body_name);
        sspp_scene* s = nullptr;
        ck(sspp_scene_create(m, SSPP_MODE_BODY, body, 0, &s), "scene (free body)");
        scene_.reset(s);
        sspp_ces_config c{};
        c.samples = sample_count; c.checks = check_points; c.total_points = init_points;
        c.w_collision = collision_weight; c.elite_fraction = elite_fraction; c.inc = inc; c.dec = dec;
        c.sigma_floor = sigma_floor; c.var_beta = var_ema_beta; c.mean_lr = mean_lr;
        c.stddev_min = stddev_min; c.stddev_max = stddev_max;
        c.z_min = z_min;
        c.dist_z_min = stddev_initial;  // tsp.h:53 -> Planner(..., z_min = stddev_initial)
        c.sigma0 = 0.3;                 // Planner::sigma0_ (tsp_planner.h:177)
        c.lo = lo_.data(); c.hi = hi_.data();
        // Planner never copies cfg.z_min / floor_* into its Evaluator
        c.floor_z_min = 0.0; c.floor_margin = 0.01; c.floor_scale = 10.0;
        c.seed = seed;
        sspp_ces* p = nullptr;
        ck(sspp_ces_create(scene_.get(), &c, 1, &p), "TaskSpacePlanner");
        ces_.reset(p);
        K_ = init_points - 2;
        via_ = linear(Point{0, 0, 0, 0}, Point{0, 0, 0, 0});
    }

    // plan(start, end, iterate) (tsp.h:58-60 -> tsp_planner.h:72-145)
    std::vector<PathCandidate> plan(py::array_t<double, py::array::forcecast> start,
                                    py::array_t<double, py::array::forcecast> end, bool iterate) {
        return plan_iterations(start, end, iterate, 1);
    }

    std::vector<PathCandidate> plan_iterations(py::array_t<double, py::array::forcecast> start,
                                               py::array_t<double, py::array::forcecast> end,
                                               bool iterate, int iterations) {
        const Point a = point_of(start, "start"), b = point_of(end, "end");
        if (iterations < 1) throw py::value_error("iterations must be >= 1");
        via_ = linear(a, b);
        const int n = samples_ + 2, KD = 4 * K_;
        std::vector<double> L(n), Cnf(n), Cwf(n), cost(n), vias((size_t)n * KD), mean(KD), sigma(KD), lb(KD);
        std::vector<uint8_t> st(n);
        sspp_ces_state s{};
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = sspp_ces_plan(ces_.get(), a.data(), b.data(), iterate ? 1 : 0, iterations, nullptr);
            if (rc >= 0)
                rc = sspp_ces_read(ces_.get(), &s, L.data(), Cnf.data(), Cwf.data(), cost.data(), st.data(),
                                   vias.data(), mean.data(), sigma.data(), lb.data(), nullptr);
        }
        ck(rc, "plan");
        successes_.clear(); failures_.clear(); sampled_.clear();
        for (int i = 0; i < s.n_candidates; ++i) {
            PathCandidate c;
            for (int v = 0; v < K_; ++v) {
                const double* q = &vias[(size_t)i * KD + 4 * v];
                c.via.push_back({q[0], q[1], q[2], q[3]});
            }
            c.L = L[i]; c.C_nf = Cnf[i]; c.C_wf = Cwf[i];
            c.status = st[i] ? SolverStatus::Converged : SolverStatus::Failed;
            sampled_.push_back(c.via);
            (st[i] ? successes_ : failures_).push_back(std::move(c));
        }
        mean_ = mean; sigma_ = sigma;
        // path_ = initLinear, replaced by fromVias(last_best_) when this call found a success
        std::vector<Point> pts = via_;
        if (s.n_success > 0)
            for (int v = 0; v < K_; ++v) pts[1 + v] = {lb[4 * v], lb[4 * v + 1], lb[4 * v + 2], lb[4 * v + 3]};
        path_ = spline_through(pts);
        last_state_ = s;
        return successes_;
    }

    std::vector<PathCandidate> successes() const { return successes_; }
    std::vector<PathCandidate> failures() const { return failures_; }
    std::vector<ViaSet> sampled_sets() const { return sampled_; }
    std::vector<Point> sampled_via_pts() const {
        std::vector<Point> out;
        for (auto& S : sampled_) out.push_back(S.empty() ? Point{0, 0, 0, 0} : S.front());
        return out;
    }
    std::vector<Point> via_pts() const { return via_; }
    Point mean() const { return first(mean_); }
    Point stddev() const { return first(sigma_); }
    Point limits_min() const { return lo_; }
    Point limits_max() const { return hi_; }
    Point evaluate(double u) const { return path_.eval(u); }
    std::vector<Point> path_pts(int N) const {
        std::vector<Point> pts;
        for (int i = 0; i < N; ++i) pts.push_back(path_.eval(N > 1 ? (double)i / (N - 1) : 0.0));
        return pts;
    }
    const Spline& spline() const { return path_; }
    // PathModel::fromVias (tsp_path_model.h:32-43): the given vias replace interior slots 1..
    Spline spline_from_vias(const ViaSet& vias) const {
        if ((int)vias.size() > K_) throw py::value_error("at most " + std::to_string(K_) + " via points");
        std::vector<Point> pts = via_;
        for (size_t v = 0; v < vias.size(); ++v) pts[1 + v] = vias[v];
        return spline_through(pts);
    }
    int n_vias() const { return K_; }
    sspp_ces_state last_state_{};

private:
    std::vector<Point> linear(const Point& a, const Point& b) const {  // PathModel::setupLinear
        std::vector<Point> v(total_points_);
        for (int i = 0; i < total_points_; ++i) {
            const double t = (double)i / (total_points_ - 1);
            for (int d = 0; d < 4; ++d) v[i][d] = (1.0 - t) * a[d] + t * b[d];
        }
        return v;
    }
    static Point first(const std::vector<double>& x) {
        return x.size() >= 4 ? Point{x[0], x[1], x[2], x[3]} : Point{0, 0, 0, 0};
    }

    struct ModelDel { void operator()(sspp_model* m) const { sspp_model_free(m); } };
    struct SceneDel { void operator()(sspp_scene* s) const { sspp_scene_free(s); } };
    struct CesDel { void operator()(sspp_ces* c) const { sspp_ces_free(c); } };
    std::unique_ptr<sspp_model, ModelDel> model_;
    std::unique_ptr<sspp_scene, SceneDel> scene_;
    std::unique_ptr<sspp_ces, CesDel> ces_;
    Point lo_, hi_;
    int total_points_, samples_, K_ = 1;
    std::vector<Point> via_;
    std::vector<double> mean_, sigma_;
    std::vector<PathCandidate> successes_, failures_;
    std::vector<ViaSet> sampled_;
    Spline path_;
};

py::list points(const std::vector<Point>& v) {
    py::list l;
    for (auto& p : v) l.append(arr(p));
    return l;
}

}  // namespace

PYBIND11_MODULE(_tsp, m) {
    m.doc() = "MI355X-native TaskSpacePlanner (CES over sampled via points; include/sspp/tsp.h)";

    py::enum_<SolverStatus>(m, "SolverStatus")
        .value("Converged", SolverStatus::Converged)
        .value("Failed", SolverStatus::Failed)
        .value("BelowFloor", SolverStatus::BelowFloor)
        .value("MaxIter", SolverStatus::MaxIter)
        .value("Unknown", SolverStatus::Unknown)
        .export_values();
    m.def("solver_status_to_string", &status_str);

    py::class_<Spline>(m, "Spline")
        .def(py::init<>())
        .def("ctrls", [](py::object self) {
                 Spline& s = self.cast<Spline&>();
                 const int nn = s.n();
                 return py::array_t<double>({4, nn}, {(ssize_t)(nn * sizeof(double)), (ssize_t)sizeof(double)},
                                            s.ctrl.data(), self);
             })
        .def("knots", [](py::object self) {
                 Spline& s = self.cast<Spline&>();
                 return py::array_t<double>({(ssize_t)s.knots.size()}, {(ssize_t)sizeof(double)},
                                            s.knots.data(), self);
             })
        .def("__call__", [](const Spline& s, double u) { return arr(s.eval(u)); }, py::arg("u"));

    py::class_<GradientStep>(m, "GradientStep")
        .def(py::init<>())
        .def_property("x", [](const GradientStep& g) { return arr(g.x); },
                      [](GradientStep& g, py::array_t<double, py::array::forcecast> a) { g.x = point_of(a, "x"); })
        .def_readwrite("f", &GradientStep::f);

    py::class_<PathCandidate>(m, "PathCandidate")
        .def(py::init<>())
        .def_property("via", [](const PathCandidate& c) { return points(c.via); },
                      [](PathCandidate& c, py::list l) {
                          c.via.clear();
                          for (auto h : l) c.via.push_back(point_of(h.cast<py::array_t<double, py::array::forcecast>>(), "via"));
                      })
        .def_readwrite("refined", &PathCandidate::refined)
        .def_readwrite("steps", &PathCandidate::steps)
        .def_readwrite("status", &PathCandidate::status)
        .def_readwrite("L", &PathCandidate::L)
        .def_readwrite("C_nf", &PathCandidate::C_nf)
        .def_readwrite("C_wf", &PathCandidate::C_wf)
        .def("__repr__", [](const PathCandidate& c) {
            return std::string("PathCandidate(status=") + status_str(c.status) + ", L=" + std::to_string(c.L) +
                   ", C_nf=" + std::to_string(c.C_nf) + ", C_wf=" + std::to_string(c.C_wf) + ")";
        });

    using P = TaskSpacePlanner;
    py::class_<P>(m, "TaskSpacePlanner")
        .def(py::init<const std::string&, const std::string&, double, double, double, double, double, double,
                      int, int, int, int, double, double, py::array_t<double, py::array::forcecast>,
                      py::array_t<double, py::array::forcecast>, bool, double, double, double, double,
                      double, double, uint64_t>(),
             py::arg("xml_string"), py::arg("body_name"), py::arg("stddev_initial") = 0.3,
             py::arg("stddev_min") = 0.01, py::arg("stddev_max") = 0.5,
             py::arg("stddev_increase_factor") = 1.5, py::arg("stddev_decay_factor") = 0.95,
             py::arg("elite_fraction") = 0.3, py::arg("sample_count") = 50, py::arg("check_points") = 50,
             py::arg("gd_iterations") = 0, py::arg("init_points") = 3, py::arg("collision_weight") = 1.0,
             py::arg("z_min") = 0.0,
             py::arg("limits_min") = py::array_t<double>(4, std::array<double, 4>{-2, -2, -2, -2}.data()),
             py::arg("limits_max") = py::array_t<double>(4, std::array<double, 4>{2, 2, 2, 2}.data()),
             py::arg("enable_gradient_descent") = false, py::arg("sigma_floor") = 0.0,
             py::arg("var_ema_beta") = 0.2, py::arg("mean_lr") = 0.5, py::arg("max_step_norm") = 0.1,
             py::arg("floor_margin") = 0.01, py::arg("floor_penalty_scale") = 10.0,
             py::arg("seed") = 0x5EEDull)
        .def("plan", &P::plan, py::arg("start"), py::arg("end"), py::arg("iterate_flag") = false)
        .def("plan_iterations", &P::plan_iterations, py::arg("start"), py::arg("end"),
             py::arg("iterate_flag") = false, py::arg("iterations") = 1)
        .def("get_succesful_path_candidates", &P::successes)
        .def("get_failed_path_candidates", &P::failures)
        .def("get_sampled_via_sets", [](const P& p) {
            py::list out;
            for (auto& S : p.sampled_sets()) out.append(points(S));
            return out;
        })
        .def("get_sampled_via_pts", [](const P& p) { return points(p.sampled_via_pts()); })
        .def("get_via_pts", [](const P& p) { return points(p.via_pts()); })
        .def("get_current_mean", [](const P& p) { return arr(p.mean()); })
        .def("get_current_stddev", [](const P& p) { return arr(p.stddev()); })
        .def("get_limits_min", [](const P& p) { return arr(p.limits_min()); })
        .def("get_limits_max", [](const P& p) { return arr(p.limits_max()); })
        .def("evaluate", [](const P& p, double u, py::object s) {
                 if (s.is_none()) return arr(p.evaluate(u));
                 return arr(s.cast<const Spline&>().eval(u));
             }, py::arg("u"), py::arg("spline") = py::none())
        .def("get_path_pts", [](const P& p, int n) { return points(p.path_pts(n)); }, py::arg("n") = 10)
        .def("get_ctrl_pts", [](const P& p) {
                 const Spline& s = p.spline();
                 py::array_t<double> a({4, s.n()});
                 std::copy(s.ctrl.begin(), s.ctrl.end(), a.mutable_data());
                 return a;
             })
        .def("get_knot_vector", [](const P& p) {
                 const Spline& s = p.spline();
                 return py::array_t<double>((ssize_t)s.knots.size(), s.knots.data());
             })
        .def("set_verbose", [](P&, bool) {}, py::arg("on"))
        .def("spline_from_via", [](const P& p, py::array_t<double, py::array::forcecast> v) {
                 return p.spline_from_vias(ViaSet{point_of(v, "via")});
             }, py::arg("via"))
        .def("spline_from_vias", [](const P& p, py::list l) {
                 ViaSet vs;
                 for (auto h : l) vs.push_back(point_of(h.cast<py::array_t<double, py::array::forcecast>>(), "via"));
                 return p.spline_from_vias(vs);
             }, py::arg("vias"))
        .def("reset", [](P&) {})
        .def_property_readonly("last_n_success", [](const P& p) { return p.last_state_.n_success; })
        .def_property_readonly("last_best_slot", [](const P& p) { return p.last_state_.best_slot; })
        .def_property_readonly("last_best_cost", [](const P& p) { return p.last_state_.best_cost; });
    m.attr("__backend__") = "hip-gfx950";
}
