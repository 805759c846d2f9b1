// sspp_pybind.cpp — the `_sspp` Python extension: drop-in for the reference's pybind11 module.
//
// Reference surface: src/sspp_bindings.cpp:14-69 (PYBIND11_MODULE(_sspp)):
//   SamplingPathPlanner{3,6,7,9}(xml_string)  .initializePath .evaluate(u) .evaluate(spline, u)
//   .sampleWithNoise .checkCollision .computeArcLength .findBestPath .get_ctrl_pts
//   .plan(start, end, sigma, limits, sample_count=50, check_points=50, init_points=10)
//       -> (bool, list[SplineN])
//   Spline{3,6,7,9}()  .ctrls() -> (N, n_ctrl) float64 view
//   create_model_capsule(uint64), create_data_capsule(uint64)
// Everything planner-side goes through the C ABI (include/sspp_hip.h) into the HIP kernels;
// this file holds no numerics beyond argument marshalling.
//
// Deliberate differences: candidates come from a counter-based Philox
// stream (seed attribute, default 0x5EED) instead of per-thread std::default_random_engine
// (SURVEY Q9); successful paths are returned in candidate order and ties in findBestPath go
// to the lowest index (Q10); the GIL is released while the GPU works; sampleWithNoise takes an
// integer candidate id as its `generator`; checkCollision ignores its `data` argument.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <iostream>
#include <memory>
#include <chrono>
#include <mutex>
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

template <int N>
struct Spline {
    std::vector<double> knots;  // n + 4
    std::vector<double> ctrl;   // stored [N][n] (row = dof) so ctrls() is a zero-copy view
    int n() const { return (int)(ctrl.size() / N); }
    std::vector<double> ctrl_nd() const {  // [n][N] for the C ABI
        int nn = n();
        std::vector<double> out((size_t)nn * N);
        for (int d = 0; d < N; ++d)
            for (int j = 0; j < nn; ++j) out[(size_t)j * N + d] = ctrl[(size_t)d * nn + j];
        return out;
    }
    void set_from_nd(const double* k, int nk, const double* c, int nn) {
        knots.assign(k, k + nk);
        ctrl.resize((size_t)N * nn);
        for (int d = 0; d < N; ++d)
            for (int j = 0; j < nn; ++j) ctrl[(size_t)d * nn + j] = c[(size_t)j * N + d];
    }
    // Eigen's Matrix<double, N, 1> reaches Python as a numpy array of shape (N,)
    py::array_t<double> eval(double u) const {
        if (ctrl.empty()) throw std::runtime_error("evaluate on an empty spline");
        py::array_t<double> out((ssize_t)N);
        std::vector<double> c = ctrl_nd();
        ck(sspp_spline_eval(knots.data(), (int)knots.size(), 3, c.data(), N, u, out.mutable_data()),
           "evaluate");
        return out;
    }
};

std::vector<double> vec_of(py::array_t<double, py::array::forcecast> a, int N, const char* name) {
    auto b = a.request();
    if (b.size != N)
        throw py::value_error(std::string(name) + ": expected " + std::to_string(N) +
                              " values (shape (N,) or (N,1)), got " + std::to_string(b.size));
    const double* p = static_cast<const double*>(b.ptr);
    // handle arbitrary strides via a contiguous copy
    py::array_t<double> c = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(a);
    p = c.data();
    return std::vector<double>(p, p + N);
}

template <int N>
class Planner {
public:
    explicit Planner(const std::string& xml) : xml_path_(xml) {
        sspp_model* m = nullptr;
        int rc = sspp_model_load_mjcf(xml.c_str(), &m);
        if (rc < 0)
            throw std::runtime_error(std::string("Failed to load MuJoCo model from XML: ") + sspp_last_error());
        model_.reset(m);
    }

    bool initializePath(py::array_t<double, py::array::forcecast> start,
                        py::array_t<double, py::array::forcecast> end, Spline<N>& s, int num_points) {
        auto a = vec_of(start, N, "start"), b = vec_of(end, N, "end");
        if (num_points < 4) throw py::value_error("num_points must be >= 4 for a cubic spline");
        std::vector<double> u(num_points), pts((size_t)num_points * N), knots(num_points + 4),
            ctrl((size_t)num_points * N);
        for (int i = 0; i < num_points; ++i) {
            double t = (double)i / (num_points - 1);
            u[i] = t;
            for (int d = 0; d < N; ++d) pts[(size_t)i * N + d] = (1 - t) * a[d] + t * b[d];
        }
        ck(sspp_interpolate(pts.data(), num_points, N, 3, u.data(), knots.data(), ctrl.data()),
           "initializePath");
        s.set_from_nd(knots.data(), (int)knots.size(), ctrl.data(), num_points);
        return true;
    }

    // The device state (scene tables, the job of the last plan() shape, candidate buffers,
    // pinned staging) lives in one sspp_planner per object; a call allocates nothing on the
    // device and copies back only the feasible candidates (sspp_hip.h, sspp_planner_plan).
    py::tuple plan(py::array_t<double, py::array::forcecast> start,
                   py::array_t<double, py::array::forcecast> end, double sigma,
                   py::array_t<double, py::array::forcecast> limits, int sample_count,
                   int check_points, int init_points) {
        auto a = vec_of(start, N, "start"), b = vec_of(end, N, "end"), l = vec_of(limits, N, "limits");
        if (sample_count < 1) throw py::value_error("sample_count must be >= 1");
        if (init_points < 4) throw py::value_error("init_points must be >= 4");
        if (check_points < 2) throw py::value_error("check_points must be >= 2");
        auto lk = lock();  // held until the shared buffers below have been read
        ensure_planner();
        const int n = init_points;
        const size_t nd = (size_t)n * N;
        knots_buf_.resize(n + 4);
        if (ids_buf_.size() < (size_t)sample_count) {
            ids_buf_.resize(sample_count);
            arc_buf_.resize(sample_count);
        }
        if (ctrl_buf_.size() < (size_t)sample_count * nd) ctrl_buf_.resize((size_t)sample_count * nd);
        sspp_best best{};
        int64_t nf = 0;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = sspp_planner_plan(planner_.get(), a.data(), b.data(), sigma, l.data(), sample_count,
                                   check_points, init_points, seed, 0, knots_buf_.data(), &nf,
                                   ids_buf_.data(), arc_buf_.data(), ctrl_buf_.data(), &best);
        }
        ck(rc, "plan");
        py::list paths;
        for (int64_t k = 0; k < nf; ++k) {
            Spline<N> s;
            s.set_from_nd(knots_buf_.data(), (int)knots_buf_.size(), ctrl_buf_.data() + (size_t)k * nd, n);
            paths.append(py::cast(std::move(s)));
        }
        std::cout << "Sampled " << sample_count << " splines. Successful paths found: "
                  << best.count << std::endl;
        bool found = best.index >= 0;
        if (found) {
            // the winner is one of the compacted rows (ids ascending)
            for (int64_t k = 0; k < nf; ++k) {
                if (ids_buf_[(size_t)k] != best.index) continue;
                path_.set_from_nd(knots_buf_.data(), (int)knots_buf_.size(), ctrl_buf_.data() + (size_t)k * nd, n);
                break;
            }
        }
        last_best_cost = best.cost;
        last_best_index = best.index;
        last_feasible_ids.assign(ids_buf_.begin(), ids_buf_.begin() + nf);
        return py::make_tuple(found, paths);
    }

    py::array_t<double> evaluate(double u) const { return path_.eval(u); }
    py::array_t<double> evaluate_s(const Spline<N>& s, double u) const { return s.eval(u); }

    Spline<N> sampleWithNoise(const Spline<N>& init, double sigma,
                              py::array_t<double, py::array::forcecast> limits, py::object generator) {
        auto l = vec_of(limits, N, "limits");
        int64_t id = 0;
        try { id = generator.cast<int64_t>(); }
        catch (const py::cast_error&) {
            throw py::type_error("sampleWithNoise: `generator` must be an integer candidate id "
                                 "(the GPU sampler is counter-based Philox, not std::default_random_engine)");
        }
        std::vector<double> c = init.ctrl_nd(), out(c.size());
        ck(sspp_sample_ctrl_host(init.knots.data(), 3, c.data(), init.n(), N, sigma, l.data(), seed,
                                 id, 1, out.data()), "sampleWithNoise");
        Spline<N> s;
        s.set_from_nd(init.knots.data(), (int)init.knots.size(), out.data(), init.n());
        return s;
    }

    // include/sspp.h:132-150 checks u = i / num_samples for i = 0..num_samples (num_samples >= 1)
    bool checkCollision(const Spline<N>& s, int num_samples, py::object /*data*/) {
        if (num_samples < 1) throw py::value_error("num_samples must be >= 1");
        if (s.ctrl.empty()) throw py::value_error("checkCollision on an empty spline");
        auto lk = lock();
        ensure_planner();
        double arc;
        uint8_t feas;
        sspp_best best;
        std::vector<double> c = s.ctrl_nd();
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = sspp_planner_score(planner_.get(), s.knots.data(), 3, c.data(), 1, s.n(), num_samples, 1,
                                    &arc, &feas, &best);
        }
        ck(rc, "checkCollision");
        return feas == 0;
    }

    double computeArcLength(const Spline<N>& s, int check_points) {
        if (check_points < 2) throw py::value_error("check_points must be >= 2");
        if (s.ctrl.empty()) throw py::value_error("computeArcLength on an empty spline");
        auto lk = lock();
        ensure_planner();
        double arc;
        uint8_t feas;
        sspp_best best;
        std::vector<double> c = s.ctrl_nd();
        ck(sspp_planner_score(planner_.get(), s.knots.data(), 3, c.data(), 1, s.n(), check_points, 0,
                              &arc, &feas, &best), "computeArcLength");
        return arc;
    }

    bool findBestPath(const std::vector<Spline<N>>& paths, Spline<N>& best_spline, int check_points) {
        if (paths.empty()) return false;
        if (check_points < 2) throw py::value_error("check_points must be >= 2");
        const Spline<N>& f = paths.front();
        bool same = true;
        for (auto& s : paths) same = same && s.knots == f.knots && s.n() == f.n();
        double best = INFINITY;
        int64_t bi = -1;
        if (same) {
            std::vector<double> all;
            all.reserve(paths.size() * f.ctrl.size());
            for (auto& s : paths) { auto c = s.ctrl_nd(); all.insert(all.end(), c.begin(), c.end()); }
            std::vector<double> arc(paths.size());
            std::vector<uint8_t> feas(paths.size());
            sspp_best b;
            auto lk = lock();
            ensure_planner();
            ck(sspp_planner_score(planner_.get(), f.knots.data(), 3, all.data(), (int64_t)paths.size(),
                                  f.n(), check_points, 0, arc.data(), feas.data(), &b),
               "findBestPath");
            best = b.cost; bi = b.index;
        } else {
            for (size_t i = 0; i < paths.size(); ++i) {
                double c = computeArcLength(paths[i], check_points);
                if (c < best) { best = c; bi = (int64_t)i; }
            }
        }
        if (bi < 0) return false;
        best_spline = paths[(size_t)bi];
        return true;
    }

    py::array_t<double> get_ctrl_pts(py::object self) {
        int nn = path_.n();
        return py::array_t<double>({N, nn}, {(ssize_t)(nn * sizeof(double)), (ssize_t)sizeof(double)},
                                   path_.ctrl.data(), self);
    }

    uint64_t seed = 0x5EED;
    double last_best_cost = INFINITY;
    int64_t last_best_index = -1;
    std::vector<int64_t> last_feasible_ids;  // candidate ids of the last plan()'s paths

private:
    struct ModelDel { void operator()(sspp_model* m) const { sspp_model_free(m); } };
    struct SceneDel { void operator()(sspp_scene* s) const { sspp_scene_free(s); } };
    struct PlannerDel { void operator()(sspp_planner* p) const { sspp_planner_free(p); } };

    // One call at a time per object: plan / checkCollision / computeArcLength / findBestPath
    // share the sspp_planner's device and pinned buffers and this object's host buffers.  The
    // mutex is taken with the GIL released (a thread holding it re-acquires the GIL after its
    // device call, so waiting for it while holding the GIL would deadlock).
    std::unique_lock<std::mutex> lock() {
        std::unique_lock<std::mutex> lk(mu_, std::defer_lock);
        py::gil_scoped_release nogil;
        lk.lock();
        return lk;
    }

    void ensure_planner() {
        if (planner_) return;
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        if (!scene_) {
            sspp_scene* s = nullptr;
            // count_static = 1: checkCollision's ncon is the whole scene's (include/sspp.h:143-144,
            // Q7), static-static contacts included
            ck(sspp_scene_create(model_.get(), SSPP_MODE_QPOS, N, 1, &s), "scene");
            scene_.reset(s);
        }
        const auto t1 = clk::now();
        sspp_planner* p = nullptr;
        ck(sspp_planner_create(scene_.get(), N, &p), "planner");
        planner_.reset(p);
        scene_us_ = std::chrono::duration<double, std::micro>(t1 - t0).count();
        planner_us_ = std::chrono::duration<double, std::micro>(clk::now() - t1).count();
    }

public:
    // diagnostics, not the reference's API: where a fresh object's first plan() spends its time —
    // the device scene tables, the planner (its HIP stream), and the job of the plan() shape
    // (tables, buffers, the asynchronous pre-pass's start), microseconds
    py::dict timings() {
        py::dict d;
        d["scene_create_us"] = scene_us_;
        d["planner_create_us"] = planner_us_;
        int64_t v = -1;
        if (planner_ && sspp_planner_get_option(planner_.get(), SSPP_OPT_CREATE_US, &v) == SSPP_OK)
            d["job_create_us"] = (double)v;
        return d;
    }

private:
    double scene_us_ = 0.0, planner_us_ = 0.0;

    std::string xml_path_;
    std::unique_ptr<sspp_model, ModelDel> model_;
    std::unique_ptr<sspp_scene, SceneDel> scene_;
    std::unique_ptr<sspp_planner, PlannerDel> planner_;  // declared after scene_: freed first
    std::vector<double> knots_buf_, arc_buf_, ctrl_buf_;
    std::vector<int64_t> ids_buf_;
    Spline<N> path_;
    std::mutex mu_;
};

template <int N>
void bind(py::module& m, const std::string& planner_name, const std::string& spline_name) {
    using S = Spline<N>;
    using P = Planner<N>;
    py::class_<S>(m, spline_name.c_str())
        .def(py::init<>())
        .def("ctrls", [](py::object self) {
                 S& s = self.cast<S&>();
                 int nn = s.n();
                 return py::array_t<double>({N, nn},
                                            {(ssize_t)(nn * sizeof(double)), (ssize_t)sizeof(double)},
                                            s.ctrl.data(), self);
             })
        .def("knots", [](const S& s) { return py::array_t<double>((ssize_t)s.knots.size(), s.knots.data()); })
        .def("__call__", [](const S& s, double u) { return s.eval(u); }, py::arg("u"));

    py::class_<P>(m, planner_name.c_str())
        .def(py::init<const std::string&>(), py::arg("xml_string"))
        .def("initializePath", &P::initializePath, py::arg("start"), py::arg("end"),
             py::arg("init_spline"), py::arg("num_points") = 10)
        .def("evaluate", &P::evaluate, py::arg("u"))
        .def("evaluate", &P::evaluate_s, py::arg("spline"), py::arg("u"))
        .def("sampleWithNoise", &P::sampleWithNoise, py::arg("init_spline"), py::arg("sigma"),
             py::arg("limits"), py::arg("generator"))
        .def("checkCollision", &P::checkCollision, py::arg("spline"), py::arg("num_samples"),
             py::arg("data") = py::none())
        .def("computeArcLength", &P::computeArcLength, py::arg("spline"), py::arg("check_points"))
        .def("findBestPath", &P::findBestPath, py::arg("successful_paths"), py::arg("best_spline"),
             py::arg("check_points") = 10)
        .def("get_ctrl_pts", [](py::object self) { return self.cast<P&>().get_ctrl_pts(self); })
        .def("plan", &P::plan, py::arg("start"), py::arg("end"), py::arg("sigma"), py::arg("limits"),
             py::arg("sample_count") = 50, py::arg("check_points") = 50, py::arg("init_points") = 10)
        .def_readwrite("seed", &P::seed)
        .def_readonly("last_best_cost", &P::last_best_cost)
        .def_readonly("last_best_index", &P::last_best_index)
        .def_readonly("last_feasible_ids", &P::last_feasible_ids)
        .def("_timings", &P::timings);
}

}  // namespace

PYBIND11_MODULE(_sspp, m) {
    m.doc() = "MI355X-native SamplingPathPlanner (drop-in for the reference's _sspp module)";
    bind<3>(m, "SamplingPathPlanner3", "Spline3");
    bind<6>(m, "SamplingPathPlanner6", "Spline6");
    bind<7>(m, "SamplingPathPlanner7", "Spline7");
    bind<9>(m, "SamplingPathPlanner9", "Spline9");
    m.def("create_model_capsule", [](uint64_t p) { return py::capsule(reinterpret_cast<void*>(p), "mjModel"); });
    m.def("create_data_capsule", [](uint64_t p) { return py::capsule(reinterpret_cast<void*>(p), "mjData"); });
    m.attr("__backend__") = "hip-gfx950";
}
