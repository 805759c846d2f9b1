// Sanitizer driver (SURVEY §5 "CPU restatement built with -fsanitize=address,undefined"):
// runs the host C++ of the product (MJCF loader + xml_lite, spline fitting, C-ABI model
// helpers) and the oracle's C restatement (scene build, FK, every narrowphase including the
// exact cylinder-box test and the box-box manifold, both scorers, the CES update) under
// AddressSanitizer + UndefinedBehaviorSanitizer, host code only.  Exit 0 = clean.
// Test infrastructure: built and run by tests/test_sanitize.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "sspp_hip.h"
extern "C" {
#include "sspp_oracle.h"
}

static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::fprintf(stderr, "CHECK failed %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

static or_model as_oracle(const sspp_model_view& v) {
    or_model m;
    m.nbody = v.nbody; m.body_parent = v.body_parent; m.body_jnt_type = v.body_jnt_type;
    m.body_qpos_adr = v.body_qpos_adr; m.body_pos = v.body_pos; m.body_quat = v.body_quat;
    m.ngeom = v.ngeom; m.geom_type = v.geom_type; m.geom_body = v.geom_body;
    m.geom_contype = v.geom_contype; m.geom_conaffinity = v.geom_conaffinity;
    m.geom_size = v.geom_size; m.geom_pos = v.geom_pos; m.geom_quat = v.geom_quat;
    m.geom_margin = v.geom_margin; m.nexclude = v.nexclude; m.exclude = v.exclude;
    m.nq = v.nq; m.qpos0 = v.qpos0;
    return m;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "sspp_amd/scenes";
    std::mt19937_64 rng(1234);
    std::normal_distribution<double> N01(0.0, 1.0);
    // ---- MJCF loader: the shipped scenes and malformed inputs
    for (const char* bad : {"/nonexistent.xml", "tests/sanitize/san_main.cpp"}) {
        sspp_model* m = nullptr;
        CHECK(sspp_model_load_mjcf(bad, &m) < 0 && m == nullptr);
        CHECK(std::strlen(sspp_last_error()) > 0);
    }
    for (const char* scene : {"robocrane.xml", "stacking.xml", "planner.xml"}) {
        sspp_model* m = nullptr;
        const std::string path = dir + "/" + scene;
        CHECK(sspp_model_load_mjcf(path.c_str(), &m) == 0);
        if (!m) continue;
        sspp_model_view v;
        CHECK(sspp_model_view_get(m, &v) == 0);
        double pt[4];
        CHECK(sspp_model_body_point(m, "no_such_body", pt) < 0);
        or_model om = as_oracle(v);
        // SamplingPathPlanner window over the first free joint + TaskSpacePlanner body mode
        const int dof = 7;
        or_scene* s = or_scene_create(&om, 0, dof);
        CHECK(s != nullptr);
        int body = -1;
        for (int b = 1; b < v.nbody && body < 0; ++b)
            if (v.body_jnt_type[b] == 0) body = b;
        or_scene* st = body > 0 ? or_scene_create(&om, 1, body) : nullptr;
        // ---- spline fitting + sampling + scoring
        const int n = 10, p = 3, W = 64, B = 96;
        std::vector<double> u(n), pts(n * dof), knots(n + p + 1), ctrl0(n * dof);
        double q0[7];
        for (int k = 0; k < 7; ++k) q0[k] = v.qpos0[k];
        for (int i = 0; i < n; ++i) {
            u[i] = (double)i / (n - 1);
            for (int d = 0; d < dof; ++d) pts[i * dof + d] = q0[d] + (d == 1 ? 0.2 * u[i] : 0.0);
        }
        CHECK(sspp_interpolate(pts.data(), n, dof, p, u.data(), knots.data(), ctrl0.data()) == 0);
        std::vector<double> ok(n + p + 1), oc(n * dof);
        CHECK(or_interpolate(pts.data(), n, dof, p, u.data(), ok.data(), oc.data()) == 0);
        double e[7];
        CHECK(sspp_spline_eval(knots.data(), n + p + 1, p, ctrl0.data(), dof, 0.37, e) == 0);
        std::vector<double> limits(dof, 1.0), ctrl((size_t)B * n * dof), arc(B);
        std::vector<uint8_t> feas(B);
        or_sample_sspp(ctrl0.data(), n, dof, p, 0.08, limits.data(), 0x5EED, 0, B, ctrl.data(), 0);
        or_sample_sspp(ctrl0.data(), n, dof, p, 0.08, limits.data(), 0x5EED, 0, B, ctrl.data(), 1);
        if (s) {
            CHECK(or_sspp_score(s, knots.data(), n + p + 1, p, ctrl.data(), n, dof, B, W, 0, 0, 2, 0,
                                arc.data(), feas.data()) == 0);
            double best;
            (void)or_argmin(arc.data(), feas.data(), B, &best);
        }
        if (st) {
            // random (x, y, z, yaw) points around the scene: every narrowphase pair type
            for (int t = 0; t < 4000; ++t) {
                double q[4] = {0.5 + 0.3 * N01(rng), 0.05 + 0.3 * N01(rng), 0.15 + 0.1 * N01(rng), N01(rng)};
                double c; int nd;
                (void)or_point_contacts(st, q, 1, &c, &nd);
            }
            const int K = 1, cp = 48, NB = 64;
            double mean[4] = {q0[0], q0[1], q0[2] + 0.1, 0.0}, sig[4] = {0.2, 0.2, 0.1, 0.5};
            double lo[4] = {-1, -1, 0, -3.2}, hi[4] = {1, 1, 1, 3.2}, a[4], b[4];
            for (int k = 0; k < 3; ++k) { a[k] = q0[k]; b[k] = q0[k] + 0.1; }
            a[3] = 0.0; b[3] = 0.3;
            std::vector<double> vias(NB * K * 4), L(NB), Cnf(NB), Cwf(NB), cost(NB);
            std::vector<uint8_t> status(NB);
            or_sample_tsp(mean, sig, K, lo, hi, 0.0, 0x5EED, 0, NB, vias.data());
            CHECK(or_tsp_score(st, a, b, vias.data(), K, NB, cp, 1.0, 0, 2, L.data(), Cnf.data(),
                               Cwf.data(), status.data(), cost.data()) == 0);
        }
        if (s) or_scene_destroy(s);
        if (st) or_scene_destroy(st);
        sspp_model_free(m);
    }
    if (fails) std::fprintf(stderr, "%d checks failed\n", fails);
    std::printf("sanitize driver done\n");
    return fails ? 1 : 0;
}
