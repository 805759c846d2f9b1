// sspp_capi.cpp — C ABI: errors, model loading/inspection, host spline utilities.
#include <cmath>
#include <cstring>
#include <string>

#include "model.h"

namespace sspp {
namespace {
thread_local std::string g_err;
}
int set_error(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
void clear_error() { g_err.clear(); }
}  // namespace sspp

extern "C" {

const char* sspp_last_error(void) { return sspp::g_err.c_str(); }

int sspp_version(void) { return 10000; /* 0.1.0 */ }

int sspp_model_load_mjcf(const char* xml_path, sspp_model** out) {
    sspp::clear_error();
    if (!xml_path || !out) return sspp::set_error(SSPP_E_INVAL, "sspp_model_load_mjcf: null argument");
    auto* m = new sspp_model();
    int rc = sspp::load_mjcf(xml_path, *m);
    if (rc != SSPP_OK) {
        delete m;
        return rc;
    }
    *out = m;
    return SSPP_OK;
}

int sspp_model_view_get(const sspp_model* m, sspp_model_view* v) {
    if (!m || !v) return sspp::set_error(SSPP_E_INVAL, "null argument");
    v->nbody = m->nbody();
    v->body_parent = m->body_parent.data();
    v->body_jnt_type = m->body_jnt_type.data();
    v->body_qpos_adr = m->body_qpos_adr.data();
    v->body_pos = m->body_pos.data();
    v->body_quat = m->body_quat.data();
    v->ngeom = m->ngeom();
    v->geom_type = m->geom_type.data();
    v->geom_body = m->geom_body.data();
    v->geom_contype = m->geom_contype.data();
    v->geom_conaffinity = m->geom_conaffinity.data();
    v->geom_size = m->geom_size.data();
    v->geom_pos = m->geom_pos.data();
    v->geom_quat = m->geom_quat.data();
    v->geom_margin = m->geom_margin.data();
    v->nexclude = (int)m->exclude.size() / 2;
    v->exclude = m->exclude.data();
    v->nq = (int)m->qpos0.size();
    v->qpos0 = m->qpos0.data();
    return SSPP_OK;
}

int sspp_model_body_id(const sspp_model* m, const char* name) {
    if (!m || !name) return sspp::set_error(SSPP_E_INVAL, "null argument");
    for (int b = 0; b < m->nbody(); ++b)
        if (m->body_names[b] == name) return b;
    return sspp::set_error(SSPP_E_SCENE, std::string("Body with name '") + name + "' not found.");
}

int sspp_model_geom_id(const sspp_model* m, const char* name) {
    if (!m || !name) return sspp::set_error(SSPP_E_INVAL, "null argument");
    for (int g = 0; g < m->ngeom(); ++g)
        if (m->geom_names[g] == name) return g;
    return sspp::set_error(SSPP_E_SCENE, std::string("Geom with name '") + name + "' not found.");
}

// Utility::get_body_point (include/utility.h:228-259): (x, y, z, yaw) of a free body at
// qpos0; yaw = ZYX-Euler yaw of the joint quaternion (atan2 form; equal to Eigen's
// eulerAngles(2,1,0)[0] for the shipped scenes' pure-yaw orientations).
int sspp_model_body_point(const sspp_model* m, const char* name, double out[4]) {
    int b = sspp_model_body_id(m, name);
    if (b < 0) return b;
    if (m->body_jnt_type[b] != 0)
        return sspp::set_error(SSPP_E_SCENE, std::string("Body '") + name + "' is not a free joint.");
    const double* q = &m->qpos0[m->body_qpos_adr[b]];
    out[0] = q[0]; out[1] = q[1]; out[2] = q[2];
    const double w = q[3], x = q[4], y = q[5], z = q[6];
    out[3] = std::atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z));
    return SSPP_OK;
}

void sspp_model_free(sspp_model* m) { delete m; }

int sspp_interpolate(const double* pts, int n, int D, int degree, const double* u, double* knots,
                     double* ctrl) {
    sspp::clear_error();
    if (!pts || !u || !knots || !ctrl) return sspp::set_error(SSPP_E_INVAL, "null argument");
    if (sspp::interpolate(pts, n, D, degree, u, knots, ctrl) != 0)
        return sspp::set_error(SSPP_E_INVAL, "interpolation failed (need n >= degree + 1, distinct parameters)");
    return SSPP_OK;
}

int sspp_spline_eval(const double* knots, int n_knots, int degree, const double* ctrl, int D,
                     double u, double* out) {
    if (!knots || !ctrl || !out || degree < 1 || degree > 15 || n_knots < 2 * degree + 2)
        return sspp::set_error(SSPP_E_INVAL, "sspp_spline_eval: bad argument");
    int span = sspp::span_of(u, degree, knots, n_knots);
    double N[16];
    sspp::basis_funcs(u, degree, knots, n_knots, N);
    const double* c0 = ctrl + (size_t)(span - degree) * D;
    for (int d = 0; d < D; ++d) {
        double acc = N[0] * c0[d];
        for (int r = 1; r <= degree; ++r) acc = std::fma(N[r], c0[(size_t)r * D + d], acc);
        out[d] = acc;
    }
    return SSPP_OK;
}

int sspp_best_check(const sspp_best* recs, int n) {
    if (!recs || n < 0) return sspp::set_error(SSPP_E_INVAL, "null argument");
    int64_t lost = 0, first = -1;
    for (int i = 0; i < n; ++i)
        if (recs[i].reserved != 0) {
            lost += recs[i].reserved;
            if (first < 0) first = i;
        }
    if (lost)
        return sspp::set_error(SSPP_E_INCOMPLETE, "result record " + std::to_string(first) + " reports " +
                                                      std::to_string(lost) +
                                                      " lost candidates (split launch survivor queue): the "
                                                      "step's outputs are incomplete");
    return SSPP_OK;
}

int sspp_best_reduce(const sspp_best* parts, int n, sspp_best* out) {
    if (!parts || !out || n < 0) return sspp::set_error(SSPP_E_INVAL, "null argument");
    if (const int rc = sspp_best_check(parts, n)) return rc;
    sspp_best b;
    b.cost = INFINITY; b.index = -1; b.count = 0; b.reserved = 0;
    for (int i = 0; i < n; ++i) {
        b.count += parts[i].count;
        if (parts[i].index < 0) continue;
        if (b.index < 0 || parts[i].cost < b.cost ||
            (parts[i].cost == b.cost && parts[i].index < b.index)) {
            b.cost = parts[i].cost;
            b.index = parts[i].index;
        }
    }
    *out = b;
    return SSPP_OK;
}

}  // extern "C"
