// mjcf.cpp — MJCF scene loader (the subset the planner's scenes use).
//
// Replaces mj_loadXML for the candidate-scoring path (reference: include/sspp.h:44-63 loads
// the scene with mj_loadXML and treats the constructor string as a file path).
// Semantics follow MuJoCo's compiler for what the shipped scenes contain:
//   * bodies depth-first pre-order, world body 0, geoms ordered body by body;
//   * <freejoint/> or <joint type="free"/> -> 7 qpos each, qpos0 = (pos, normalised quat);
//     any other joint type is rejected (SSPP_E_UNSUPPORTED) — hinge chains are out of scope;
//   * nested <default class=...> with inheritance; element class = `class` attribute, else the
//     innermost enclosing body's `childclass`, else "main"; explicit attributes win;
//   * orientation from quat / euler (<compiler angle eulerseq>) / axisangle, normalised;
//   * <contact><exclude body1 body2/>.
#include <cmath>
#include <fstream>
#include <map>
#include <sstream>

#include "model.h"
#include "xml_lite.h"

namespace sspp {
namespace {

const std::map<std::string, int> kGeomTypes = {
    {"plane", 0}, {"hfield", 1}, {"sphere", 2}, {"capsule", 3}, {"ellipsoid", 4},
    {"cylinder", 5}, {"box", 6}, {"mesh", 7}, {"sdf", 8}};

using AttrMap = std::map<std::string, std::string>;

struct Defaults {
    std::map<std::string, std::map<std::string, AttrMap>> cls;  // class -> tag -> attrs
    std::map<std::string, std::string> parent;                   // "" = none

    AttrMap resolve(const std::string& c, const std::string& tag) const {
        std::vector<std::string> chain;
        std::string cur = c;
        while (!cur.empty()) {
            chain.push_back(cur);
            auto it = parent.find(cur);
            if (it == parent.end()) break;
            cur = it->second;
        }
        AttrMap out;
        for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
            auto ci = cls.find(*it);
            if (ci == cls.end()) continue;
            auto ti = ci->second.find(tag);
            if (ti == ci->second.end()) continue;
            for (auto& kv : ti->second) out[kv.first] = kv.second;
        }
        return out;
    }
};

std::vector<double> floats(const std::string& s) {
    std::vector<double> v;
    std::istringstream is(s);
    double x;
    while (is >> x) v.push_back(x);
    return v;
}

void normq(double* q) {
    double s = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
    double n = std::sqrt(s);
    if (n > 0) { for (int k = 0; k < 4; ++k) q[k] = q[k] / n; }
    else { q[0] = 1; q[1] = q[2] = q[3] = 0; }
}

void qmul(const double* a, const double* b, double* r) {
    double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}

struct Compiler { bool degree = true; std::string seq = "xyz"; };

void orientation(const AttrMap& a, const Compiler& c, double* q) {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
    auto it = a.find("quat");
    if (it != a.end()) {
        auto v = floats(it->second);
        if (v.size() != 4) throw std::runtime_error("quat needs 4 numbers");
        for (int k = 0; k < 4; ++k) q[k] = v[k];
        normq(q);
        return;
    }
    it = a.find("euler");
    if (it != a.end()) {
        auto e = floats(it->second);
        if (e.size() != 3 || c.seq.size() != 3) throw std::runtime_error("bad euler");
        for (int k = 0; k < 3; ++k) {
            double ang = c.degree ? e[k] * M_PI / 180.0 : e[k];
            char ax = c.seq[k];
            double r[4] = {std::cos(ang / 2), 0, 0, 0};
            int idx = (ax == 'x' || ax == 'X') ? 1 : (ax == 'y' || ax == 'Y') ? 2 : 3;
            r[idx] = std::sin(ang / 2);
            double t[4];
            if (ax >= 'a') qmul(q, r, t); else qmul(r, q, t);
            for (int j = 0; j < 4; ++j) q[j] = t[j];
        }
        normq(q);
        return;
    }
    it = a.find("axisangle");
    if (it != a.end()) {
        auto v = floats(it->second);
        if (v.size() != 4) throw std::runtime_error("axisangle needs 4 numbers");
        double ang = c.degree ? v[3] * M_PI / 180.0 : v[3];
        double n = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double s = std::sin(ang / 2) / n;
        q[0] = std::cos(ang / 2); q[1] = v[0] * s; q[2] = v[1] * s; q[3] = v[2] * s;
        normq(q);
        return;
    }
    for (const char* k : {"xyaxes", "zaxis", "fromto"})
        if (a.count(k)) throw std::runtime_error(std::string("unsupported orientation attribute ") + k);
}

void read_defaults(const XNode& node, Defaults& d, const std::string& parent, bool top) {
    std::string name = "main";
    if (!top) {
        auto c = node.get("class");
        if (!c) throw std::runtime_error("nested <default> without class");
        name = *c;
    }
    if (!top || !d.parent.count(name)) d.parent[name] = parent;
    d.cls[name];
    for (auto& k : node.kids) {
        if (k->tag == "default") read_defaults(*k, d, name, false);
        else for (auto& a : k->attrs) d.cls[name][k->tag][a.first] = a.second;
    }
}

struct Loader {
    sspp_model& m;
    Defaults dfl;
    Compiler comp;
    std::vector<std::vector<size_t>> body_geoms_tmp;
    struct GeomTmp { std::string name; int type; double size[3], pos[3], quat[4]; int ct, ca; double margin; int body; };
    std::vector<GeomTmp> geoms;
    int nq = 0;

    explicit Loader(sspp_model& mm) : m(mm) {}

    AttrMap attrs_of(const XNode& n, const std::string& childclass) {
        auto c = n.get("class");
        AttrMap a = dfl.resolve(c ? *c : childclass, n.tag);
        for (auto& kv : n.attrs) a[kv.first] = kv.second;
        return a;
    }

    void add_geom(const XNode& n, int body, const std::string& cc) {
        AttrMap a = attrs_of(n, cc);
        GeomTmp g{};
        g.name = a.count("name") ? a["name"] : "";
        std::string t = a.count("type") ? a["type"] : "sphere";
        auto ti = kGeomTypes.find(t);
        if (ti == kGeomTypes.end()) throw std::runtime_error("unknown geom type " + t);
        g.type = ti->second;
        auto sz = floats(a.count("size") ? a["size"] : "0 0 0");
        for (int k = 0; k < 3; ++k) g.size[k] = k < (int)sz.size() ? sz[k] : 0.0;
        auto ps = floats(a.count("pos") ? a["pos"] : "0 0 0");
        if (ps.size() != 3) throw std::runtime_error("geom pos needs 3 numbers");
        for (int k = 0; k < 3; ++k) g.pos[k] = ps[k];
        orientation(a, comp, g.quat);
        g.ct = a.count("contype") ? std::stoi(a["contype"]) : 1;
        g.ca = a.count("conaffinity") ? std::stoi(a["conaffinity"]) : 1;
        g.margin = a.count("margin") ? std::stod(a["margin"]) : 0.0;
        g.body = body;
        geoms.push_back(g);
    }

    void walk(const XNode& node, int parent, const std::string& cc) {
        for (auto& kp : node.kids) {
            const XNode& k = *kp;
            if (k.tag == "geom") {
                add_geom(k, parent, cc);
            } else if (k.tag == "body") {
                auto chc = k.get("childclass");
                std::string ncc = chc ? *chc : cc;
                int bid = m.nbody();
                int jnt = -1, adr = -1;
                for (auto& jp : k.kids) {
                    std::string jt;
                    if (jp->tag == "freejoint") jt = "free";
                    else if (jp->tag == "joint") {
                        auto tt = jp->get("type");
                        if (tt) jt = *tt;
                        else {
                            auto c = jp->get("class");
                            AttrMap da = dfl.resolve(c ? *c : ncc, "joint");
                            jt = da.count("type") ? da["type"] : "hinge";
                        }
                    } else continue;
                    if (jt != "free") throw std::runtime_error("unsupported joint type '" + jt + "'");
                    if (jnt == 0) throw std::runtime_error("body with two free joints");
                    jnt = 0; adr = nq; nq += 7;
                }
                AttrMap ba;
                for (auto& kv : k.attrs) ba[kv.first] = kv.second;
                auto ps = floats(ba.count("pos") ? ba["pos"] : "0 0 0");
                if (ps.size() != 3) throw std::runtime_error("body pos needs 3 numbers");
                double q[4];
                orientation(ba, comp, q);
                m.body_names.push_back(ba.count("name") ? ba["name"] : "");
                m.body_parent.push_back(parent);
                m.body_jnt_type.push_back(jnt);
                m.body_qpos_adr.push_back(adr);
                for (int j = 0; j < 3; ++j) m.body_pos.push_back(ps[j]);
                for (int j = 0; j < 4; ++j) m.body_quat.push_back(q[j]);
                if (jnt == 0) {
                    for (int j = 0; j < 3; ++j) m.qpos0.push_back(ps[j]);
                    for (int j = 0; j < 4; ++j) m.qpos0.push_back(q[j]);
                }
                walk(k, bid, ncc);
            } else if (k.tag == "frame" || k.tag == "replicate" || k.tag == "attach") {
                throw std::runtime_error("unsupported MJCF element <" + k.tag + ">");
            }
        }
    }

    void run(const XNode& root) {
        if (root.tag != "mujoco") throw std::runtime_error("root element is not <mujoco>");
        for (auto& k : root.kids) {
            if (k->tag == "compiler") {
                if (auto a = k->get("angle")) comp.degree = (*a != "radian");
                if (auto s = k->get("eulerseq")) comp.seq = *s;
            } else if (k->tag == "include") {
                throw std::runtime_error("unsupported MJCF element <include>");
            }
        }
        dfl.parent["main"] = "";
        dfl.cls["main"];
        for (auto& k : root.kids)
            if (k->tag == "default") read_defaults(*k, dfl, "", true);
        // world body
        m.body_names.push_back("world");
        m.body_parent.push_back(-1);
        m.body_jnt_type.push_back(-1);
        m.body_qpos_adr.push_back(-1);
        for (int j = 0; j < 3; ++j) m.body_pos.push_back(0.0);
        m.body_quat.insert(m.body_quat.end(), {1.0, 0.0, 0.0, 0.0});
        for (auto& k : root.kids)
            if (k->tag == "worldbody") walk(*k, 0, "main");
        // geoms ordered body by body (stable within a body)
        for (int b = 0; b < m.nbody(); ++b) {
            for (auto& g : geoms) {
                if (g.body != b) continue;
                m.geom_names.push_back(g.name);
                m.geom_type.push_back(g.type);
                m.geom_body.push_back(g.body);
                m.geom_contype.push_back(g.ct);
                m.geom_conaffinity.push_back(g.ca);
                m.geom_size.insert(m.geom_size.end(), g.size, g.size + 3);
                m.geom_pos.insert(m.geom_pos.end(), g.pos, g.pos + 3);
                m.geom_quat.insert(m.geom_quat.end(), g.quat, g.quat + 4);
                m.geom_margin.push_back(g.margin);
            }
        }
        for (auto& k : root.kids) {
            if (k->tag != "contact") continue;
            for (auto& e : k->kids) {
                if (e->tag != "exclude") continue;
                auto b1 = e->get("body1"), b2 = e->get("body2");
                if (!b1 || !b2) throw std::runtime_error("<exclude> needs body1 and body2");
                int i1 = -1, i2 = -1;
                for (int b = 0; b < m.nbody(); ++b) {
                    if (m.body_names[b] == *b1) i1 = b;
                    if (m.body_names[b] == *b2) i2 = b;
                }
                if (i1 < 0 || i2 < 0) throw std::runtime_error("<exclude> names an unknown body");
                m.exclude.push_back(i1);
                m.exclude.push_back(i2);
            }
        }
    }
};

}  // namespace

int load_mjcf(const std::string& path, sspp_model& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return set_error(SSPP_E_IO, "Failed to load MJCF model: cannot open '" + path + "'");
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    try {
        XmlReader rd(text);
        auto root = rd.parse();
        sspp_model m;
        m.path = path;
        Loader L(m);
        L.run(*root);
        out = std::move(m);
    } catch (const std::exception& e) {
        std::string w = e.what();
        int code = w.find("unsupported") != std::string::npos ? SSPP_E_UNSUPPORTED : SSPP_E_SCENE;
        return set_error(code, "Failed to load MJCF model '" + path + "': " + w);
    }
    return SSPP_OK;
}

}  // namespace sspp
