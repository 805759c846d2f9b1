"""Independent MJCF reader for the oracle — TEST INFRASTRUCTURE ONLY.

Reads the subset of MJCF the shipped scenes use (``mjcf/robocrane/robocrane.xml``,
``mjcf/stacking.xml``, ``mjcf/planner.xml`` in the reference) into the flat MuJoCo-like
arrays ``oracle/sspp_oracle.h::or_model`` expects.  It is written separately from the
product's C++ loader (``sspp_amd/csrc/mjcf.cpp``) so the two can be cross-checked.

MuJoCo semantics restated (mj_loadXML / mjCModel::Compile, MuJoCo unpinned):
  * bodies in depth-first pre-order, world body = 0; geoms ordered body by body;
  * free joints (``<freejoint/>`` or ``<joint type="free"/>``) get 7 qpos each in body
    order, qpos0 = (body pos, normalised body quat);
  * default classes nest; an element uses ``class=`` or the innermost ``childclass``
    of its enclosing bodies, else ``main``; explicit attributes win;
  * quaternions are normalised at compile time; ``euler`` honours ``<compiler angle>``
    and ``eulerseq``;
  * ``<contact><exclude body1 body2/>`` pairs.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET

import numpy as np

GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4,
              "cylinder": 5, "box": 6, "mesh": 7, "sdf": 8}


def _floats(s):
    return [float(x) for x in s.split()]


def _normq(q):
    n = math.sqrt(sum(x * x for x in q))
    return [x / n for x in q] if n > 0 else [1.0, 0.0, 0.0, 0.0]


def _qmul(a, b):
    return [a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
            a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
            a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
            a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]]


class _Defaults:
    def __init__(self):
        self.cls = {}  # name -> {elemtag: {attr: value}}
        self.parent = {}

    def resolve(self, cls, tag):
        chain = []
        c = cls
        while c is not None:
            chain.append(c)
            c = self.parent.get(c)
        out = {}
        for c in reversed(chain):
            out.update(self.cls.get(c, {}).get(tag, {}))
        return out


def _read_defaults(node, dfl, parent):
    name = node.get("class", "main")
    dfl.parent[name] = parent
    dfl.cls.setdefault(name, {})
    for ch in node:
        if ch.tag == "default":
            _read_defaults(ch, dfl, name)
        else:
            dfl.cls[name].setdefault(ch.tag, {}).update(ch.attrib)


def _orientation(attrs, compiler):
    if "quat" in attrs:
        return _normq(_floats(attrs["quat"]))
    if "euler" in attrs:
        e = _floats(attrs["euler"])
        if compiler["angle"] == "degree":
            e = [math.radians(x) for x in e]
        q = [1.0, 0.0, 0.0, 0.0]
        seq = compiler["eulerseq"]
        for ang, ax in zip(e, seq):
            axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ax.lower()]
            r = [math.cos(ang / 2)] + [math.sin(ang / 2) * a for a in axis]
            q = _qmul(q, r) if ax.islower() else _qmul(r, q)
        return _normq(q)
    if "axisangle" in attrs:
        v = _floats(attrs["axisangle"])
        ang = math.radians(v[3]) if compiler["angle"] == "degree" else v[3]
        n = math.sqrt(v[0] ** 2 + v[1] ** 2 + v[2] ** 2)
        s = math.sin(ang / 2) / n
        return _normq([math.cos(ang / 2), v[0] * s, v[1] * s, v[2] * s])
    return [1.0, 0.0, 0.0, 0.0]


def load(path):
    root = ET.parse(path).getroot()
    compiler = {"angle": "degree", "eulerseq": "xyz"}
    for c in root.iter("compiler"):
        compiler["angle"] = c.get("angle", compiler["angle"])
        compiler["eulerseq"] = c.get("eulerseq", compiler["eulerseq"])
    dfl = _Defaults()
    dfl.cls["main"] = {}
    dfl.parent["main"] = None
    for d in root.findall("default"):
        # the top-level <default> is class "main"; nested ones name themselves
        for ch in d:
            if ch.tag == "default":
                _read_defaults(ch, dfl, "main")
            else:
                dfl.cls["main"].setdefault(ch.tag, {}).update(ch.attrib)

    bodies = [dict(name="world", parent=-1, pos=[0.0] * 3, quat=[1.0, 0, 0, 0], jnt=-1, adr=-1)]
    body_geoms = [[]]
    nq = [0]
    qpos0 = []

    def geom_attrs(node, childclass):
        cls = node.get("class", childclass)
        a = dfl.resolve(cls, "geom")
        a.update(node.attrib)
        return a

    def add_geom(node, bid, childclass):
        a = geom_attrs(node, childclass)
        gtype = GEOM_TYPES[a.get("type", "sphere")]
        size = _floats(a.get("size", "0 0 0")) + [0.0, 0.0, 0.0]
        body_geoms[bid].append(dict(
            name=a.get("name", ""), type=gtype, size=size[:3],
            pos=_floats(a.get("pos", "0 0 0")), quat=_orientation(a, compiler),
            contype=int(a.get("contype", "1")), conaffinity=int(a.get("conaffinity", "1")),
            margin=float(a.get("margin", "0"))))

    def walk(node, parent, childclass):
        for ch in node:
            if ch.tag == "geom":
                add_geom(ch, parent, childclass)
            elif ch.tag == "body":
                cc = ch.get("childclass", childclass)
                battr = dict(ch.attrib)
                bid = len(bodies)
                jnt, adr = -1, -1
                for j in ch:
                    if j.tag == "freejoint":
                        jt = "free"
                    elif j.tag == "joint":
                        jt = j.get("type") or dfl.resolve(j.get("class", cc), "joint").get(
                            "type", "hinge")
                    else:
                        continue
                    if jt != "free":
                        raise ValueError("unsupported joint type %r in %s" % (jt, path))
                    jnt, adr = 0, nq[0]
                    nq[0] += 7
                pos = _floats(battr.get("pos", "0 0 0"))
                quat = _orientation(battr, compiler)
                bodies.append(dict(name=battr.get("name", ""), parent=parent, pos=pos,
                                   quat=quat, jnt=jnt, adr=adr))
                body_geoms.append([])
                if jnt == 0:
                    qpos0.extend(pos + quat)
                walk(ch, bid, cc)

    wb = root.find("worldbody")
    walk(wb, 0, "main")

    excludes = []
    names = {b["name"]: i for i, b in enumerate(bodies)}
    for c in root.findall("contact"):
        for e in c.findall("exclude"):
            excludes.append((names[e.get("body1")], names[e.get("body2")]))

    geoms = []
    for bid, gl in enumerate(body_geoms):
        for g in gl:
            g["body"] = bid
            geoms.append(g)

    m = dict(
        body_names=[b["name"] for b in bodies],
        geom_names=[g["name"] for g in geoms],
        body_parent=np.array([b["parent"] for b in bodies], np.int32),
        body_jnt_type=np.array([b["jnt"] for b in bodies], np.int32),
        body_qpos_adr=np.array([b["adr"] for b in bodies], np.int32),
        body_pos=np.array([b["pos"] for b in bodies], np.float64).reshape(-1, 3),
        body_quat=np.array([b["quat"] for b in bodies], np.float64).reshape(-1, 4),
        geom_type=np.array([g["type"] for g in geoms], np.int32),
        geom_body=np.array([g["body"] for g in geoms], np.int32),
        geom_contype=np.array([g["contype"] for g in geoms], np.int32),
        geom_conaffinity=np.array([g["conaffinity"] for g in geoms], np.int32),
        geom_size=np.array([g["size"] for g in geoms], np.float64).reshape(-1, 3),
        geom_pos=np.array([g["pos"] for g in geoms], np.float64).reshape(-1, 3),
        geom_quat=np.array([g["quat"] for g in geoms], np.float64).reshape(-1, 4),
        geom_margin=np.array([g["margin"] for g in geoms], np.float64),
        exclude=np.array(excludes, np.int32).reshape(-1, 2),
        qpos0=np.array(qpos0, np.float64),
    )
    return m
