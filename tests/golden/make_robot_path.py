"""Fixture: the reference's only real robot path, scripts/bspline_params.npy.

Run ONLY in the build container (needs /root/reference; never on the GPU box):
    python tests/golden/make_robot_path.py

The file is what /root/reference/scripts/main_bspline.py:198-209 saves: a 0-d object array
holding {"knot_vec": f8[10], "ctr_pts": f8[7, 9], "k": 2} (np.save of a dict).  It is NOT
unpickled: numpy.load(allow_pickle=False) refuses it, and torch's weights-only unpickler
(torch.load(weights_only=True)'s loader, numpy's reconstruct globals allow-listed) refuses its
protocol-3 SHORT_BINBYTES opcode.  Instead pickletools.genops tokenizes the byte stream — it
builds no object and calls nothing — and this script checks that the stream has exactly the
expected structure (the dict keys, the two ndarray reconstructions with their shapes, dtype
'<f8', C order, the raw data bytes, k = 2) and decodes the data bytes with np.frombuffer.

Outputs tests/golden/robot_path.json: the knots, the 7 x 9 control points and k, plus the
reference's own BSplines.bspline (imported with `casadi` stubbed, as make_golden.py does) at
u = i / 127, i = 0..127, and the joint-space arc length over those points (H7's chord sum).
"""
import importlib.util
import json
import os
import pickletools
import sys
import types

import numpy as np

NPY = "/root/reference/scripts/bspline_params.npy"
REF = "/root/reference/sspp"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "robot_path.json")


def parse_npy_dict(path):
    raw = open(path, "rb").read()
    assert raw[:6] == b"\x93NUMPY" and raw[6] == 1, "npy v1 header"
    hl = int.from_bytes(raw[8:10], "little")
    header = raw[10:10 + hl].decode("latin1")
    assert "'descr': '|O'" in header and "'shape': ()" in header, header
    ops = [(op.name, arg) for op, arg, _ in pickletools.genops(raw[10 + hl:])]
    globals_ = {arg for name, arg in ops if name == "GLOBAL"}
    assert globals_ == {"numpy.core.multiarray _reconstruct", "numpy ndarray", "numpy dtype"}, globals_
    out, key, shape = {}, None, None
    for i, (name, arg) in enumerate(ops):
        if name == "BINUNICODE" and arg in ("knot_vec", "ctr_pts", "k"):
            key, shape = arg, None
        elif key and name in ("BININT1", "BININT") and shape is None and ops[i - 1][0] == "MARK":
            # state tuple of ndarray.__setstate__: (version, shape, dtype, is_fortran, data)
            dims = []
            j = i + 1
            while ops[j][0] in ("BININT1", "BININT"):
                dims.append(ops[j][1])
                j += 1
            assert ops[j][0] in ("TUPLE1", "TUPLE2", "TUPLE3", "TUPLE"), ops[j]
            shape = tuple(dims)
        elif key in ("knot_vec", "ctr_pts") and name in ("SHORT_BINBYTES", "BINBYTES") and shape:
            assert ops[i - 1][0] == "NEWFALSE", "C order"
            assert len(arg) == 8 * int(np.prod(shape))
            out[key] = np.frombuffer(arg, dtype="<f8").reshape(shape).copy()
            key = None
        elif key == "k" and name == "BININT1":
            out["k"] = int(arg)
            key = None
    assert sorted(out) == ["ctr_pts", "k", "knot_vec"], sorted(out)
    return out


def main():
    d = parse_npy_dict(NPY)
    knots, ctrl, k = d["knot_vec"], d["ctr_pts"], d["k"]
    assert knots.shape == (10,) and ctrl.shape == (7, 9) and k == 2
    sys.modules.setdefault("casadi", types.ModuleType("casadi"))
    spec = importlib.util.spec_from_file_location("ref_BSplines", os.path.join(REF, "BSplines.py"))
    bs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bs)
    W = 128
    us = [i / (W - 1) for i in range(W)]
    pts = np.array([np.asarray(bs.bspline(u, knots, ctrl, k), np.float64) for u in us])
    arc = float(np.sum(np.linalg.norm(np.diff(pts, axis=0), axis=1)))
    json.dump({"source": "scripts/bspline_params.npy (reference; main_bspline.py:198-209), tokenized "
                         "with pickletools.genops, never unpickled",
               "k": k, "knots": knots.tolist(), "ctrl": ctrl.tolist(),
               "W": W, "u": us, "bspline": pts.tolist(), "arc_length": arc},
              open(OUT, "w"), indent=1)
    print("wrote", OUT, "arc", arc)


if __name__ == "__main__":
    main()
