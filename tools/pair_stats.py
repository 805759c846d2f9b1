"""Analysis (oracle-based, CPU): which collision pairs end the phase-1 scan of k_sspp_c2f.

For config-2 candidates, evaluates the phase-1 waypoints (first G1 of the coarse-to-fine order)
and reports, per pair, how often it has a contact at any of them — the pairs worth testing first.
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import mjcf_ref  # noqa: E402
from oracle import oracle as O  # noqa: E402

path = os.path.join(os.path.dirname(__file__), "..", "sspp_amd", "scenes", "robocrane.xml")
model = mjcf_ref.load(path)
sc = O.Scene(model, 0, 7)
L = O.lib()
L.or_point_pair_contacts.restype = C.c_int
L.or_point_pair_contacts.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_void_p, C.c_void_p, C.c_void_p]
start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
u = np.array([i / 9 for i in range(10)])
knots, ctrl0 = O.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
B, W, G1 = 1024, 128, 16


def order(W):
    out, cur = [], [(0, W)]
    while cur:
        nxt = []
        for lo, hi in cur:
            if lo > hi:
                continue
            mid = lo + (hi - lo) // 2
            out.append(mid)
            nxt += [(lo, mid - 1), (mid + 1, hi)]
        cur = nxt
    return out


ords = order(W)[:G1]
ctrl = O.sample_sspp(ctrl0, 3, 0.08, np.ones(7), 0x5EED, 0, B)
cnt = np.zeros(64, np.int32)
g1 = np.zeros(64, np.int32)
g2 = np.zeros(64, np.int32)
npair = None
hits = []
for b in range(B):
    h = np.zeros(64, bool)
    for i in ords:
        q = O.spline_eval(knots, 3, ctrl[b], i / W)
        npair = L.or_point_pair_contacts(sc.ptr, q.ctypes.data_as(C.POINTER(C.c_double)),
                                         cnt.ctypes.data, g1.ctypes.data, g2.ctypes.data)
        h[:npair] |= cnt[:npair] > 0
    hits.append(h[:npair])
hits = np.array(hits)
names = model.get("geom_names") if isinstance(model, dict) else None
print("pairs", npair, "candidates with a phase-1 contact:", hits.any(1).mean())
for k in np.argsort(-hits.mean(0)):
    nm = ("%s-%s" % (names[g1[k]], names[g2[k]])) if names else "%d-%d" % (g1[k], g2[k])
    print("%3d %-40s hit frac %.3f  only-this %.3f" % (k, nm, hits[:, k].mean(),
                                                       (hits[:, k] & (hits.sum(1) == 1)).mean()))
