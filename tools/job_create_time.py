"""Host time of SsppJob creation (pair tables, waypoint order, the hit-order pre-pass) for the
bench job, per scan order: python tools/job_create_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import sspp_amd as S  # noqa: E402

model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
scene = S.Scene(model, 0, 7)
n, W = 10, 128
start = np.array([0.5, 0.15, 0.136, 0.707, 0.0, 0.0, 0.707])
end = np.array([0.5, -0.05, 0.136, 0.707, 0.0, 0.0, 0.707])
u = np.array([i / (n - 1) for i in range(n)])
knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
for sigma in (0.08, 0.0):  # a sampling job (hit order) and a scoring job (gap order)
    S.SsppJob(scene, knots, 3, ctrl0, sigma, np.ones(7), W, max_batch=4096)  # warm the runtime
    ts, cfg = [], None
    for _ in range(5):
        t0 = time.perf_counter()
        j = S.SsppJob(scene, knots, 3, ctrl0, sigma, np.ones(7), W, max_batch=4096)
        ts.append(time.perf_counter() - t0)
        cfg = j.config()
        del j
    print("sigma %.2f (%s order) job create ms: median %.2f min %.2f, pre-pass %.2f ms" % (
        sigma, cfg["pair_order"], 1e3 * sorted(ts)[2], 1e3 * min(ts), cfg["prepass_ms"]))
