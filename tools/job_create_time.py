"""Host time of SsppJob creation (pair tables incl. the phase-1 hit order) for the bench job,
per SSPP_PAIR_ORDER mode: python tools/job_create_time.py"""
import os
import subprocess
import sys
import time

if len(sys.argv) == 1:
    for mode in ("1", "2"):
        env = dict(os.environ, SSPP_PAIR_ORDER=mode)
        subprocess.check_call([sys.executable, __file__, "run"], env=env)
    sys.exit(0)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import sspp_amd as S

model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
scene = S.Scene(model, 0, 7)
n, W = 10, 128
start = np.array([0.5, 0.15, 0.136, 0.707, 0.0, 0.0, 0.707])
end = np.array([0.5, -0.05, 0.136, 0.707, 0.0, 0.0, 0.707])
u = np.array([i / (n - 1) for i in range(n)])
knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), W, max_batch=4096)  # warm the runtime
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    j = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), W, max_batch=4096)
    ts.append(time.perf_counter() - t0)
    del j
print("SSPP_PAIR_ORDER=%s job create ms: median %.2f min %.2f" % (os.environ["SSPP_PAIR_ORDER"],
      1e3 * sorted(ts)[2], 1e3 * min(ts)))
