"""Profiling helper: per-batch kernel time for the scoring path (robocrane sspp / stacking tsp).

    SSPP_ABLATE=<mask> SSPP_LIB_PATH=<variant .so> CONFIG=robocrane|stacking python tools/ablate.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sspp_amd as S  # noqa: E402

cfg = os.environ.get("CONFIG", "robocrane")
B = int(os.environ.get("B", "4096" if cfg == "robocrane" else "16384"))
if cfg == "robocrane":
    model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
    scene = S.Scene(model, 0, 7)
    start = np.array([0.5, 0.15, 0.136, 0.707, 0, 0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0, 0, 0.707])
    u = np.array([i / 9 for i in range(10)])
    knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
    jobs = [S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=B) for _ in range(4)]
    outs = [j.alloc(B) for j in jobs]
    job, o = jobs[0], outs[0]

    def run(i, best, k=0, stream=None):
        jobs[k].sample_score(i * B, B, outs[k]["arc"], outs[k]["feasible"],
                             best if k == 0 or best is None else outs[k]["best"], stream=stream)
    feas = lambda: int(o["feasible"].sum().item())  # noqa: E731
else:
    model = S.Model(os.path.join(S.SCENE_DIR, "stacking.xml"))
    scene = S.Scene(model, 1, "block1")
    start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
    end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
    jobs = [S.TspJob(scene, start, end, 1, 128, mean=(start + 0.5 * (end - start)).reshape(1, 4),
                     sigma=np.full((1, 4), 0.2), lo=np.array([-0.5, -0.5, 0.0, -1.6]),
                     hi=np.array([0.5, 0.5, 0.6, 1.6]), max_batch=B) for _ in range(4)]
    outs = [j.alloc(B) for j in jobs]
    job, o = jobs[0], outs[0]

    def run(i, best, k=0, stream=None):
        q = outs[k]
        jobs[k].sample_score(i * B, B, q["L"], q["Cnf"], q["Cwf"], q["status"], q["cost"],
                             best if k == 0 or best is None else q["best"], stream=stream)
    feas = lambda: int(o["status"].sum().item())  # noqa: E731
for i in range(20):
    run(i, o["best"])
torch.cuda.synchronize()
res = {}
for name, best in (("kernel_only", None), ("full_step", o["best"])):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(200):
        run(i, best)
    e1.record()
    torch.cuda.synchronize()
    res[name] = e0.elapsed_time(e1) / 200 * 1e3
import time  # noqa: E402
# host enqueue cost and two-stream pipelining (independent batches alternate streams)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(200):
    run(i, o["best"])
res["host_enqueue"] = (time.perf_counter() - t0) / 200 * 1e6
torch.cuda.synchronize()
streams = [torch.cuda.Stream() for _ in range(4)]
for ns in (2, 3, 4):
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(400):
            k = i % ns
            run(i, o["best"], k, streams[k])
        torch.cuda.synchronize()
        res["streams%d_wall" % ns] = (time.perf_counter() - t0) / 400 * 1e6
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(200):
    run(i, o["best"])
torch.cuda.synchronize()
res["one_stream_wall"] = (time.perf_counter() - t0) / 200 * 1e6
print(json.dumps(dict(env={k: v for k, v in os.environ.items() if k.startswith("SSPP_")}, config=cfg, lib=os.path.basename(os.environ.get("SSPP_LIB_PATH", "default")),
                      ablate=int(os.environ.get("SSPP_ABLATE", "0")), B=B, us=res, feasible=feas())))
