"""Timeline of one k_sspp_wq1 + k_sspp_wq2 launch pair (a -DSSPP_WG_TIMING variant via
SSPP_LIB_PATH): per tile and per survivor item, wall-clock start / end (100 MHz) and shader-clock
phases.  python tools/wq_timing.py [steps_per_launch] [out.json]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sspp_amd as S  # noqa: E402
from sspp_amd import _lib  # noqa: E402

spl = int(sys.argv[1]) if len(sys.argv) > 1 else 1
out_path = sys.argv[2] if len(sys.argv) > 2 else None
L = _lib.lib()
model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
scene = S.Scene(model, 0, 7)
start = np.array([0.5, 0.15, 0.136, 0.707, 0.0, 0.0, 0.707])
end = np.array([0.5, -0.05, 0.136, 0.707, 0.0, 0.0, 0.707])
u = np.array([i / 9 for i in range(10)])
knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
B = 4096
job = S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), 128, max_batch=B)
arcs = [torch.empty(spl * B, dtype=torch.float64, device="cuda")]
feas = [torch.empty(spl * B, dtype=torch.uint8, device="cuda")]
ex = S.SsppSteps([job], [torch.cuda.current_stream()], B, arcs, feas, steps_per_launch=spl)
best = torch.zeros((spl, 4), dtype=torch.int64, device="cuda")
for i in range(20):
    ex.enqueue(spl, i * spl * B, B, best)
torch.cuda.synchronize()
L.sspp_debug_wq_reset()
ex.enqueue(spl, 999 * spl * B, B, best)
torch.cuda.synchronize()
n = 8 << 16
t = (C.c_ulonglong * n)()
it = (C.c_ulonglong * n)()
L.sspp_debug_wq_times(t, it, n)
t = np.frombuffer(t, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
it = np.frombuffer(it, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
t = t[t[:, 0] != 0]
it = it[it[:, 0] != 0]
w0 = t[:, 0].min()
ts, te = (t[:, 0] - w0) / 100.0, (t[:, 5] - w0) / 100.0
ph = np.diff(t[:, 1:5], axis=1)
res = {"steps_per_launch": spl, "tiles": int(len(t)),
       "tile_start_us": {p: float(np.percentile(ts, p)) for p in (0, 50, 90, 100)},
       "tile_end_us": {p: float(np.percentile(te, p)) for p in (10, 50, 90, 99, 100)},
       "tile_dur_us": {p: float(np.percentile(te - ts, p)) for p in (10, 50, 90, 99, 100)},
       "tile_clk_mean": dict(zip(["ctrl_sampling", "phase1_scan", "epilogue"], map(float, ph.mean(axis=0)))),
       "tile_clk_p99": dict(zip(["ctrl_sampling", "phase1_scan", "epilogue"], map(float, np.percentile(ph, 99, axis=0)))),
       "survivors": int(t[:, 6].sum()), "tiles_with_survivors": int((t[:, 6] > 0).sum())}
if len(it):
    cs, ce = (it[:, 0] - w0) / 100.0, (it[:, 5] - w0) / 100.0
    iph = np.diff(it[:, 1:5], axis=1)
    final = (it[:, 7] >> 32) & 1
    hit = (it[:, 7] >> 33) & 1
    hit0 = (it[:, 6] >> 32) & 1
    npairs = it[:, 6] & 0xffffffff
    res.update({"items": int(len(it)), "item_claim_us": {p: float(np.percentile(cs, p)) for p in (0, 50, 90, 100)},
                "item_end_us": {p: float(np.percentile(ce, p)) for p in (50, 90, 99, 100)},
                "item_dur_us": {p: float(np.percentile(ce - cs, p)) for p in (10, 50, 90, 99, 100)},
                "item_clk_mean": dict(zip(["build", "scan", "final"], map(float, iph.mean(axis=0)))),
                "item_clk_max": dict(zip(["build", "scan", "final"], map(float, iph.max(axis=0)))),
                "items_final": int(final.sum()), "items_hit": int(hit.sum()), "items_skipped": int(hit0.sum()),
                "item_pairs_mean": float(npairs.mean()),
                "scan_clk_no_hit_mean": float(iph[hit == 0, 1].mean()) if (hit == 0).any() else None,
                "scan_clk_hit_mean": float(iph[hit == 1, 1].mean()) if (hit == 1).any() else None,
                "slowest_items": [[float(cs[i]), float(ce[i]), int(npairs[i]), int(hit[i]), int(final[i]),
                                   [int(x) for x in iph[i]]] for i in np.argsort(ce)[-8:]]})
print(json.dumps(res, indent=1))
if out_path:
    json.dump(res, open(out_path, "w"), indent=1)
