"""Per-workgroup timeline of one driver-shaped k_sspp_c2f launch (--steps 20 --warmup 5, 20
steps in one launch).  Needs a -DSSPP_WG_TIMING variant via SSPP_LIB_PATH.
    python tools/wg_timing.py [steps] [out.json]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from sspp_amd import _lib  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
out_path = sys.argv[2] if len(sys.argv) > 2 else None
sys.argv = ["bench.py", "--steps", str(steps), "--warmup", "5", "--no-cpu-baseline",
            "--steps-per-launch", str(min(steps, 32)), "--split", os.environ.get("WGT_SPLIT", "1")]
args = bench.parse()
device = torch.device("cuda", 0)
B, step, kernel_only, bytes_per, flops_per, meta, ctx = bench.setup_robocrane(args, device)
run = bench.native_runner(args, ctx, B, 1, 0, device)
run(5)
torch.cuda.synchronize()
run(steps)
torch.cuda.synchronize()
cfg = ctx["job"].config()  # the shape the timed launch ran
nt, g1 = (int(x) for x in cfg["shape"].split("x"))
cpb = (nt // 64) * (64 // g1)
nwg = steps * ((B + cpb - 1) // cpb)
buf = (C.c_ulonglong * (4 * nwg))()
_lib.lib().__getattr__("sspp_debug_wg_times")(buf, 4 * nwg)
a = np.frombuffer(buf, dtype=np.uint64).reshape(nwg, 4).astype(np.int64)
t0 = a[:, 0].min()
st = (a[:, 0] - t0) / 100.0  # wall clock: 100 MHz -> us
en = (a[:, 1] - t0) / 100.0
dur = en - st
ns = a[:, 3]
res = {"workgroups": int(nwg), "span_us": float(en.max()),
       "dur_us_pcts": {p: float(np.percentile(dur, p)) for p in (10, 50, 90, 99, 100)},
       "dur_us_by_survivors": {int(k): [int((ns == k).sum()), float(dur[ns == k].mean())]
                               for k in np.unique(ns)},
       "start_us_pcts": {p: float(np.percentile(st, p)) for p in (0, 10, 50, 90, 100)},
       "end_us_pcts": {p: float(np.percentile(en, p)) for p in (10, 50, 90, 99, 100)},
       "last_20_end": [[float(st[i]), float(en[i]), int(ns[i])] for i in np.argsort(en)[-20:]],
       "concurrency_at": {t: int(((st <= t) & (en > t)).sum()) for t in (5, 10, 20, 40, 60, 80)}}
ph = (C.c_ulonglong * (8 * nwg))()
_lib.lib().__getattr__("sspp_debug_wg_phases")(ph, 8 * nwg)
ph = np.frombuffer(ph, dtype=np.uint64).reshape(nwg, 8)[:, :7].astype(np.int64)
d = np.diff(ph, axis=1)  # shader clocks per phase
names = ["prologue_ctrl", "sampling", "phase1", "phase2", "phase3_arc", "epilogue_argmin"]
res["phase_clocks_mean"] = {n: float(d[:, i].mean()) for i, n in enumerate(names)}
res["phase_clocks_by_survivors"] = {int(k): {n: float(d[ns == k, i].mean()) for i, n in enumerate(names)}
                                    for k in np.unique(ns)}
if cfg.get("split"):  # the survivor queue: the last arriver's epilogue and every popped survivor
    b2 = (C.c_ulonglong * (8 * 4096))()
    _lib.lib().__getattr__("sspp_debug_p2_times")(b2, 8 * 4096)
    ep = np.frombuffer(b2, dtype=np.uint64).reshape(4096, 8)[4095].astype(np.int64)
    b3 = (C.c_ulonglong * (8 * 8192))()
    _lib.lib().__getattr__("sspp_debug_p2_waves")(b3, 8 * 8192)
    w = np.frombuffer(b3, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
    w = w[w[:, 0] >= t0]  # this launch's survivors (older slots hold earlier launches)
    ws, we = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0
    order = np.argsort(we)
    keys = sorted(set(map(tuple, w[:, 2:5].tolist())))
    sel = {k: (w[:, 2] == k[0]) & (w[:, 3] == k[1]) & (w[:, 4] == k[2]) for k in keys}
    res["p2"] = {"survivors": int(len(w)), "grid": int(ep[2]),
                 "epilogue_us": [float((ep[0] - t0) / 100.0), float((ep[1] - t0) / 100.0)],
                 "survivor_start_us_pcts": {p: float(np.percentile(ws, p)) for p in (0, 50, 90, 100)},
                 "survivor_end_us_pcts": {p: float(np.percentile(we, p)) for p in (10, 50, 90, 99, 100)},
                 "survivor_dur_us_pcts": {p: float(np.percentile(we - ws, p)) for p in (10, 50, 90, 99, 100)},
                 "by_passes(passes/fp64/feasible)": {"%d/%d/%d" % k: [int(m.sum()), float((we - ws)[m].mean()),
                                                                   float(w[m, 5].mean()), float(w[m, 6].mean())]
                                                      for k, m in sel.items()},
                 "last_10": [[float(ws[i]), float(we[i])] + w[i, 2:8].tolist() for i in order[-10:]]}
print(json.dumps(res, indent=1))
if out_path:
    json.dump(res, open(out_path, "w"), indent=1)
