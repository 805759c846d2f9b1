"""Where the driver-shaped region (bench.py --steps 20 --warmup 5) spends its time: host enqueue
(Python -> ctypes -> C++ executor -> hipLaunchKernel) versus the wait in torch.cuda.synchronize,
repeated; with SSPP_LIB_PATH pointing at an -DSSPP_ABLATE=64 variant the kernel is empty and the
region is the launch floor.  python tools/floor.py [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
args = bench.parse(["--steps", "20", "--warmup", "5", "--no-cpu-baseline"])
device = torch.device("cuda", 0)
B, step, kernel_only, bytes_per, flops_per, meta, ctx = bench.setup_robocrane(args, device)
run = bench.native_runner(args, ctx, B, 1, 0, device)
run(5)
torch.cuda.synchronize()
enq, wait, tot = [], [], []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(20)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enq.append(t1 - t0), wait.append(t2 - t1), tot.append(t2 - t0)
med = lambda v: float(np.median(v) * 1e6)  # noqa: E731
print(json.dumps({"library": os.environ.get("SSPP_LIB_PATH", "default"), "region_us_median": med(tot),
                  "enqueue_us_median": med(enq), "sync_wait_us_median": med(wait),
                  "region_us_min": float(np.min(tot) * 1e6)}))
