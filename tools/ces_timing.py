"""Per-kernel timing of one CES iteration (begin / eval / update) on the multi-goal problem.
    python tools/ces_timing.py [samples] [goal]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import sspp_amd as S  # noqa: E402


def main(samples=4096, goal=0):
    model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
    scene = S.Scene(model, 1, model.body_id("gripper_collision_with_block/"))
    pl = S.CesPlanner(scene, sample_count=samples, check_points=128, init_points=3,
                      limits_min=bench.MG_LO, limits_max=bench.MG_HI)
    st, en = bench.MULTIGOAL[goal]
    pl.plan(st, en, iterate=False, iterations=3)
    torch.cuda.synchronize()
    out = {}
    for name, fn in (("begin", lambda: pl.begin(st, en, True)), ("eval", lambda: pl.eval()),
                     ("update", lambda: pl.update())):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            fn()
        e0.record()
        for _ in range(100):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = e0.elapsed_time(e1) * 10.0
    r = pl.read()
    out.update(n_success=r["n_success"], n_elite=r["n_elite"], samples=samples)
    print(json.dumps(out))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
