"""One rank of tests/test_multiproc_gpu.py: a gloo process group whose ranks share cuda:0.

    python tests/mp_worker.py MODE WORLD RANK PORT OUT.json [BATCH]

MODE steps: bench.py's robocrane step protocol (bench.native_runner: executor launches on two
            streams, one all-gather of the chunk's per-step argmin records, device reduction)
MODE ces:   CesPlanner.step with world ranks, driven on a non-default stream
Every rank writes its results to OUT.json.  Test infrastructure only.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mode, world, rank, port, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    batch = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if world > 1:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % port, world_size=world,
                                rank=rank)
    import bench
    import sspp_amd as S
    res = {}
    if mode == "steps":
        argv = sys.argv
        sys.argv = ["bench.py", "--streams", "2", "--steps-per-launch", "4", "--chunk", "12",
                    "--batch", str(batch or 4096)]
        args = bench.parse()
        sys.argv = argv
        B, _, _, _, _, _, ctx = bench.setup_robocrane(args, dev)
        recs = []
        run = bench.native_runner(args, ctx, B, world, rank, dev,
                                  on_chunk=lambda r: recs.append(r.clone()))
        run(30)  # chunks of 12, 12, 6 steps
        torch.cuda.synchronize()
        res["records"] = [x.cpu().numpy().tolist() for x in recs]
    elif mode == "ces":
        model = S.Model(os.path.join(S.SCENE_DIR, "stacking.xml"))
        scene = S.Scene(model, 1, model.body_id("block1"))
        pl = S.CesPlanner(scene, sample_count=777, check_points=64, limits_min=(-0.5, -0.5, 0.0, -1.6),
                          limits_max=(0.5, 0.5, 0.6, 1.6), world=world, rank=rank)
        start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
        end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
        stream = torch.cuda.Stream(dev)  # not torch's current stream
        its = []
        for t in range(4):
            pl.step(start, end, iterate=t > 0, stream=stream)
            stream.synchronize()
            r = pl.read()
            its.append({k: np.asarray(r[k]).tolist() for k in ("mean", "sigma", "last_best", "elites")}
                       | {"best_slot": r["best_slot"], "n_success": r["n_success"]})
        res["iterations"] = its
    else:
        raise SystemExit("unknown mode " + mode)
    with open(out, "w") as f:
        json.dump(res, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
