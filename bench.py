"""Benchmark: candidate paths scored per second (BASELINE.json metric), MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config robocrane|stacking|multigoal]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

--gpus N means N ranks, one per GPU: run without WORLD_SIZE and N > 1, bench.py starts itself
under torch.distributed.run as a child process (before anything touches a GPU), forwards its
output and exits with its status; under a launcher, WORLD_SIZE must equal N.

A step is one pass of the hot path over one batch of synthetic candidates: on-device Philox
sampling of the perturbed control points, B-spline evaluation, free-joint FK, collision against
the scene, arc-length cost and the argmin over feasible candidates (include/sspp.h:194-225).
Default workload = BASELINE.json configs[1]: SamplingPathPlanner7 on the robocrane scene,
4096 candidates x 128 waypoints per GPU (weak scaling: every rank scores its own 4096
candidates with globally unique Philox ids; the per-step global argmin is one RCCL all-gather
of a 32-byte record per rank, reduced on the device). Consecutive steps are independent
batches and alternate over --streams (default 2) HIP streams, each with its own job, so one
batch's argmin tail and launch gap hide under the next batch's scoring.

Printed (rank 0): one JSON line with value = candidates scored per second over all ranks,
a `roofline` object for the dominant kernel (k_sspp_c2f), a `binding_roofline` (FP64 VALU) object, and a
`cpu_baseline` object (the oracle — test infrastructure, oracle/ — timed on a bounded sample
of the same workload on the host cores, N=1 only, with a parity check on that sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
# kernel revision: PMC records (profiles/*_latest.json) measured on another revision of the
# kernels are not attached to a line (tools/update_latest.py stamps them)
KERNEL_REV = "r06"
FP64_PEAK_TFLOPS = 78.6    # FP64 vector (VALU) spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: robocrane 8192, stacking 1024, multigoal 128)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default: steps / 32)")
    ap.add_argument("--config", default="robocrane", choices=["robocrane", "stacking", "multigoal"])
    ap.add_argument("--batch", type=int, default=0, help="candidates per GPU per step (default: config)")
    ap.add_argument("--waypoints", type=int, default=128)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-launches", type=int, default=200)
    ap.add_argument("--streams", type=int, default=4,
                    help="independent batches in flight (one job + stream/graph branch each)")
    ap.add_argument("--mode", default="native", choices=["native", "eager", "dropin", "tsp-anytime"],
                    help="native: the C++ step executor enqueues --chunk steps per call "
                         "(robocrane); eager: one Python-level launch per step; dropin: "
                         "per-call latency of the reference's entry point "
                         "_sspp.SamplingPathPlanner7.plan (src/sspp_bindings.cpp:43-50); "
                         "tsp-anytime: the reference's ICRA anytime loop over "
                         "_tsp.TaskSpacePlanner.plan (src/main_icra_benchmark.cpp:67-89)")
    ap.add_argument("--sampler", default="fp64", choices=["fp64", "fp32"],
                    help="robocrane sampleWithNoise normals: fp64 Box-Muller (default, bit-exact "
                         "oracle) or the opt-in fp32 quad sampler")
    ap.add_argument("--budgets-ms", default="10,20,50", help="tsp-anytime: wall-clock budgets")
    ap.add_argument("--tsp-form", type=int, default=None,
                    help="stacking: force the k_tsp form (SSPP_OPT_TSP_FORM 0..3; tuning, every form "
                         "gives bit-identical results)")
    ap.add_argument("--tsp-rep", type=int, default=None,
                    help="stacking: k_tsp sub-batches per workgroup (SSPP_OPT_TSP_REP 1..16, -1 by "
                         "batch size; tuning, bit-identical results)")
    ap.add_argument("--mg-group", type=int, default=1, choices=[0, 1],
                    help="multigoal: this rank's goals as one chain of batched launches per "
                         "iteration (sspp_ces_plan_group, one k_tsp_group over every goal; default) "
                         "or one planner per stream (A/B; results identical)")
    ap.add_argument("--mg-chunk", type=int, default=1,
                    help="multigoal: iterations per goal before the next goal's (0: all of a goal's "
                         "iterations in one call)")
    ap.add_argument("--shape", default="",
                    help="robocrane: force the k_sspp_c2f launch shape NTxG1 (e.g. 64x4; tuning, "
                         "default: chosen per launch by the library); the line reports it")
    ap.add_argument("--scan", default="fp32", choices=["fp32", "fp64"],
                    help="robocrane: k_sspp_c2f's FP32-filtered scan (default; FP64 decides whatever "
                         "FP32 cannot certify, results identical) or the all-FP64 scan (A/B)")
    ap.add_argument("--split", type=int, default=1, choices=[0, 1],
                    help="robocrane: split multi-step launches (k_sspp_c2f's workgroups queue their "
                         "phase-1 survivors and finish queued survivors; default) or each workgroup "
                         "finishes its own (A/B; results identical)")
    ap.add_argument("--chunk", type=int, default=80, help="native mode: steps per executor call")
    ap.add_argument("--steps-per-launch", type=int, default=40,
                    help="native mode: independent steps (each its own B candidates, outputs and "
                         "argmin) grouped into one kernel launch; 40 x 4096 candidates = 5120 "
                         "workgroups of 128 x 4 = two resident rounds of the chip")
    a = ap.parse_args(argv)
    if a.steps is None and a.mode == "tsp-anytime":
        a.steps = 10  # trials per budget and mode
    if a.steps is None:
        a.steps = {"robocrane": 8192, "stacking": 1024, "multigoal": 128}[a.config]
    if a.warmup is None:
        a.warmup = max(1, a.steps // 32)
    return a


def roofline_spl(args):
    """Steps per launch of the roofline launches: the timed loop's launch shape, i.e. the
    executor's steps per launch, or all the timed steps when they are fewer (the driver's
    --steps 20 run is one launch of 20 steps)."""
    return min(args.steps, args.steps_per_launch) if args.mode == "native" else 1


def setup_robocrane(args, device):
    import sspp_amd as S
    model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
    scene = S.Scene(model, 0, 7)
    start = np.array([0.5, 0.15, 0.136, 0.707, 0.0, 0.0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0.0, 0.0, 0.707])
    n, W = 10, args.waypoints
    u = np.array([i / (n - 1) for i in range(n)])
    knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
    B = args.batch or 4096
    sampler = S.SAMPLER_FP32 if args.sampler == "fp32" else S.SAMPLER_FP64
    jobs = [S.SsppJob(scene, knots, 3, ctrl0, 0.08, np.ones(7), W, seed=S.DEFAULT_SEED, max_batch=B,
                      sampler=sampler) for _ in range(args.streams)]
    if args.shape:
        nt, g1 = (int(x) for x in args.shape.lower().split("x"))
        for j in jobs:
            j.set_shape(nt, g1)
    for j in jobs:
        j.set_option(S.OPT_F32, 1 if args.scan == "fp32" else 0)
        j.set_option(S.OPT_SPLIT, args.split)
    bufs = [j.alloc(B, device=device) for j in jobs]
    job = jobs[0]

    def step(first_id, best, lane=0, stream=None):
        jobs[lane].sample_score(first_id, B, bufs[lane]["arc"], bufs[lane]["feasible"], best,
                                stream=stream)

    roof = {}

    def kernel_only(first_id):
        # one launch exactly as the timed loop issues it: steps_per_launch steps of B
        # candidates (each with its own outputs and argmin record), on the current stream
        import torch
        spl = roofline_spl(args)
        if spl == 1:
            job.sample_score(first_id, B, bufs[0]["arc"], bufs[0]["feasible"], None)
            return
        if "ex" not in roof:
            roof["ex"] = make_executor([torch.cuda.current_stream()], spl, jobs[:1])
            roof["best"] = torch.zeros((spl, 4), dtype=torch.int64, device=device)
        roof["ex"].enqueue(spl, first_id * spl, B, roof["best"])

    def make_executor(streams, spl, js=None):
        import torch
        js = jobs if js is None else js
        arcs = [torch.empty(spl * B, dtype=torch.float64, device=device) for _ in js]
        feas = [torch.empty(spl * B, dtype=torch.uint8, device=device) for _ in js]
        return S.SsppSteps(js, streams[:len(js)], B, arcs, feas, steps_per_launch=spl)

    def isolated_step_us(n=30):
        # one B-candidate launch alone on the idle current stream, HIP events around each
        import torch
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for i in range(n + 5):
            e0.record(st)
            job.sample_score((1 << 41) + i * B, B, bufs[0]["arc"], bufs[0]["feasible"], None)
            e1.record(st)
            torch.cuda.synchronize()
            if i >= 5:
                ts.append(e0.elapsed_time(e1) * 1e3)
        return float(np.median(ts))

    def set_order(order):
        for j in jobs:
            j.set_option(S.OPT_ORDER, order)

    def validate():
        # after the timed region: no split launch of any job lost a survivor (the queue's
        # lost-work check, cumulative per job; a loss would also be in that step's record)
        lost = sum(j.get_option(S._lib.OPT_SPLIT_LOST) for j in jobs)
        if lost:
            raise S.SsppError("split launches lost %d survivors" % lost)
        return dict(split_lost=lost, split_handoffs=sum(j.get_option(S._lib.OPT_SPLIT_HANDOFFS) for j in jobs))

    def timed_instance(first_id):
        # one launch exactly as the timed loop issues it (the roofline's executor: jobs[0], the
        # timed steps per launch); returns per-step (arc, feasible) of steps 0 and spl - 1, the
        # launch's records and whether it was split
        import torch
        spl = roofline_spl(args)
        if spl == 1:
            return None
        if "ex" not in roof:
            kernel_only(0)  # builds the executor (the roofline launches normally have)
        roof["ex"].enqueue(spl, first_id, B, roof["best"])
        torch.cuda.synchronize()
        arc, fe = roof["ex"].arc_bufs[0].cpu().numpy(), roof["ex"].feas_bufs[0].cpu().numpy()
        steps = sorted({0, spl - 1})
        return dict(spl=spl, steps=steps, split=bool(job.get_option(S._lib.OPT_LAST_SPLIT)),
                    shape=job.config()["shape"], records=S.check_records(roof["best"]),
                    arc={i: arc[i * B:(i + 1) * B] for i in steps}, feas={i: fe[i * B:(i + 1) * B] for i in steps})

    n_, D, p = 10, 7, 3
    # SURVEY §8(d) algorithmic work per candidate
    bytes_per = n_ * D * 8 + 8 + 1
    flops_per = (2 * W + 1) * 2 * (p + 1) * D + (W - 1) * (3 * D + 1) + \
        (W + 1) * (40 + 42 + 48 + 8 * 450 + 300)
    meta = dict(workload="robocrane SamplingPathPlanner7 (block_green free joint), sigma 0.08",
                candidates_per_gpu=B, waypoints=W, init_points=n_, degree=p, dof=D)
    # the job's effective configuration (sampler, launch shape, scan orders, the creation's
    # hit-order pre-pass), read back from the library after the timed region
    ctx = dict(kind="sspp", kernel_name="k_sspp_c2f", effective=job.config,
               job=job, knots=knots, ctrl0=ctrl0, W=W, scene_path=model.path, p=p,
               make_executor=make_executor, isolated_step_us=isolated_step_us, set_order=set_order,
               validate=validate, timed_instance=timed_instance, per_launch=B * roofline_spl(args))
    return B, step, kernel_only, bytes_per, flops_per, meta, ctx


def setup_stacking(args, device):
    import sspp_amd as S
    model = S.Model(os.path.join(S.SCENE_DIR, "stacking.xml"))
    scene = S.Scene(model, 1, "block1")
    start = model.body_point("block1") + np.array([0, 0, 0.02, 0])
    end = model.body_point("block2") + np.array([0, 0, 0.22, 0])
    K, cp = 1, args.waypoints
    mean = (start + 0.5 * (end - start)).reshape(1, 4)
    sigma = np.full((1, 4), 0.2)
    lo, hi = np.array([-0.5, -0.5, 0.0, -1.6]), np.array([0.5, 0.5, 0.6, 1.6])
    B = args.batch or 16384
    jobs = [S.TspJob(scene, start, end, K, cp, mean=mean, sigma=sigma, lo=lo, hi=hi, z_min=0.0,
                     max_batch=B) for _ in range(args.streams)]
    if args.tsp_form is not None:
        for j in jobs:
            j.set_option(S.OPT_TSP_FORM, args.tsp_form)
    if args.tsp_rep is not None:
        for j in jobs:
            j.set_option(S.OPT_TSP_REP, args.tsp_rep)
    bufs = [j.alloc(B, device=device) for j in jobs]
    job = jobs[0]

    def step(first_id, best, lane=0, stream=None):
        q = bufs[lane]
        jobs[lane].sample_score(first_id, B, q["L"], q["Cnf"], q["Cwf"], q["status"], q["cost"],
                                best, stream=stream)

    def kernel_only(first_id):
        q = bufs[0]
        job.sample_score(first_id, B, q["L"], q["Cnf"], q["Cwf"], q["status"], q["cost"], None)

    n_, D = K + 2, 4
    bytes_per = n_ * D * 8 + 8 + 1
    flops_per = (2 * cp + 1) * 2 * 3 * D + cp * (3 * D + 1) + cp * (40 + 42 + 48 + 2 * 450)
    meta = dict(workload="stacking.xml TaskSpacePlanner (block1), K=1 via, sigma 0.2",
                candidates_per_gpu=B, waypoints=cp, vias=K, degree=2, dof=4)
    # the k_tsp form of the timed launches (SSPP_OPT_TSP_FORM read-back: 0 inline narrowphase,
    # 3 deferred box-box contact polygons, ...)
    ctx = dict(kind="tsp", job=job, start=start, end=end, mean=mean, sigma=sigma, lo=lo, hi=hi,
               cp=cp, scene_path=model.path, body=model.body_id("block1"),
               effective=lambda: dict(tsp_form=int(job.get_option(S.OPT_TSP_FORM)),
                                      tsp_rep=int(job.get_option(S.OPT_TSP_REP))))
    return B, step, kernel_only, bytes_per, flops_per, meta, ctx


# BASELINE.json configs[4] ("TSP multi-goal", SURVEY 8(d) row 5 — build-defined: the reference
# has no multi-goal logic): 8 independent TaskSpacePlanner problems on robocrane.xml with the
# free gripper (7 collidable geoms) moving between fixed (start, goal) pairs around the lego
# wall; 4096 sampled via sets (+ mean set + forwarded best) per problem and CES iteration.
MULTIGOAL = [((0.5, 0.15, 0.27, 0.0), (0.5, -0.05, 0.27, 0.0)),
             ((0.5, -0.05, 0.27, 0.0), (0.5, 0.15, 0.27, 0.0)),
             ((0.5, 0.15, 0.27, 1.5708), (0.5, -0.05, 0.27, 1.5708)),
             ((0.3, 0.05, 0.22, 0.0), (0.7, 0.05, 0.22, 0.0)),
             ((0.7, 0.05, 0.22, 0.0), (0.3, 0.05, 0.22, 0.0)),
             ((0.35, 0.2, 0.25, 0.0), (0.65, -0.1, 0.25, 0.5)),
             ((0.65, 0.2, 0.25, 0.0), (0.35, -0.1, 0.25, -0.5)),
             ((0.5, 0.25, 0.3, 0.0), (0.5, -0.15, 0.22, 0.0))]
MG_LO, MG_HI = (0.0, -0.4, 0.0, -1.6), (1.0, 0.5, 0.8, 1.6)


def setup_multigoal(args, device, world, rank):
    """One CES iteration of every goal this rank owns (goal g -> rank g % world) per step."""
    import torch
    import sspp_amd as S
    model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
    body = model.body_id("gripper_collision_with_block/")
    scene = S.Scene(model, 1, body)
    samples, cp = args.batch or 4096, args.waypoints
    mine = [g for g in range(len(MULTIGOAL)) if g % world == rank]
    pls = [S.CesPlanner(scene, sample_count=samples, check_points=cp, init_points=3,
                        limits_min=MG_LO, limits_max=MG_HI, seed=S.DEFAULT_SEED + g) for g in mine]
    streams = [torch.cuda.Stream(device) for _ in pls]
    started = [False] * len(pls)

    st_mine = np.array([MULTIGOAL[g][0] for g in mine], dtype=np.float64)
    en_mine = np.array([MULTIGOAL[g][1] for g in mine], dtype=np.float64)

    def run_steps(k):
        if args.mg_group and pls:  # every goal's iteration in the same batched launches
            S.CesPlanner.plan_group(pls, st_mine, en_mine, iterate=started[0], iterations=k, stream=streams[0])
            started[0] = True
            return
        if args.mg_chunk <= 0:  # every goal's k iterations in one call per goal
            for i, (g, pl) in enumerate(zip(mine, pls)):
                st, en = MULTIGOAL[g]
                pl.plan(st, en, iterate=started[i], iterations=k, stream=streams[i])
                started[i] = True
            return
        # the goals take turns, mg_chunk iterations each: every hardware queue then holds work of
        # several goals, so one goal's small CES kernels overlap another goal's evaluation
        done = 0
        while done < k:
            c = min(args.mg_chunk, k - done)
            for i, (g, pl) in enumerate(zip(mine, pls)):
                st, en = MULTIGOAL[g]
                pl.plan(st, en, iterate=started[i], iterations=c, stream=streams[i])
                started[i] = True
            done += c

    def kernel_only(first_id):
        if args.mg_group:  # one group iteration: k_ces_begin_group, k_tsp_group, the update
            S.CesPlanner.plan_group(pls, st_mine, en_mine, iterate=True, iterations=1,
                                    stream=torch.cuda.current_stream())
        else:
            pls[0].eval(rank=0, stream=torch.cuda.current_stream())

    bytes_per = 3 * 4 * 8 + 8 + 1
    flops_per = (2 * cp + 1) * 2 * 3 * 4 + cp * (3 * 4 + 1) + cp * (40 + 7 * 42 + 48 + 8 * 450)
    meta = dict(workload="robocrane TaskSpacePlanner multi-goal (gripper, 7 geoms), %d goals, "
                         "full CES iterations (eval + elites + distribution update)" % len(MULTIGOAL),
                goals=len(MULTIGOAL), goals_this_rank=len(mine), samples_per_goal=samples,
                candidates_per_goal=samples + 2, waypoints=cp, vias=1, degree=2, dof=4)
    meta["launch_form"] = "k_tsp_group (all goals per iteration)" if args.mg_group else "k_tsp per goal"
    ctx = dict(kind="multigoal", kernel_name="k_tsp_group" if args.mg_group else "k_tsp", run_steps=run_steps,
               planners=pls, mine=mine,
               scene_path=model.path, body=body, cp=cp, samples=samples)
    # candidates per step over ALL ranks: every goal's list (mean set + best + samples)
    return (samples + 2) * len(MULTIGOAL) // max(1, world), None, kernel_only, bytes_per, \
        flops_per, meta, ctx


def cpu_baseline(args, ctx, B, device):
    """Oracle (CPU restatement, oracle/) timed on a bounded sample of the same workload."""
    import torch
    from oracle import mjcf_ref
    from oracle import oracle as O
    import sspp_amd as S
    threads = cpu_threads(args)
    model = mjcf_ref.load(ctx["scene_path"])
    if ctx["kind"] == "multigoal":
        return cpu_baseline_multigoal(args, ctx, model, threads)
    timed = None
    if ctx["kind"] == "sspp":
        job = ctx["job"]
        osc = O.Scene(model, 0, 7)

        def run_on(c):
            return O.sspp_score(osc, ctx["knots"], ctx["p"], c, ctx["W"], nthreads=threads)

        def sample(first, n):
            return O.sample_sspp(ctx["ctrl0"], ctx["p"], 0.08, np.ones(7), S.DEFAULT_SEED, first, n,
                                 sampler=O.SAMPLER_FP32 if args.sampler == "fp32" else O.SAMPLER_FP64)
        # parity on the timed kernel instance itself: one launch of the timed loop's shape (same
        # executor, steps per launch, split survivor queue), its first and last steps against
        # the oracle on the same Philox candidates (the sampler is bit-exact with the oracle's)
        first_t = 1 << 42
        timed = ctx["timed_instance"](first_t)
        if timed is not None:
            par = dict(instance=dict(steps_per_launch=timed["spl"], split=timed["split"], shape=timed["shape"],
                                     steps_checked=timed["steps"]),
                       candidates=0, max_abs_cost_diff=0.0, feasible_identical=True, argmin_identical=True,
                       record_identical=True)
            for i in timed["steps"]:
                f0 = first_t + i * B
                arc_c, feas_c = run_on(sample(f0, B))
                arc_g, feas_g = timed["arc"][i], timed["feas"][i]
                fin = np.isfinite(arc_c) & np.isfinite(arc_g)
                k = O.argmin(arc_c, feas_c)[0]
                rec = S.decode_best(timed["records"][i])
                par["candidates"] += B
                if fin.any():
                    par["max_abs_cost_diff"] = max(par["max_abs_cost_diff"], float(np.abs(arc_c[fin] - arc_g[fin]).max()))
                par["feasible_identical"] &= bool(np.array_equal(feas_c, feas_g))
                par["argmin_identical"] &= bool(k == O.argmin(arc_g, feas_g)[0])
                par["record_identical"] &= bool(rec[1] == (f0 + k if k >= 0 else -1) and rec[2] == int(feas_c.sum()))
        else:
            out = job.alloc(B, device=device, with_ctrl=True)
            job.sample_score(0, B, out["arc"], out["feasible"], out["best"], ctrl_out=out["ctrl"])
            torch.cuda.synchronize()
            ctrl = out["ctrl"].cpu().numpy()
            arc_g, feas_g = out["arc"].cpu().numpy(), out["feasible"].cpu().numpy()
    else:
        job = ctx["job"]
        osc = O.Scene(model, 1, ctx["body"])
        out = job.alloc(B, device=device, with_vias=True)
        job.sample_score(0, B, out["L"], out["Cnf"], out["Cwf"], out["status"], out["cost"],
                         out["best"], vias_out=out["vias"])
        torch.cuda.synchronize()
        ctrl = out["vias"].cpu().numpy()
        arc_g, feas_g = out["cost"].cpu().numpy(), out["status"].cpu().numpy()

        def run_on(v):
            L, Cnf, Cwf, st, cost = O.tsp_score(osc, ctx["start"], ctx["end"], v, ctx["cp"],
                                                nthreads=threads)
            return cost, st

        def sample(first, n):
            return O.sample_tsp(ctx["mean"], ctx["sigma"], ctx["lo"], ctx["hi"], 0.0,
                                S.DEFAULT_SEED, first, n)
    if timed is not None:
        parity = par
    else:
        # parity on the GPU's own step-0 batch (identical control points / via sets)
        arc_c, feas_c = run_on(ctrl)
        fin = np.isfinite(arc_c) & np.isfinite(arc_g)
        parity = dict(candidates=int(B),
                      max_abs_cost_diff=float(np.abs(arc_c[fin] - arc_g[fin]).max()) if fin.any() else 0.0,
                      feasible_identical=bool(np.array_equal(feas_c, feas_g)),
                      argmin_identical=bool(O.argmin(arc_c, feas_c)[0] == O.argmin(arc_g, feas_g)[0]))
    # timed: successive batches (sampling included, as in the GPU step) for ~cpu_seconds; the
    # sampler (single-threaded oracle call) and the scorer (OpenMP over candidates) are timed
    # separately as well, so their rates can be told apart
    done, batch, t_smp, t_scr, t0 = 0, 0, 0.0, 0.0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        ta = time.perf_counter()
        c = sample((batch + 1) * B, B)
        tb = time.perf_counter()
        run_on(c)
        t_smp += tb - ta
        t_scr += time.perf_counter() - tb
        done += B
        batch += 1
    dt = time.perf_counter() - t0
    return dict(value=done / dt, unit="candidate paths scored/s", cores=threads, kind="port",
                sample="%d candidates (%d batches of %d, sampling included) in %.1f s; "
                       "OpenMP schedule(dynamic,1) over candidates" % (done, batch, B, dt),
                scoring_only_value=done / t_scr, sampling_only_value=done / t_smp,
                sampling_threads=1, **cpu_info(), parity=parity)


def cpu_threads(args):
    """Threads of the CPU baseline: --cpu-threads, else OMP_NUM_THREADS (the GPU box sets it to
    its CPU share), else every CPU this process may run on."""
    if args.cpu_threads:
        return args.cpu_threads
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env:
        return env
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return dict(cpu_model=model, host_cpus=os.cpu_count(), affinity_cpus=aff,
                omp_num_threads=os.environ.get("OMP_NUM_THREADS"))


def cpu_baseline_multigoal(args, ctx, model, threads):
    """The oracle's full TaskSpacePlanner iteration (oracle.ces_plan) on goal 0, bounded."""
    from oracle import oracle as O
    osc = O.Scene(model, 1, ctx["body"])
    st, en = (np.array(x) for x in MULTIGOAL[0])
    # parity on the device planner's first iteration of goal 0 (same Philox ids)
    import sspp_amd as S
    import torch
    pl = S.CesPlanner(ctx["planners"][0].scene, sample_count=ctx["samples"], check_points=ctx["cp"],
                      init_points=3, limits_min=MG_LO, limits_max=MG_HI, seed=S.DEFAULT_SEED)
    pl.plan(st, en, iterate=False, iterations=1)
    torch.cuda.synchronize()
    r = pl.read()
    rec = O.ces_plan(osc, st, en, 1, ctx["samples"], ctx["cp"], seed=S.DEFAULT_SEED, lo=MG_LO,
                     hi=MG_HI, nthreads=threads)[0]
    parity = dict(candidates=int(r["n_candidates"]),
                  max_abs_cost_diff=float(np.abs(np.where(np.isfinite(r["cost"]), r["cost"], 0) -
                                                 np.where(np.isfinite(rec["cost"]), rec["cost"], 0)).max()),
                  status_identical=bool(np.array_equal(r["status"], rec["status"])),
                  best_slot_identical=bool(r["best_slot"] == rec["best_slot"]),
                  mean_max_abs_diff=float(np.abs(r["mean"] - rec["mean"]).max()))
    done, it, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        O.ces_plan(osc, st, en, 1, ctx["samples"], ctx["cp"], seed=S.DEFAULT_SEED + it, lo=MG_LO,
                   hi=MG_HI, nthreads=threads)
        done += ctx["samples"] + 1
        it += 1
    dt = time.perf_counter() - t0
    return dict(value=done / dt, unit="candidate paths scored/s (full CES iterations)", cores=threads,
                kind="port", sample="%d CES iterations of goal 0 (%d candidates) in %.1f s" % (it, done, dt),
                **cpu_info(), parity=parity)


def native_runner(args, ctx, B, world, rank, device, on_chunk=None):
    """The timed loop's step protocol (robocrane).  The C++ step executor enqueues G steps per
    call, round robin over --streams streams (one job each): step t scores global ids
    (t * world + rank) * B + [0, B), so the candidate set does not depend on the rank count.
    With several ranks each chunk's G per-step argmin records (32 B each) go through ONE
    all-gather on the main stream and are reduced per step on the device (lowest cost, lowest
    id).  on_chunk(records) receives each chunk's per-step global records (tests)."""
    import torch
    import sspp_amd as S
    ns = args.streams
    G = max(1, args.chunk)
    main = torch.cuda.current_stream()
    streams = [main] + [torch.cuda.Stream(device) for _ in range(ns - 1)]
    ex = ctx["make_executor"](streams, args.steps_per_launch)
    best = torch.zeros((G, 4), dtype=torch.int64, device=device)
    gbufs = {}
    counter = [0]

    def gbuf(g):
        if g not in gbufs:
            gbufs[g] = (torch.zeros((world, g, 4), dtype=torch.int64, device=device),
                        torch.zeros((g, 4), dtype=torch.int64, device=device))
        return gbufs[g]

    # prime every branch before warmup: one launch per stream, so no stream sees its first
    # work inside the timed region (ids past any timed step's; results discarded)
    ex.enqueue(ns * args.steps_per_launch, 1 << 40, world * B, None)
    torch.cuda.synchronize()

    # per chunk size: the records view and its device address, made before any timed region
    # (no per-call slicing or allocation inside it)
    views = {g: (best[:g], best[:g].data_ptr()) for g in range(1, G + 1)}
    if world > 1:
        for g in range(1, G + 1):
            gbuf(g)

    def run_steps(k):
        while k > 0:
            g = min(G, k)
            rec, rec_ptr = views[g]
            # the records buffer is reused per chunk: when they are consumed (gathered, or
            # handed to on_chunk) every branch joins the main stream, and the next chunk's
            # branches start after the consumer
            sync_rec = world > 1 or on_chunk is not None
            if sync_rec:
                for st in streams[1:]:
                    st.wait_stream(main)
            ex.enqueue(g, (counter[0] * world + rank) * B, world * B, rec_ptr)
            if sync_rec:
                for st in streams[1:]:
                    main.wait_stream(st)
            if world > 1:
                gat, gout = gbuf(g)
                S.all_gather_records(gat, rec)
                S.reduce_best_steps(gat, gout)
                rec = gout
            if on_chunk is not None:
                on_chunk(rec)
            counter[0] += g
            k -= g
    return run_steps


def run_dropin(args):
    """Latency of the drop-in entry point, SamplingPathPlanner7.plan(start, end, sigma, limits,
    sample_count, check_points, init_points) on the robocrane workload (BASELINE configs[1]):
    host call -> initializePath -> device sampling + scoring + argmin -> compaction of the
    feasible candidates into pinned memory -> Python list of Spline7.  Inputs are host arrays,
    as the reference's callers pass them."""
    import torch
    from sspp import _sspp
    import sspp_amd as S
    planner = _sspp.SamplingPathPlanner7(os.path.join(S.SCENE_DIR, "robocrane.xml"))
    start = np.array([0.5, 0.15, 0.136, 0.707, 0.0, 0.0, 0.707])
    end = np.array([0.5, -0.05, 0.136, 0.707, 0.0, 0.0, 0.707])
    B, W, n = args.batch or 4096, args.waypoints, 10
    limits = np.ones(7)
    # plan() prints one line per call (include/sspp.h:221): keep it off the JSON line's stdout
    sys.stdout.flush()
    saved = os.dup(1)
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)
    try:
        for _ in range(args.warmup):
            planner.plan(start, end, 0.08, limits, B, W, n)
        lat, nfeas = [], []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ta = time.perf_counter()
            ok, paths = planner.plan(start, end, 0.08, limits, B, W, n)
            lat.append(time.perf_counter() - ta)
            nfeas.append(len(paths))
        total = time.perf_counter() - t0
        # the cold side: a fresh planner's first plan() (its job is created in that call: tables,
        # device buffers, pinned outputs; the hit-order pre-pass runs asynchronously beside it)
        # and its next calls, in this already-initialised process
        cold, cold_parts = [], []
        for _ in range(3):
            fresh = _sspp.SamplingPathPlanner7(os.path.join(S.SCENE_DIR, "robocrane.xml"))
            ts = []
            for _ in range(4):
                ta = time.perf_counter()
                fresh.plan(start, end, 0.08, limits, B, W, n)
                ts.append((time.perf_counter() - ta) * 1e6)
            cold.append(ts)
            cold_parts.append({k: round(v, 1) for k, v in fresh._timings().items()})
            del fresh
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
        os.close(devnull)
    # one executor step of the same shape for comparison: a single 4096-candidate launch on an
    # idle stream (isolated: no overlap with other steps), HIP events
    model = S.Model(os.path.join(S.SCENE_DIR, "robocrane.xml"))
    u = np.array([i / (n - 1) for i in range(n)])
    knots, ctrl0 = S.interpolate(np.array([(1 - t) * start + t * end for t in u]), 3, u)
    job = S.SsppJob(S.Scene(model, 0, 7), knots, 3, ctrl0, 0.08, limits, W, max_batch=B)
    out = job.alloc(B, device="cuda")
    for i in range(20):
        job.sample_score(i * B, B, out["arc"], out["feasible"], out["best"])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ks = []
    for i in range(50):
        e0.record()
        job.sample_score((100 + i) * B, B, out["arc"], out["feasible"], out["best"])
        e1.record()
        torch.cuda.synchronize()
        ks.append(e0.elapsed_time(e1) * 1e3)
    lat_us = np.array(lat) * 1e6
    line = {
        "metric": "drop-in SamplingPathPlanner7.plan per-call latency (robocrane, 4096 x 128)",
        "value": float(np.median(lat_us)), "unit": "us/plan (median)", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "higher_is_better": False,
        "candidates_per_s": B * args.steps / total,
        "latency_us": {"median": float(np.median(lat_us)), "p10": float(np.percentile(lat_us, 10)),
                       "p90": float(np.percentile(lat_us, 90)), "mean": float(lat_us.mean())},
        "feasible_per_plan": float(np.mean(nfeas)),
        # a fresh SamplingPathPlanner7: first plan() (scene tables, planner stream, job creation
        # included), then calls 2-4; median and max over the fresh objects, with the first call's
        # parts (cold_call_parts_us) — the first fresh object in a process also creates a new HIP
        # hardware queue for its stream (drop-in)
        "first_call_us": float(np.median([c[0] for c in cold])),
        "first_call_us_max": float(np.max([c[0] for c in cold])),
        "cold_calls_us": [[round(x, 1) for x in c] for c in cold],
        "cold_call_parts_us": cold_parts,
        "isolated_step_kernel_us": float(np.median(ks)),
        "dtype": "f64", "data": "synthetic (on-device Philox candidates around a linear init spline)",
        "config": {"workload": "robocrane SamplingPathPlanner7.plan(start, end, 0.08, ones(7), %d, %d, %d)"
                               % (B, W, n), "call": "_sspp (pybind11) -> sspp_planner_plan (C ABI)",
                   "sampler": "fp64"},
    }
    print(json.dumps(line))


# src/main_icra_benchmark.cpp:151-179: the planner configuration and the start / end points of
# the reference's ICRA anytime benchmark (robocrane model, 1 via, gripper as the moving body)
ICRA = dict(stddev_initial=0.2, stddev_min=1e-4, stddev_max=0.5, stddev_increase_factor=1.5,
            stddev_decay_factor=0.9, elite_fraction=0.3, sample_count=15, check_points=40,
            gd_iterations=0, init_points=3, collision_weight=1.0, z_min=0.1,
            limits_min=(0.0, -0.7, 0.1, -1.6), limits_max=(0.7, 0.7, 0.6, 1.6),
            enable_gradient_descent=False, sigma_floor=0.005, var_ema_beta=0.2, mean_lr=0.5,
            max_step_norm=0.1, floor_margin=0.01, floor_penalty_scale=10.0)
ICRA_BODY = "gripper_collision_with_block/"


def path_len_xyz(planner, n=50):
    pts = np.array(planner.get_path_pts(n))[:, :3]
    return float(np.linalg.norm(np.diff(pts, axis=0), axis=1).sum())


def run_tsp_anytime(args):
    """The reference's anytime benchmark (src/main_icra_benchmark.cpp:67-119, 199-221) on the
    drop-in `_tsp.TaskSpacePlanner`: per budget, `steps` cold trials (a fresh planner each,
    construction untimed) and `steps` warm trials (one planner), each trial = plan(q0, qT, False)
    then plan(q0, qT, True) until the wall-clock budget is spent.  Reports the latency of one
    plan(..., True) call (host call -> CES iteration on the device -> results back as Python
    objects) and the iterations each budget holds; the oracle's CES iteration (oracle.ces_plan,
    same sizes) is timed beside it as the CPU baseline."""
    from sspp import _tsp
    import sspp_amd as S
    xml = os.path.join(S.SCENE_DIR, "robocrane.xml")
    model = S.Model(xml)
    q0 = model.body_point("block_green/") + np.array([0, 0, 0.02, 0])
    qT = model.body_point("block_orange/") + np.array([0, 0, 0.02, 0])
    budgets = [int(b) for b in args.budgets_ms.split(",") if b]
    N = args.steps

    def make():
        return _tsp.TaskSpacePlanner(xml, ICRA_BODY, **ICRA)

    iter_lat = []

    def anytime(pl, budget_ms):
        t0 = time.perf_counter()
        deadline = t0 + budget_ms / 1e3
        ok = len(pl.plan(q0, qT, False)) > 0
        iters = 1
        best = path_len_xyz(pl) if ok else float("inf")
        while time.perf_counter() < deadline:
            ta = time.perf_counter()
            now_ok = len(pl.plan(q0, qT, True)) > 0
            iter_lat.append(time.perf_counter() - ta)
            iters += 1
            if now_ok:
                ok = True
                best = min(best, path_len_xyz(pl))
        return (time.perf_counter() - t0) * 1e3, ok, best if ok else 0.0, iters

    for _ in range(max(1, args.warmup)):
        anytime(make(), 5)
    iter_lat.clear()
    res = {}
    for B in budgets:
        row = {}
        for mode in ("cold", "warm"):
            runs = []
            pl = make()
            for _ in range(N):
                if mode == "cold":
                    pl = make()
                runs.append(anytime(pl, B))
            ms = np.array([r[0] for r in runs])
            succ = [r for r in runs if r[1]]
            row[mode] = {"succ": len(succ), "trials": N, "mean_ms": float(ms.mean()),
                         "std_ms": float(ms.std()), "min_ms": float(ms.min()), "max_ms": float(ms.max()),
                         "avg_iters": float(np.mean([r[3] for r in runs])),
                         "avg_len_m": float(np.mean([r[2] for r in succ])) if succ else None}
        res[str(B)] = row
    lat_us = np.array(iter_lat) * 1e6
    # plan(..., True) alone, back to back (no path-length bookkeeping between the calls)
    pl = make()
    pl.plan(q0, qT, False)
    t0 = time.perf_counter()
    for _ in range(200):
        pl.plan(q0, qT, True)
    tight_us = (time.perf_counter() - t0) / 200 * 1e6
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline_anytime(args, model, q0, qT)
    line = {
        "metric": "TaskSpacePlanner.plan(q0, qT, True) latency, ICRA anytime benchmark size",
        "value": float(np.median(lat_us)), "unit": "us/iteration (median, inside the anytime loop)",
        "n_gpus": 1, "steps": N, "warmup": args.warmup, "higher_is_better": False,
        "latency_us": {"median": float(np.median(lat_us)), "p10": float(np.percentile(lat_us, 10)),
                       "p90": float(np.percentile(lat_us, 90)), "back_to_back": tight_us},
        "iterations_per_budget": {b: {m: r[m]["avg_iters"] for m in r} for b, r in res.items()},
        "budgets": res, "dtype": "f64", "data": "robocrane.xml, block_green/ -> block_orange/ (+2 cm z)",
        "config": {"workload": "ICRA anytime (src/main_icra_benchmark.cpp:151-179): 15 samples x 40 "
                               "checks, 1 via, body %s" % ICRA_BODY,
                   "call": "_tsp (pybind11) -> sspp_ces_plan + sspp_ces_read (C ABI)"},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line))


def cpu_baseline_anytime(args, model, q0, qT):
    """oracle.ces_plan (test infrastructure) at the ICRA size: seconds per CES iteration on the
    host, single-threaded (the reference's scorer is OpenMP over 17 candidates)."""
    from oracle import mjcf_ref
    from oracle import oracle as O
    osc = O.Scene(mjcf_ref.load(model.path), 1, model.body_id(ICRA_BODY))
    cfg = dict(frac=ICRA["elite_fraction"], inc=ICRA["stddev_increase_factor"],
               dec=ICRA["stddev_decay_factor"], sigma_floor=ICRA["sigma_floor"],
               var_beta=ICRA["var_ema_beta"], mean_lr=ICRA["mean_lr"], sd_min=ICRA["stddev_min"],
               sd_max=ICRA["stddev_max"], dist_z_min=ICRA["stddev_initial"],
               lo=ICRA["limits_min"], hi=ICRA["limits_max"])
    its = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < min(args.cpu_seconds, 5.0):
        O.ces_plan(osc, q0, qT, 20, ICRA["sample_count"], ICRA["check_points"], z_min=ICRA["z_min"],
                   nthreads=1, **cfg)
        its += 20
    dt = time.perf_counter() - t0
    return dict(value=dt / its * 1e6, unit="us/iteration", cores=1, kind="port",
                sample="%d CES iterations (20-iteration oracle.ces_plan runs) in %.1f s" % (its, dt),
                iterations_per_budget={str(b): b * 1e3 / (dt / its * 1e6)
                                       for b in [int(x) for x in args.budgets_ms.split(",") if x]},
                **cpu_info())


def rank_launch_cmd(argv, n, port):
    """The child command of `bench.py --gpus N` run without a launcher: this script under
    torch.distributed.run with N ranks on one node (same arguments)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv):
    """--gpus N > 1 without WORLD_SIZE: start the N ranks as a child process (subprocess, no
    exec, nothing has touched the GPU yet) and return its exit status."""
    import socket
    import subprocess
    import torch
    visible = torch.cuda.device_count()  # counts devices without initialising them
    if visible < args.gpus:
        print("bench.py: --gpus %d needs %d visible GPUs, found %d" % (args.gpus, args.gpus, visible),
              file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    sys.stdout.flush()
    return subprocess.call(rank_launch_cmd(argv, args.gpus, port))


def bench_line(args, ctx, meta, world, ns, native, B, elapsed, enqueue_s, kernel_s, bytes_per, flops_per,
               per_launch, traffic, traffic_src, exec_per, exec_src, cpu, extras):
    """The JSON line (rank 0).  `roofline` is the metric's HBM figure for the dominant kernel
    (algorithmic bytes per launch / HIP-event launch time; `traffic` and `traffic_frac` are the
    PMC-measured HBM bytes per launch and their rate against the peak); `binding_roofline` is
    the resource that actually bounds it, FP64 VALU (PMC-executed flops per candidate)."""
    total = args.steps * B * world
    if ctx["kind"] == "multigoal":
        # every goal's mean set + samples, whatever the rank count; the forwarded best
        # (and, before the first success, the padding slot in its place) is not counted
        total = args.steps * (ctx["samples"] + 1) * len(MULTIGOAL)
    value = total / elapsed
    ach_exec = None if exec_per is None else exec_per * per_launch / kernel_s / 1e12
    ach_gbs = bytes_per * per_launch / kernel_s / 1e9
    config = dict(meta, streams=ns, launch=("CES iteration chains (sspp_ces_plan), one stream per goal"
                                            if "run_steps" in ctx else
                                            "native executor, %d steps/call, %d steps/launch"
                                            % (args.chunk, args.steps_per_launch)
                                            if native else "eager"),
                  parallelism="dp%d (candidate shards, RCCL all-gather argmin)" % world)
    if "order1_elapsed_s" in extras:
        # throughput at the hit order (the default) over throughput at order 1, same run
        config["order_gain"] = extras["order1_elapsed_s"] / elapsed
    line = {
        "metric": {"robocrane": "candidate paths scored/sec (7-DoF, 128 waypts) at 1/2/4/8 MI355X; HBM %peak",
                   "stacking": "candidate paths scored/sec (stacking.xml TSP)",
                   "multigoal": "candidate paths scored/sec (TSP multi-goal, full CES iterations)"}[args.config],
        "value": value,
        "unit": "candidate paths/s",
        "n_gpus": world,
        "ranks_joined": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "host_enqueue_ms": enqueue_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if ctx["kind"] == "multigoal" else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (on-device Philox candidates around a linear init spline)",
        "config": config,
        "roofline": {"bound": "hbm", "achieved": ach_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                     # the measured bytes' rate against the peak (the candidates are generated
                     # in-kernel, so far below the algorithmic figure above)
                     "traffic_frac": None if traffic is None else traffic / kernel_s / (HBM_PEAK_GBS * 1e9),
                     "algorithmic_bytes_per_launch": bytes_per * per_launch,
                     "kernel": ctx.get("kernel_name", "k_tsp"),
                     "kernel_us": kernel_s * 1e6, "candidates_per_launch": per_launch,
                     "bytes_per_candidate": bytes_per,
                     # the same bytes at the timed loop's rate (launches overlap on streams)
                     "steady_state_GBps": bytes_per * value / 1e9 / max(1, world)},
        # what bounds the kernel: FP64 VALU with the flops it EXECUTES (PMC: 64 lanes x F64 wave
        # instructions, FMA = 2; profiles/fp64_latest.json) over the same launches as
        # `roofline`.  SURVEY 8(d)'s fixed charge table (every pair at every waypoint, no credit
        # for early exit / culling) is kept for reference only: it overstates the work ~70x for
        # the early-exit feasibility path.
        "binding_roofline": {"bound": "fp64_valu", "achieved": ach_exec, "peak": FP64_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": None if ach_exec is None else ach_exec / FP64_PEAK_TFLOPS,
                             "flops_per_candidate_executed": exec_per, "source": exec_src,
                             "flops_per_candidate_charged": flops_per,
                             # the same executed flops at the timed loop's rate (launches overlap)
                             "steady_state_TFLOPs": None if exec_per is None else
                             exec_per * value / 1e12 / max(1, world)},
        "cpu_baseline": cpu,
    }
    vi = extras.get("valu_issue")
    if vi:
        # the FP32-filtered scan moved most of the arithmetic off FP64: the binding resource is
        # VALU issue (PMC: ~4 cycles per wave instruction per SIMD over the dispatch's cycles) at
        # the measured occupancy; the FP64 figure stays beside it
        fp64 = line["binding_roofline"]
        line["binding_roofline"] = {"bound": "valu_issue", "achieved": vi["per_simd"], "peak": 1.0,
                                    "unit": "VALU issue-slot fraction per SIMD (PMC)", "frac": vi["per_simd"],
                                    "mean_occupancy_waves_per_cu": vi.get("occupancy"), "source": vi.get("source"),
                                    "fp64_valu": fp64}
    if "isolated_step_us" in extras:
        # one B-candidate batch (a single plan()'s worth) alone on the device
        line["isolated_step_us"] = extras["isolated_step_us"]
        line["single_plan_cand_per_s"] = B / (extras["isolated_step_us"] * 1e-6)
    return line


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if world_env is None and args.gpus > 1:
        if args.mode in ("dropin", "tsp-anytime"):
            print("bench.py: --mode %s is a single-GPU latency benchmark" % args.mode, file=sys.stderr)
            return 2
        return launch_ranks(args, argv)
    if world_env is not None and int(world_env) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (world_env, args.gpus), file=sys.stderr)
        return 2
    if args.mode == "dropin":
        run_dropin(args)
        return 0
    if args.mode == "tsp-anytime":
        run_tsp_anytime(args)
        return 0
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        world = dist.get_world_size()  # the ranks that joined
    device = torch.device("cuda", local)
    import sspp_amd as S

    if args.config == "multigoal":
        B, step, kernel_only, bytes_per, flops_per, meta, ctx = setup_multigoal(args, device, world, rank)
    else:
        setup = setup_robocrane if args.config == "robocrane" else setup_stacking
        B, step, kernel_only, bytes_per, flops_per, meta, ctx = setup(args, device)

    ns = args.streams
    native = args.mode == "native" and "make_executor" in ctx
    if "run_steps" in ctx:
        run_steps = ctx["run_steps"]
    elif native:
        run_steps = native_runner(args, ctx, B, world, rank, device)
    else:
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device) for _ in range(ns - 1)]
        gathered = [torch.zeros((world, 4), dtype=torch.int64, device=device) for _ in range(ns)]
        gbest = [S.best_tensor(device) for _ in range(ns)]
        local_best = [S.best_tensor(device) for _ in range(ns)]
        counter = [0]

        def full_step(i):
            # step i runs on stream i % ns: consecutive batches overlap, so one batch's argmin
            # tail and launch gap hide under the next batch's scoring (the steps are independent)
            lane = i % ns
            first = (i * world + rank) * B  # globally unique candidate ids
            with torch.cuda.stream(streams[lane]):
                step(first, local_best[lane], lane, streams[lane])
                if world > 1:
                    S.all_gather_records(gathered[lane], local_best[lane])
                    S.reduce_best_device(gathered[lane], gbest[lane], stream=streams[lane])

        def run_steps(k):
            for _ in range(k):
                full_step(counter[0])
                counter[0] += 1

    run_steps(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    t_enq = time.perf_counter()  # host enqueue done (diagnostic: enqueue vs wait in the region)
    torch.cuda.synchronize()
    if world > 1:  # a single rank has no barrier to bracket, so nothing left to synchronise
        dist.barrier()
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # roofline of the dominant kernel: HIP events on the stream the kernel runs on
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(args.roofline_launches):
        kernel_only(i * B)
    e1.record(stream)
    torch.cuda.synchronize()
    kernel_s = e0.elapsed_time(e1) / 1e3 / args.roofline_launches

    # the effective configuration of the timed launches, read before the CPU baseline's parity
    # batch (one launch of B candidates, which runs at the latency shape)
    if "effective" in ctx:
        meta.update(ctx["effective"]())
    if "validate" in ctx:  # the timed launches lost no work (raises otherwise)
        meta.update(ctx["validate"]())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, ctx, B, device)

    per_launch = ((ctx["samples"] + 2) * (len(ctx["mine"]) if args.mg_group else 1) if ctx["kind"] == "multigoal"
                  else ctx.get("per_launch", B))
    # PMC records (tools/update_latest.py) are keyed by config, or config_b<B>_w<W> off the
    # default shape, and used only for launches of the recorded kernel and size
    pmc_key = args.config if (args.waypoints == 128 and not args.batch) else \
        "%s_b%d_w%d" % (args.config, B, args.waypoints)
    if args.config == "robocrane" and args.mode == "native" and roofline_spl(args) != 40:
        pmc_key += "_spl%d" % roofline_spl(args)  # records of another launch shape
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if os.path.exists(tf):
        rec = json.load(open(tf)).get(pmc_key)
        if rec and rec.get("kernel") == ctx.get("kernel_name", "k_tsp") and rec.get("rev") == KERNEL_REV and \
                rec.get("candidates_per_launch") == per_launch:
            traffic, traffic_src = rec["hbm_bytes_per_launch"], rec["source"]

    lib_path = os.environ.get("SSPP_LIB_PATH")
    if lib_path:  # a variant build (profiling only): say so on the line
        meta["library"] = lib_path
    extras = {}
    if rank == 0 and world == 1 and "isolated_step_us" in ctx:
        # one plan()-sized batch alone on an idle stream (HIP events per launch): the latency
        # side of the same kernel, beside the fused multi-step throughput above
        extras["isolated_step_us"] = ctx["isolated_step_us"]()
    if world == 1 and "set_order" in ctx and args.mode == "native":
        # what the hit-order pre-pass buys: the same timed run at scan order 1 (mean-path gap
        # pairs, bisection waypoints; bit-identical results), after the main region
        ctx["set_order"](1)
        run_steps(args.warmup)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        run_steps(args.steps)
        torch.cuda.synchronize()
        extras["order1_elapsed_s"] = time.perf_counter() - t1
    if rank == 0:
        exec_per, exec_src = None, None
        ff = os.path.join(ROOT, "profiles", "fp64_latest.json")
        if os.path.exists(ff):
            rec = json.load(open(ff)).get(pmc_key)
            if rec and rec.get("kernel") == ctx.get("kernel_name", "k_tsp") and rec.get("rev") == KERNEL_REV and \
                    rec.get("candidates_per_launch", per_launch) == per_launch:
                exec_per, exec_src = rec["fp64_flops_per_candidate"], rec["source"]
                if rec.get("valu_issue_per_simd") is not None:
                    extras["valu_issue"] = {"per_simd": rec["valu_issue_per_simd"],
                                            "occupancy": rec.get("mean_occupancy_per_cu"), "source": rec["source"]}
        line = bench_line(args, ctx, meta, world, ns, native, B, elapsed, t_enq - t0, kernel_s, bytes_per,
                          flops_per, per_launch, traffic, traffic_src, exec_per, exec_src, cpu, extras)
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
