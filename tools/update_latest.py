"""Fold a PMC evidence run (tools/runs/gpu_pmc.sh) into profiles/traffic_latest.json and
profiles/fp64_latest.json, which bench.py reads for roofline.traffic / roofline_fp64.
    python tools/update_latest.py gpurun_out/TAG profiles/PREFIX
Per config: the dominant kernel's launches of the roofline shape (GRID, else the most frequent grid),
mean FETCH_SIZE / WRITE_SIZE per launch (KiB; HBM bytes = 1024 * (2 * FETCH + WRITE), the
gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md) and the executed FP64 flops (64 lanes x
(ADD + MUL + TRANS + 2 FMA) F64 wave instructions).  Also writes PREFIX_<config>_pmc.json."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import KERNEL_REV  # noqa: E402  (records of another kernel revision are not attached)

# record keys: the bench config, or config_b<batch>_w<waypoints> off the default shape
KERNEL = {"robocrane": "k_sspp_c2f", "stacking": "k_tsp", "multigoal": "k_tsp_group",
          "robocrane_b32768_w256": "k_sspp_c2f", "robocrane_spl20": "k_sspp_c2f"}
PER_LAUNCH = {"robocrane": 40 * 4096, "stacking": 16384, "multigoal": 8 * 4098,
              "robocrane_b32768_w256": 40 * 32768, "robocrane_spl20": 20 * 4096}
STEPS = {"robocrane": "--steps 80 --warmup 4 (40 steps x 4096 candidates per launch)",
         "stacking": "--config stacking --steps 4 --warmup 1",
         "multigoal": "--config multigoal --steps 4 --warmup 1",
         "robocrane_b32768_w256": "--batch 32768 --waypoints 256 --steps 80 --warmup 4 (config-4 shard)",
         "robocrane_spl20": "--steps 20 --warmup 5 (the driver's run: one launch of 20 steps x 4096)"}


def rows(path, kern):
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return []
    return [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]


# the timed launch's grid (threads) where other launches of the same kernel share the run: the
# 128 x 4 shape holds 32 candidates per 128-thread workgroup (4 threads per candidate)
GRID = {"robocrane": 4 * 40 * 4096, "robocrane_spl20": 4 * 20 * 4096}


def per_launch(rs, counters, grid=None):
    """{counter: mean per launch} over the launches of `grid`, else of the most frequent grid."""
    if grid is None or not any(int(r["Grid_Size"]) == grid for r in rs):
        grid = collections.Counter(r["Grid_Size"] for r in rs).most_common(1)[0][0]
    grid = str(grid)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rs:
        if r["Grid_Size"] == grid and r["Counter_Name"] in counters:
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {c: sum(v.values()) / len(v) for c, v in acc.items()}
    out["launches"] = max(len(v) for v in acc.values())
    out["grid"] = int(grid)
    for k in ("VGPR_Count", "SGPR_Count", "Scratch_Size", "LDS_Block_Size"):
        out[k] = int(next(r[k] for r in rs if r["Grid_Size"] == grid))
    return out


def main(src, prefix):
    tf, ff = "profiles/traffic_latest.json", "profiles/fp64_latest.json"
    traffic = json.load(open(tf)) if os.path.exists(tf) else {}
    fp64 = json.load(open(ff)) if os.path.exists(ff) else {}
    for cfg, kern in KERNEL.items():
        d = os.path.join(src, cfg)
        if not os.path.isdir(d):
            continue
        res = {"kernel": kern, "candidates_per_launch": PER_LAUNCH[cfg], "command": STEPS[cfg]}
        fr, wr = rows(os.path.join(d, "pmc_fetch"), kern), rows(os.path.join(d, "pmc_write"), kern)
        if fr and wr:
            g = GRID.get(cfg)
            f, w = per_launch(fr, {"FETCH_SIZE"}, g), per_launch(wr, {"WRITE_SIZE"}, g)
            res.update(FETCH_SIZE_KiB=f["FETCH_SIZE"], WRITE_SIZE_KiB=w["WRITE_SIZE"], launches=f["launches"],
                       grid=f["grid"], vgpr=f["VGPR_Count"], sgpr=f["SGPR_Count"],
                       scratch_per_lane=f["Scratch_Size"], lds=f["LDS_Block_Size"])
            res["hbm_bytes_per_launch"] = 1024.0 * (2.0 * f["FETCH_SIZE"] + w["WRITE_SIZE"])
            traffic[cfg] = {"kernel": kern, "rev": KERNEL_REV, "hbm_bytes_per_launch": res["hbm_bytes_per_launch"],
                            "candidates_per_launch": PER_LAUNCH[cfg],
                            "source": "%s_%s_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, "
                                      "FETCH x2 gfx950 correction; %s)" % (prefix, cfg, STEPS[cfg])}
        pr = rows(os.path.join(d, "p1"), kern)
        if pr:
            m = per_launch(pr, {r["Counter_Name"] for r in pr}, GRID.get(cfg))
            res["mix"] = m
            fl = 64.0 * (m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] +
                         m["SQ_INSTS_VALU_TRANS_F64"] + 2 * m["SQ_INSTS_VALU_FMA_F64"])
            res["fp64_flops_per_launch"] = fl
            res["fp64_flops_per_candidate"] = fl / PER_LAUNCH[cfg]
            fp64[cfg] = {"kernel": kern, "rev": KERNEL_REV, "fp64_flops_per_candidate": res["fp64_flops_per_candidate"],
                         "candidates_per_launch": PER_LAUNCH[cfg],
                         "source": "%s_%s_pmc.json: 64 x (ADD+MUL+TRANS+2 FMA)_F64 wave instructions per "
                                   "launch / %d candidates" % (prefix, cfg, PER_LAUNCH[cfg])}
        occ = rows(os.path.join(d, "occ", "p1"), kern)
        if occ:
            o = per_launch(occ, {r["Counter_Name"] for r in occ}, GRID.get(cfg))
            res["occupancy"] = o
            if o.get("GRBM_GUI_ACTIVE"):
                # GRBM_GUI_ACTIVE is summed over the 8 XCDs (each counts the dispatch's busy
                # cycles; the derived MeanOccupancyPerCU takes the max instead): per-XCD cycles
                cyc = o["GRBM_GUI_ACTIVE"] / 8.0
                res["dispatch_cycles"] = cyc
                # a VALU wave-instruction holds its SIMD's issue for ~4 cycles (wave64, FP64 at
                # 16 lanes per cycle): issue-slot utilisation per SIMD, 1024 SIMDs
                res["valu_issue_per_simd"] = 4.0 * o["SQ_INSTS_VALU"] / (cyc * 1024)
                # resident waves per CU averaged over the dispatch (SQ_WAVE_CYCLES: quad-cycles)
                res["waves_per_cu_from_wave_cycles"] = 4.0 * o["SQ_WAVE_CYCLES"] / (cyc * 256)
        occ2 = rows(os.path.join(d, "occ", "p2"), kern)
        if occ2:
            res["mean_occupancy_per_cu"] = per_launch(occ2, {r["Counter_Name"] for r in occ2}, GRID.get(cfg)).get("MeanOccupancyPerCU")
        ut = rows(os.path.join(d, "util"), kern)
        if ut:  # share of the 64 lanes active per VALU instruction (derived VALUUtilization, %)
            u = per_launch(ut, {r["Counter_Name"] for r in ut}, GRID.get(cfg))
            res["valu_utilization_pct"] = u.get("VALUUtilization")
            res["valu_thread_cycles"] = u.get("SQ_THREAD_CYCLES_VALU")
        if cfg in fp64 and fp64[cfg].get("rev") == KERNEL_REV and "valu_issue_per_simd" in res:
            fp64[cfg]["valu_issue_per_simd"] = res["valu_issue_per_simd"]
            fp64[cfg]["mean_occupancy_per_cu"] = res.get("mean_occupancy_per_cu")
        json.dump(res, open("%s_%s_pmc.json" % (prefix, cfg), "w"), indent=1, sort_keys=True)
        print(cfg, json.dumps(res, sort_keys=True)[:600])
    json.dump(traffic, open(tf, "w"), indent=1)
    json.dump(fp64, open(ff, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:3])
