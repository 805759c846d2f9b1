"""Summarise rocprofv3 output into profiles/: kernel stats + per-launch HBM traffic.

    python tools/pmc_summary.py <gpurun_out/TAG> <profiles/PREFIX> [roofline_launches]

Writes
  PREFIX_kernel_stats.csv  copy of the `--kernel-trace --stats` summary of the bench command;
  PREFIX_pmc.json          per kernel: mean FETCH_SIZE / WRITE_SIZE per launch (rocprofv3 reports
                           KiB) from separate --pmc passes, and the HBM bytes per launch corrected
                           as MI355X_MICROARCH.md prescribes (gfx950 FETCH_SIZE counts half the
                           bytes of wide coalesced reads -> x2; WRITE_SIZE exact); plus, from the
                           kernel trace, the average duration over all launches and over the last
                           `roofline_launches` launches of the dominant kernel (bench.py's roofline
                           region: sequential launches on one stream, timed there with HIP events).
"""
import csv
import json
import os
import shutil
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].strip()


def main(src, dst, roofline_launches=200):
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    st = os.path.join(src, "prof", "run_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, dst + "_kernel_stats.csv")
    out = {}
    for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != ctr:
                continue
            k = short(r["Kernel_Name"])
            d = out.setdefault(k, {"grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                                   "sgpr": int(r["SGPR_Count"]), "scratch_per_lane": int(r["Scratch_Size"]),
                                   "lds": int(r["LDS_Block_Size"])})
            d.setdefault(ctr, []).append(float(r["Counter_Value"]))
    for k, d in out.items():
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            if ctr in d:
                v = d.pop(ctr)
                d[ctr + "_KiB_mean"] = sum(v) / len(v)
                d[ctr + "_launches"] = len(v)
        if "FETCH_SIZE_KiB_mean" in d and "WRITE_SIZE_KiB_mean" in d:
            d["hbm_bytes_per_launch"] = 1024.0 * (2.0 * d["FETCH_SIZE_KiB_mean"] + d["WRITE_SIZE_KiB_mean"])
    tr = os.path.join(src, "prof", "run_kernel_trace.csv")
    if os.path.exists(tr):
        durs = {}
        for r in csv.DictReader(open(tr)):
            durs.setdefault(short(r["Kernel_Name"]), []).append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for k, v in durs.items():
            v.sort()
            d = out.setdefault(k, {})
            d["trace_launches"] = len(v)
            d["trace_avg_us"] = sum(x[1] for x in v) / len(v) / 1e3
            if len(v) > roofline_launches:
                tail = v[-roofline_launches:]
                d["trace_avg_us_last_%d" % roofline_launches] = sum(x[1] for x in tail) / len(tail) / 1e3
    json.dump(out, open(dst + "_pmc.json", "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:4]))
