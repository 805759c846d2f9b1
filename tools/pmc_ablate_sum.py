"""Per-launch mean of each counter for k_sspp_c2f launches of the largest grid, per ablation run.
    python tools/pmc_ablate_sum.py gpurun_out/TAG"""
import csv
import glob
import os
import sys

src = sys.argv[1]
for d in sorted(glob.glob(os.path.join(src, "ab*"))):
    if not os.path.isdir(d):
        continue
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        continue
    acc, gmax = {}, 0
    rows = [r for f in fs for r in csv.DictReader(open(f)) if "k_sspp_c2f" in r["Kernel_Name"]]
    gkey = "Grid_Size" if rows and "Grid_Size" in rows[0] else "Grid_Size_X"
    gmax = max(int(r[gkey]) for r in rows)
    for r in rows:
        if int(r[gkey]) != gmax:
            continue
        acc.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    m = {k: sum(v.values()) / len(v) for k, v in acc.items()}
    w = m.get("SQ_WAVES", 1.0)
    print(os.path.basename(d), "grid", gmax, "launches", len(next(iter(acc.values()))),
          " ".join("%s/wave=%.0f" % (k[3:], v / w) for k, v in sorted(m.items()) if k != "SQ_WAVES"),
          "waves=%.0f" % w)
