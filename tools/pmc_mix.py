"""Per-kernel mean of every PMC counter over the passes in gpurun_out/TAG/p*/ (rocprofv3 csv).
    python tools/pmc_mix.py gpurun_out/TAG [kernel-substring] [out.json]
Adds derived figures: executed FP64 flops per launch (64 lanes x (ADD + MUL + TRANS + 2 FMA)
wave instructions; masked lanes count too, so this is an upper bound on useful flops)."""
import csv
import glob
import json
import os
import sys


def main(src, ksub="k_sspp_c2f", out=None):
    acc = {}
    for f in glob.glob(os.path.join(src, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if ksub not in r["Kernel_Name"]:
                continue
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in acc.items()}
    m["launches_sampled"] = max((len(v) for v in acc.values()), default=0)
    if "SQ_INSTS_VALU_FMA_F64" in m:
        m["fp64_flops_per_launch"] = 64.0 * (m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] +
                                             m["SQ_INSTS_VALU_TRANS_F64"] + 2 * m["SQ_INSTS_VALU_FMA_F64"])
    print(json.dumps(m, indent=1, sort_keys=True))
    if out:
        json.dump(m, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
