"""The roofline launches in a rocprofv3 kernel trace of bench.py: the average duration of the
dominant kernel's last N dispatches of the most frequent grid (bench.py issues its
--roofline-launches (default 20) after the timed loop, back to back on one stream), against the
average over every dispatch (the timed loop's launches overlap on several streams, so each one
takes longer than it does alone).
    python tools/trace_roofline.py run_kernel_trace.csv KERNEL_SUBSTRING [N]"""
import collections
import csv
import sys

path, kern = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
grid = collections.Counter(r["Grid_Size_X"] for r in rows).most_common(1)[0][0]
rows = sorted((r for r in rows if r["Grid_Size_X"] == grid), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
print("kernel %s, grid %s x %s threads: %d dispatches" % (kern, grid, rows[0]["Workgroup_Size_X"], len(d)))
print("  last %d (bench.py's roofline launches, one stream): %.1f us average" % (n, sum(d[-n:]) / n))
print("  timed loop (%d, streams %s): %.1f us average" % (len(d) - n, sorted({r["Stream_Id"] for r in rows[:-n]}),
                                                       sum(d[:-n]) / max(1, len(d) - n)))
