"""Per-kernel average duration over the last N dispatches of a rocprofv3
kernel trace (run_kernel_trace.csv): the bench's timed steps follow its
warm-up launches, whose clocks are still ramping, so the whole-run average of
--stats mixes cold launches in.

  python tools/prof_tail.py <dir with *_kernel_trace.csv> <N> [name-filter]
"""
import collections
import csv
import glob
import os
import sys

d, n = sys.argv[1], int(sys.argv[2])
filt = sys.argv[3] if len(sys.argv) > 3 else "zfp_amd"
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
by = collections.defaultdict(list)
for r in rows:
    if filt in r["Kernel_Name"]:
        by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
print("kernel,dispatches,last_n,avg_ms_last_n,min_ms,max_ms,avg_ms_all")
for k, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    tail = [x[1] for x in v[-n:]]
    allv = [x[1] for x in v]
    print('"%s",%d,%d,%.4f,%.4f,%.4f,%.4f' % (k.split("(")[0], len(v), len(tail), sum(tail) / len(tail) / 1e6,
                                            min(tail) / 1e6, max(tail) / 1e6, sum(allv) / len(allv) / 1e6))
