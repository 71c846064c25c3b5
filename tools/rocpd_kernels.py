#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 run written in its SQLite (rocpd) format
(rocprofv3 -d DIR without --output-format csv): dispatches, average duration
over all and over the last N dispatches of each kernel -- the same columns as
tools/prof_tail.py prints for a CSV kernel trace.

  python tools/rocpd_kernels.py DIR/run_results.db [N] [name-filter]
"""
import collections
import sqlite3
import sys

db, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20
filt = sys.argv[3] if len(sys.argv) > 3 else "zfp_amd"
rows = sqlite3.connect(db).execute("select name, start, duration from kernels").fetchall()
by = collections.defaultdict(list)
for name, start, dur in rows:
    if filt in name:
        by[name].append((int(start), int(dur)))
print("kernel,dispatches,last_n,avg_ms_last_n,min_ms,max_ms,avg_ms_all")
for k, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    tail = [x[1] for x in v[-n:]]
    allv = [x[1] for x in v]
    print('"%s",%d,%d,%.4f,%.4f,%.4f,%.4f' % (k.split("(")[0], len(v), len(tail), sum(tail) / len(tail) / 1e6,
                                            min(tail) / 1e6, max(tail) / 1e6, sum(allv) / len(allv) / 1e6))
