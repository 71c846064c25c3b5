#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs per kernel (mean over dispatches)."""
import csv, glob, os, sys, collections, json
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        short = k.split("(")[0].replace("void ", "").replace("zfp_amd::", "")
        agg[short][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for k, m in agg.items():
    if "zfp" not in k and "encode" not in k and "decode" not in k and "enc_" not in k:
        continue
    per = collections.defaultdict(list)
    for (disp, name), vals in m.items():
        per[name].append(sum(vals))
    out[k] = {n: sum(v) / len(v) for n, v in per.items()}
for k, v in out.items():
    print(k)
    for n in sorted(v):
        print("   %-24s %16.1f" % (n, v[n]))
# HBM bytes per launch: gfx950 FETCH_SIZE counts half of the channels (KiB units),
# WRITE_SIZE all of them (MI355X_MICROARCH.md, HBM/rocprofv3 section)
for k, v in out.items():
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        v["hbm_read_bytes_per_launch"] = int(2 * v["FETCH_SIZE"] * 1024)
        v["hbm_write_bytes_per_launch"] = int(v["WRITE_SIZE"] * 1024)
        v["hbm_bytes_per_launch"] = v["hbm_read_bytes_per_launch"] + v["hbm_write_bytes_per_launch"]
for k in list(out):
    for short in ("encode3_aligned_full", "encode3_aligned", "decode3"):
        if k.startswith(short + "<float"):
            out.setdefault(short, dict(out[k], kernel=k))
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
