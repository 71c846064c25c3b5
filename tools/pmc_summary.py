#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs of one profiled command, per codec call.

usage: python tools/pmc_summary.py DIR [--bench FILE] [--encode-calls N] [--decode-calls M]

DIR holds one sub-directory per counter pass (p1, p2, ... each a rocprofv3 -d
output).  Every dispatch of a zfp kernel is counted.  Kernels are grouped into
the two kinds of codec call: encode (encode*, fixup_*) and decode (decode*,
and the index scan: scan_pass, bm_tile_*, tile_scan, index_from_pos).  A call
can launch several kernels (encode4 + its fix-ups, decode4 + its overflow
relaunch, the scan passes), so the per-call figures SUM every dispatch of the
call's kind and divide by the number of calls; `dispatches_per_call` lists
what one call launched.  The call counts come from the bench line (--bench:
the JSON line bench.py printed for this command, its `calls` field, which
also gives the workload and field that tie the summary to a bench line) or
from --encode-calls / --decode-calls.

HBM bytes: gfx950 FETCH_SIZE counts half of the channels (KiB units), so reads
are 2 x FETCH_SIZE KiB; WRITE_SIZE counts all of them (MI355X_MICROARCH.md,
HBM/rocprofv3 section).
Output: DIR/summary.json and a table on stdout.
"""
import argparse
import collections
import csv
import glob
import json
import os

ENCODE = ("encode", "fixup")
DECODE = ("decode", "scan_pass", "bm_tile", "tile_scan", "index_from_pos")


def short_name(k):
    return k.split("(")[0].replace("void ", "").replace("zfp_amd::", "").strip()


def kind_of(name):
    if name.startswith(ENCODE):
        return "encode"
    if name.startswith(DECODE):
        return "decode"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--bench", help="bench.py JSON line of the profiled command")
    ap.add_argument("--encode-calls", type=int)
    ap.add_argument("--decode-calls", type=int)
    a = ap.parse_args()
    meta = {}
    calls = {"encode": a.encode_calls, "decode": a.decode_calls}
    if a.bench:
        line = [x for x in open(a.bench).read().splitlines() if x.startswith("{")][-1]
        b = json.loads(line)
        meta = {"workload": b["config"]["workload"], "workload_key": b.get("workload_key"),
                "field_per_gpu": b["config"]["field_per_gpu"],
                "algorithmic_bytes_per_call": b["roofline"]["algorithmic_bytes_per_launch"],
                "stream_bytes": b["config"]["stream_bytes_per_gpu"]}
        for k in ("encode", "decode"):
            if calls[k] is None:
                calls[k] = b.get("calls", {}).get(k)
    # counter name -> kernel -> dispatch id -> value (summed over the CSV's rows of that dispatch)
    val = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = short_name(r["Kernel_Name"])
            if kind_of(name) is None:
                continue
            val[r["Counter_Name"]][name][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    kernels = collections.defaultdict(dict)
    for cn, per_k in val.items():
        for name, per_d in per_k.items():
            kernels[name]["dispatches"] = max(kernels[name].get("dispatches", 0), len(per_d))
            kernels[name][cn + "_total"] = sum(per_d.values())
            kernels[name][cn + "_per_dispatch"] = sum(per_d.values()) / len(per_d)
    out = {"meta": meta, "calls": calls, "kernels": kernels}
    for kind in ("encode", "decode"):
        n = calls.get(kind)
        ks = {k: v for k, v in kernels.items() if kind_of(k) == kind}
        if not ks or not n:
            continue
        c = {"calls": n, "dispatches_per_call": {k: v["dispatches"] / n for k, v in ks.items()}}
        if all("FETCH_SIZE_total" in v and "WRITE_SIZE_total" in v for v in ks.values()):
            rd = sum(2 * v["FETCH_SIZE_total"] * 1024 for v in ks.values()) / n
            wr = sum(v["WRITE_SIZE_total"] * 1024 for v in ks.values()) / n
            c.update(hbm_read_bytes_per_call=int(rd), hbm_write_bytes_per_call=int(wr),
                     hbm_bytes_per_call=int(rd + wr))
            alg = meta.get("algorithmic_bytes_per_call")
            if alg and kind == "encode":
                c["hbm_over_algorithmic"] = round((rd + wr) / alg, 4)
        for cn in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT"):
            if all(cn + "_total" in v for v in ks.values()):
                c[cn + "_per_call"] = sum(v[cn + "_total"] for v in ks.values()) / n
        out[kind + "_call"] = c
    json.dump(out, open(os.path.join(a.dir, "summary.json"), "w"), indent=1)
    for k, v in sorted(kernels.items()):
        print("%-48s dispatches %d" % (k, v["dispatches"]))
        for cn in sorted(x for x in v if x.endswith("_per_dispatch")):
            print("   %-36s %18.1f" % (cn, v[cn]))
    for kind in ("encode", "decode"):
        if kind + "_call" in out:
            print(kind, "call:", json.dumps(out[kind + "_call"]))


if __name__ == "__main__":
    main()
