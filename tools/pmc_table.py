"""Per-kernel PMC table from rocprofv3 --pmc csv runs: mean counter per dispatch
and per wave.  usage: python tools/pmc_table.py gpurun_out/<dir> [kernel-substring]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if flt not in k:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    # counters are reported per dispatch (summed over dimensions by rocprofv3)
    n = {c: sum(v) / len(v) for c, v in d.items()}
    waves = n.get("SQ_WAVES")
    print(k[:90])
    for c in sorted(n):
        per = " %.1f/wave" % (n[c] / waves) if waves else ""
        print("   %-22s %16.0f%s" % (c, n[c], per))
