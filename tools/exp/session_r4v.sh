# round-4 session v: counters of the index-scan passes (4D reversible 128^4), one rocprofv3 pass
set -o pipefail
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/r4v_scan_pmc/p1 -o run -- python $R/tools/scan_bench.py --n 128 --dims 4 --dtype f32 --mode reversible --reps 1 > $R/gpurun_out/r4v_scan_pmc.log 2>&1 || exit 1
cd $R
python3 - <<'PY' > gpurun_out/r4v_scan_pmc.txt
import csv, collections
rows = collections.defaultdict(dict)
for r in csv.DictReader(open("gpurun_out/r4v_scan_pmc/p1/run_counter_collection.csv")):
    if "scan_pass" not in r["Kernel_Name"]:
        continue
    d = rows[int(r["Dispatch_Id"])]
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for i, k in enumerate(sorted(rows)):
    d = rows[k]
    print(i + 1, " ".join("%s=%.0f" % (n, d[n]) for n in sorted(d)))
PY
head -5 gpurun_out/r4v_scan_pmc.txt; tail -5 gpurun_out/r4v_scan_pmc.txt
