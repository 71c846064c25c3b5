#!/bin/bash
# HBM traffic passes only (FETCH_SIZE, WRITE_SIZE; one rocprofv3 run each, kernel
# trace only) over any command: tools/pmc_traffic.sh OUTNAME -- cmd args...
# Writes gpurun_out/pmc_OUTNAME/summary.json (tools/pmc_summary.py: per kernel,
# hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE, KiB units).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_$1
shift; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.txt
