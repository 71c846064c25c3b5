#!/bin/bash
# Per-call HBM traffic of a bench.py workload: one rocprofv3 --pmc run per
# counter group (kernel trace only) over
#   python bench.py --workload W --steps 2 --warmup 0 --clock-warm-ms 0 --no-cpu
# then tools/pmc_summary.py with that run's bench line (workload, field, call
# counts).  usage: tools/pmc_bench.sh TAG WORKLOAD [--sq]
# Writes gpurun_out/pmc_TAG_W/{p*,bench.json,summary.json,summary.txt}; copy
# summary.json to profiles/TAG_pmc_W.json for bench.py's `traffic`.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; W=$2; SQ=$3
OUT=$R/gpurun_out/pmc_${TAG}_$W
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=("FETCH_SIZE" "WRITE_SIZE")
if [ "$SQ" = "--sq" ]; then
  PASSES+=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
fi
i=0
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/bench.py --workload $W --steps 2 --warmup 0 --clock-warm-ms 0 --no-cpu > $OUT/p$i.log 2>&1 \
    || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
  [ $i = 1 ] && grep '^{' $OUT/p1.log | tail -1 > $OUT/bench.json
  echo "pass $i ok"
done
python3 $R/tools/pmc_summary.py $OUT --bench $OUT/bench.json > $OUT/summary.txt
rm -rf $OUT/p[0-9]*/  # raw counter CSVs: tens of MB, summarised above
