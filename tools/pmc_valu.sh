#!/bin/bash
# One PMC pass (instruction counts) over the light kernel driver: quick VALU-per-wave check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_${1:-valu}
shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/p1 -o run -- \
  python $R/tools/kprof.py --iters 2 "$@" > $OUT/p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
