#!/bin/bash
# Host-resident (PCIe-inclusive) encode/decode rate of C2 through the C API,
# then one PMC pass (SQ counters only) over the device-resident encoder.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out
TAG=${1:-r1}
mkdir -p $OUT/pmc_$TAG
cd $R
timeout -k 10 300 python tools/kprof.py --host --mode rate --param 16 --iters 3 --decode > $OUT/host_$TAG.txt 2>&1 || exit 1
grep -v amdgpu.ids $OUT/host_$TAG.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
  --output-format csv -d $OUT/pmc_$TAG/p1 -o run -- python $R/tools/kprof.py --iters 2 > $OUT/pmc_$TAG/p1.log 2>&1 || exit 1
python $R/tools/pmc_summary.py $OUT/pmc_$TAG
