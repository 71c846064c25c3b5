#!/bin/bash
# Build the C2 encoder variants of tools/exp/c2var.hip (experiment harness):
# build_c2var.sh name "-D..." [name "-D..."]...
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$R/tools/exp/var
mkdir -p $OUT
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$R/zfp-par_amd/csrc/hip -I$R/include $2 -o $OUT/$1 $R/tools/exp/c2var.hip 2>&1 | grep -E "error" -A3 &
  shift 2
done
wait
ls $OUT
