#!/bin/bash
# Build libzfp_hip.so of a git revision (or the working tree: REV=WT) into
# tools/exp/var/<name>/ next to a copy of the current libzfp.so, for A/B timing:
#   tools/exp/build_rev.sh <rev|WT> <name> ["extra hipcc flags"]
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
REV=$1; NAME=$2; FLAGS=$3
D=$R/tools/exp/var/$NAME
mkdir -p $D
if [ "$REV" = WT ]; then SRC=$R; else
  SRC=$(mktemp -d /tmp/rev_XXXX)
  (cd $R && git archive $REV include zfp-par_amd/csrc) | tar -x -C $SRC
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$SRC/include -I$SRC/zfp-par_amd/csrc/host \
  -I$SRC/zfp-par_amd/csrc/hip $FLAGS -shared -o $D/libzfp_hip.so $SRC/zfp-par_amd/csrc/hip/zfp_hip.hip
cp $R/zfp-par_amd/lib/libzfp.so $D/
echo built $D
