#!/bin/bash
# Build libzfp_hip.so variants with extra -D flags into tools/exp/var/<name>/
# (each dir gets a copy of libzfp.so, whose rpath $ORIGIN picks the variant).
#   tools/exp/variants.sh name "-DFOO=1 -DBAR" [name2 "flags2" ...]
# Only zfp_hip.hip is rebuilt per variant; the generic 1D/2D/integer units are
# linked from the main build's objects.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
OBJ=$R/zfp-par_amd/build/obj
while [ $# -ge 2 ]; do
  d=$R/tools/exp/var/$1
  mkdir -p $d
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$R/include -I$R/zfp-par_amd/csrc/host \
      -I$R/zfp-par_amd/csrc/hip $2 -c -o $d/zfp_hip.o $R/zfp-par_amd/csrc/hip/zfp_hip.hip &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o $d/libzfp_hip.so $d/zfp_hip.o $OBJ/zfp_hip_n32.o $OBJ/zfp_hip_n64.o &&
    rm -f $d/zfp_hip.o ) &
  shift 2
done
wait
for d in $R/tools/exp/var/*/; do cp $R/zfp-par_amd/lib/libzfp.so $d/; done
