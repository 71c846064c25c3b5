#!/bin/bash
# A/B kernel timing of library builds: tools/ab_lib.sh "kprof args" lib_dir1 lib_dir2 ...
# (lib dirs relative to zfp-par_amd/: lib, lib_var/<name>); two alternating reps,
# the stream hash printed so variants can be checked for identical output.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ARGS=$1; shift
cd $R
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v rep $rep: $ARGS"
    timeout -k 10 150 python tools/kprof.py --lib zfp-par_amd/$v/libzfp.so --sha $ARGS 2>&1 | tail -4 || exit 1
  done
done
