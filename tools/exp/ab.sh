#!/bin/bash
# A/B kernel timing of library variants (tools/exp/var/<name>), alternating runs
#   tools/exp/ab.sh "kprof args" name1 name2 [...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
ARGS=$1; shift
cd $R
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v rep $rep: $ARGS"
    timeout -k 10 120 python tools/kprof.py --lib tools/exp/var/$v/libzfp.so $ARGS 2>&1 | tail -3 || exit 1
  done
done
