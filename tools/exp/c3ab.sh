cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in base lb3; do
  if [ $v = lb3 ]; then export ZFP_HIP_EXP_SWP=23; else unset ZFP_HIP_EXP_SWP; fi
  echo "== $v rep $rep"
  timeout -k 10 120 python tools/kprof.py --lib tools/exp/var/$v/libzfp.so --mode precision --param 32 --dtype f64 --iters 6 --sha 2>&1 | grep -v amdgpu.ids || exit 1
  timeout -k 10 120 python tools/kprof.py --lib tools/exp/var/$v/libzfp.so --mode reversible --iters 6 --sha 2>&1 | grep -v amdgpu.ids || exit 1
done
done
