set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/host_pipe.txt
for env in "" "ZFP_HIP_NO_PIPE=1"; do
  echo "== $env" >> gpurun_out/host_pipe.txt
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --mode precision --param 32 --dtype f64 --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
  env $env timeout -k 10 200 python tools/kprof.py --host --iters 3 --dims 4 --n 128 --mode reversible --decode >> gpurun_out/host_pipe.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/zfp_par_bench.py >> gpurun_out/host_pipe.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/host_pipe.txt
