# round-4 session x: new block-API/call tests, scan counters, C5 kernel split
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_block_api.py -k "compress_call" > gpurun_out/r4x_tests.txt 2>&1 || { tail -30 gpurun_out/r4x_tests.txt; exit 1; }
tail -1 gpurun_out/r4x_tests.txt
bash tools/exp/session_r4v.sh || exit 1
bash tools/exp/session_r4w.sh || exit 1
