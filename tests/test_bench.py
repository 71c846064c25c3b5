"""bench.py launcher contract on CPU (no GPU): `--gpus N` without WORLD_SIZE
re-launches itself under torch.distributed.run with N ranks, and rank 0 prints
exactly one JSON line whose n_gpus is N (gloo dry run: a numpy copy stands in
for the codec; the GPU path is exercised by the driver's bench runs)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(gpus, workload="c2"):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--dry-run",
                        "--steps", "3", "--warmup", "1", "--workload", workload], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_spawns_two_ranks():
    d = _run(2)
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert d["steps"] == 3 and d["warmup"] == 1 and d["scaling"] == "weak"
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "vs_baseline", "dtype", "config"):
        assert k in d


def test_single_rank_runs_in_process():
    d = _run(1)
    assert d["n_gpus"] == 1


@pytest.mark.parametrize("workload", ["c3", "c5"])
def test_variable_rate_workloads_launch_two_ranks(workload):
    d = _run(2, workload)
    assert d["n_gpus"] == 2 and workload in d["config"]["workload"]
