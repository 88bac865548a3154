"""The data-parallel exchange on RCCL (config 3's step, train.py:118-135),
exercised on the one GPU of the box before the driver's 8-GPU run.

* tests/rccl_worker.py: a world-size-1 ``nccl`` (RCCL) process group in one
  process; the fused stack's flat gradient buffer is all-reduced in place with the
  doc-weighted scale, eagerly and captured together with the step into ONE HIP
  graph; every replay leaves scale x the eager gradients.
* bench.py with HSG_DP_REHEARSAL=1: the bench's own multi-rank code path (RCCL
  communicator, exchange captured in the step graph) at world size 1.

Both run as subprocesses with a time limit, so a stuck collective ends the test,
not the test session."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    return dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")


def test_rccl_flat_exchange_captured_in_step_graph():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py")], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=240)
    print(out.stdout[-2000:])
    assert out.returncode == 0, out.stderr[-4000:]
    assert "replayed as one graph" in out.stdout


def test_bench_dp_path_on_rccl_world1():
    env = dict(_env(), HSG_DP_REHEARSAL="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--no-e2e",
                          "--no-cpu-baseline", "--kernel-reps", "5", "--kernel-steps", "2"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    ex = d["config"]["dp_exchange"]
    print(ex, d["ms_per_step"], d["median_ms_per_step"])
    assert "captured in the step's HIP graph" in ex and "nccl" in ex and "flat gradient buffer" in ex, ex
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["median_ms_per_step"] > 0
