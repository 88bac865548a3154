"""bench.py's multi-rank line: ``bench.py --gpus 2`` under
torch.distributed.run, world size 2 over gloo on CPU, with the device seams of
bench.HipBench replaced by tests/bench_cpu_worker.py's CPU stand-in (the product
kernels need a GPU).  The JSON line that rank 0 prints must carry the contract keys,
n_gpus = 2, the data-parallel exchange, the roofline object and the CPU baseline --
which rank 0 now times after the timed region at every world size while rank 1
waits at a barrier (every GPU count beside the CPU number)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo_json_line():
    env = dict(os.environ, HSG_DIST_BACKEND="gloo", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "bench_cpu_worker.py"), "--gpus", "2", "--config", "cfg1",
           "--steps", "2", "--warmup", "1", "--cpu-steps", "1", "--no-e2e"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout                       # exactly one JSON line, from rank 0
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 2
    assert d["config"]["parallelism"] == "dp2"
    assert "world 2" in d["config"]["dp_exchange"] and "gloo" in d["config"]["dp_exchange"]
    assert d["config"]["docs_per_gpu"] == 4                 # cfg1: 4 docs per rank, 8 in the job
    cb = d["cpu_baseline"]
    assert "error" not in cb, cb
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1
    assert "rank 0's shard of the 2-rank job" in cb["sample"]
    assert d["value"] > 0 and d["ms_per_step"] > 0
