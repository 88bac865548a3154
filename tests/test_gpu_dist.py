"""Data parallelism of the HIP path itself (train.py:130-135): two
ranks, launched by torch.distributed.run as a subprocess (gloo, both on cuda:0 of
the one-GPU box), each run the fused WSWGAT stack on its shard of a skewed
5-document batch; the hook-driven bucketed all-reduce (doc-weighted) plus
clip_grad_norm_ must reproduce the full-batch gradient and norm
(tests/dist_gpu_worker.py).  The 8-GPU RCCL run is the driver's bench."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_hip_stack_matches_full_batch():
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                          os.path.join(here, "dist_gpu_worker.py")],
                         cwd=os.path.dirname(here), env=env, capture_output=True, text=True, timeout=300)
    print(out.stdout[-2000:])
    assert out.returncode == 0, out.stderr[-4000:]
    assert out.stdout.count("max rel grad err") == 2
