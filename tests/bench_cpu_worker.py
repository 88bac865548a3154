"""Test infrastructure (tests/test_bench_dist.py): bench.py's driver logic -- rank
setup, the doc-weighted exchange, barriers, the max over ranks, the CPU baseline on
rank 0 while the other ranks wait, the one JSON line -- run on CPU over gloo, with
bench.HipBench's device seams replaced by a CPU stand-in whose step is the fp32
oracle port (oracle/dgl_udf.py) of the same stack.  The product path needs a GPU;
this checks the multi-rank plumbing the driver's N-GPU runs go through, not the
kernels.  Launched by torch.distributed.run:

    python -m torch.distributed.run --nproc-per-node 2 ... tests/bench_cpu_worker.py --gpus 2 ...
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class CpuRehearsal(bench.HipBench):
    graphs = False
    data = "CPU rehearsal of bench.py's driver logic (test only): the step is the fp32 oracle port"

    def __init__(self, args, rank, world, local):
        self.args, self.rank, self.world = args, rank, world
        self.dev = torch.device("cpu")
        torch.set_num_threads(1)

    def dist_kwargs(self, backend):
        return {}

    def load(self):
        pass

    def synchronize(self):
        pass

    def events(self, n):
        ts = [0.0] * n

        def mark(i):
            ts[i] = time.perf_counter()
        return mark, lambda i, j: (ts[j] - ts[i]) * 1e3

    def build(self, G, docs):
        from oracle import dgl_udf, fused
        args = self.args
        torch.manual_seed(args.seed)
        stack = bench.Stack(args.dropout, args.n_iter)
        offs = np.cumsum([0] + [d.n_nodes for d in docs])
        cat = lambda f: np.concatenate([f(d, o) for d, o in zip(docs, offs[:-1])])
        g = dgl_udf.UdfGraph(cat(lambda d, o: d.src + o), cat(lambda d, o: d.dst + o), cat(lambda d, o: d.unit),
                             cat(lambda d, o: d.tffrac), cat(lambda d, o: d.edtype))
        n_w, n_s = int((g.unit == 0).sum()), int((g.unit == 1).sum())
        rng = np.random.default_rng(args.seed * 7 + self.rank)
        Xw = torch.from_numpy((0.4 * rng.standard_normal((n_w, 300))).astype(np.float32))
        Xs = torch.from_numpy(rng.standard_normal((n_s, 64)).astype(np.float32))
        p1 = fused.as_params(stack.word2sent, torch.float32)
        p2 = fused.as_params(stack.sent2word, torch.float32)
        T = stack._TFembed.weight.detach().clone().requires_grad_()
        params = list(p1.values()) + list(p2.values()) + [T]

        def step():
            s = dgl_udf.stack_step(g, Xw, Xs, p1, p2, T, n_iter=args.n_iter, drop=args.dropout, training=True)
            s.sum().backward()

        def zero():
            for p in params:
                p.grad = None

        src, dst = g.src.numpy(), g.dst.numpy()
        self.n_typed = int(((g.unit[src] == 0) & (g.unit[dst] == 1)).sum())
        self.params = params
        return stack, step, zero, params

    def kernel_report(self, stack, step, zero, ms_per_step):
        return {"roofline": {"kernel": "cpu rehearsal: no kernel measured", "bound": "hbm", "achieved": 0.0,
                             "peak": bench.HBM_PEAK_GBS, "unit": "GB/s", "frac": 0.0, "traffic": None}}


if __name__ == "__main__":
    bench.main(CpuRehearsal)
