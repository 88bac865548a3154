#!/usr/bin/env python
"""Benchmark: graph-edges/sec through the WSWGAT stack fwd+bwd (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
    torchrun --nproc-per-node N bench.py --gpus N ...       (driver launches N>1)

One step = forward + backward of the HSG GAT stack W2S + n_iter x (S2W, W2S)
(HiGraph.py:99-106, n_iter=2), all heads, FFNs included, in training mode
(reference dropout 0.1), on one synthetic CNN/DM-shaped batch per GPU (config 2:
32 docs x N=35 sentences, W=600 words, k=36 words/sentence = 159,040 graph
edges incl. the s<->s phantom edges).  With N>1 each rank owns its own 32-doc
shard (weak scaling) and the step ends with the data-parallel gradient
all-reduce over RCCL (the path's one exchange step).  Encoders,
graph construction and H2D copies are outside the step.  The step
is captured once into a HIP graph and replayed.

value = E_global / t_step: all ranks' graph edges over the max-over-ranks time of
one step (timed region / K).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP32_MFMA_PEAK_TFLOPS = 157.3  # v_mfma_f32_32x32x2_f32 dense (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--n-iter", type=int, default=2)
    ap.add_argument("--dtype", choices=("f32", "bf16"), default="f32",
                    help="GEMM operand precision: f32 (parity contract) or bf16 (config 5)")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-docs", type=int, default=0,
                    help="docs in the CPU-baseline sample (0: the whole per-GPU batch)")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--kernel-steps", type=int, default=10, help="eager steps of the in-step kernel timing")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--no-e2e", action="store_true", help="skip the secondary end-to-end train-step line")
    ap.add_argument("--e2e-steps", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    return ap.parse_args()


class _HPS:
    """train.py's argparse defaults (train.py:279-309), n_iter from the bench."""

    def __init__(self, n_iter, doc_max_timesteps=50):
        self.__dict__.update(dict(
            vocab_size=50000, n_iter=n_iter, word_emb_dim=300, embed_train=False, feat_embed_size=50,
            lstm_hidden_state=128, lstm_layers=2, bidirectional=True, n_feature_size=128, hidden_size=64,
            ffn_inner_hidden_size=512, n_head=8, recurrent_dropout_prob=0.1, atten_dropout_prob=0.1,
            ffn_dropout_prob=0.1, sent_max_len=100, doc_max_timesteps=doc_max_timesteps, lr=0.0005, cuda=True))


def time_train_step(G, config, n_iter, steps, warmup, dev):
    """Secondary figure: one whole training iteration of train.py:104-133
    on this rank's batch -- HSumGraph (HSumDocGraph for cfg4) forward with the CNN +
    LSTM sentence encoder, per-sentence cross entropy summed per graph and averaged,
    the finiteness check (a host sync, as the reference does), zero_grad, backward,
    Adam.  Eager launches, random-init weights, frozen embedding (embed_train=False)."""
    from hetersumgraph_amd import HiGraph
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd.HiGraph import node_ids
    # the workload's own doc_max_timesteps (80 for the NYT50 shape): sentence
    # positions index the model's position table, checked here on the host so a
    # mismatch raises instead of faulting in the embedding gather
    hps = _HPS(n_iter, doc_max_timesteps=80 if config == "cfg5" else 50)
    pos = G.ndata["position"][node_ids(G, "dtype", 1.0)]
    if int(pos.max()) > hps.doc_max_timesteps or int(G.ndata["label"].shape[1]) > hps.doc_max_timesteps:
        raise ValueError("sentence positions / labels exceed doc_max_timesteps of the e2e model")
    torch.manual_seed(1)
    embed = torch.nn.Embedding(hps.vocab_size, hps.word_emb_dim, padding_idx=0)
    embed.weight.requires_grad = hps.embed_train
    cls = HiGraph.HSumDocGraph if config == "cfg4" else HiGraph.HSumGraph
    model = cls(hps, embed).to(dev).train()
    opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=hps.lr)
    criterion = torch.nn.CrossEntropyLoss(reduction="none")

    def step():
        outputs = model.forward(G)                                          # [n_snodes, 2]
        snode_id = G.filter_nodes(lambda nodes: nodes.data["dtype"] == 1)
        label = G.ndata["label"][snode_id].sum(-1)
        G.nodes[snode_id].data["loss"] = criterion(outputs, label).unsqueeze(-1)
        loss = hg.sum_nodes(G, "loss").mean()
        if not bool(torch.isfinite(loss).item()):          # host sync, as train.py:120
            raise RuntimeError("train loss is not finite")
        opt.zero_grad()
        loss.backward()
        opt.step()
        G.ndata.pop("loss")          # train.py sees a fresh graph per batch; this one is reused

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return dt


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def model_name(config):
    """The reference model the config's batch feeds: HSumDocGraph for the HDSG
    (doc-node) batch of config 4 (HiGraph.py:166-244), HSumGraph otherwise."""
    from hetersumgraph_amd import synth
    return "HDSG" if synth.CONFIGS[config][0] == "hdsg" else "HSG"


def workload_shape(config):
    from hetersumgraph_amd import synth
    kind, per_gpu, p = synth.CONFIGS[config]
    shape = ", ".join(f"{k}={v}" for k, v in p.items())
    return f"{per_gpu} {kind.upper()} docs/GPU x ({shape})"


def make_shard(config, rank, world, seed):
    """The global batch (32 docs per GPU, seeded) split by document across ranks
    (hetersumgraph_amd.parallel.shard_documents); returns this rank's docs, its
    batched graph, the global edge count and this rank's share of the documents
    (the weight of its per-rank-mean gradient in the global mean)."""
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.parallel import shard_documents, shard_fraction
    per_gpu = synth.CONFIGS[config][1]
    docs_all = synth.make_batch_docs(config, seed=seed, n_docs=per_gpu * world)
    docs = shard_documents(docs_all, rank, world)
    G = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    return docs, G, int(sum(len(d.src) for d in docs_all)), shard_fraction(docs_all, rank, world)


class Stack(torch.nn.Module):
    """The timed unit: W2S + n_iter x (S2W, W2S) with the reference's shapes."""

    def __init__(self, drop, n_iter):
        super().__init__()
        from hetersumgraph_amd.module.GAT import WSWGAT
        self.word2sent = WSWGAT(300, 64, 8, drop, 512, drop, 50, "W2S")
        self.sent2word = WSWGAT(64, 300, 6, drop, 512, drop, 50, "S2W")
        self._TFembed = torch.nn.Embedding(10, 50)
        self.n_iter = n_iter

    def forward(self, G, Xw, Xs):
        from hetersumgraph_amd.HiGraph import register_tfidf_table
        from hetersumgraph_amd.stack import fused_stack_ok, gat_stack
        T = self._TFembed.weight
        register_tfidf_table(G, T)
        if fused_stack_ok(G, self.word2sent, self.sent2word, T, Xw, Xs):   # as HSumGraph.gat_stack
            return gat_stack(G, self.word2sent, self.sent2word, T, Xw, Xs, self.n_iter)
        w, s = Xw, self.word2sent(G, Xw, Xs)
        for _ in range(self.n_iter):
            w = self.sent2word(G, w, s)
            s = self.word2sent(G, w, s)
        return s


# ------------------------------------------------------------------ roofline --
def edge_bytes_fwd(rel, H, D):
    """SURVEY §8(d) compulsory HBM bytes of one edge forward (hsg_gat_fwd) with
    D = H*D the concatenated width: read Z and sigma (n_src rows), the CSR offsets
    and phantom counts (8 B / destination), 5 B per typed edge (int32 source +
    uint8 tf box), write the aggregate and the softmax state m, l (2H)."""
    W = H * D
    return 4 * rel.n_src * (W + H) + 8 * rel.n_dst + 4 + 5 * rel.n_typed + 4 * rel.n_dst * (W + 2 * H)


def edge_bytes_bwd(rel, H, D):
    """SURVEY §8(d) compulsory bytes of one edge backward (dst + src passes; on S2W
    the one source-centric pass hsg_gat_bwd_src_g, which reads G instead of dOut and
    h -- the same count): read dOut and the saved state, gather Z / write dZ and
    dsigma over the sources, the CSR + CSC edge arrays (10 B / typed edge) and
    offsets."""
    W = H * D
    return (4 * (2 * rel.n_dst * W + 2 * rel.n_dst * H) + 8 * rel.n_src * (W + H) + 10 * rel.n_typed
            + 8 * (rel.n_dst + rel.n_src) + 8)


def epilogue_bytes_fwd(rel, H, D):
    """Bytes the fused forward moves beyond §8(d): the ELU + residual epilogue's
    origin read (GAT.py:56-57; a separate elementwise kernel would read h and origin
    and write out)."""
    return 4 * rel.n_dst * H * D


def step_work(rel_w, rel_s, n_iter, gemm_dtype, word_grad=False, issued=False):
    """Per-step work items (name, bytes, flops, peak TFLOP/s) of the timed stack
    (W2S + n_iter x (S2W, W2S), fwd + bwd) for the full-stack floor
    sum_k max(B_k / BW, F_k / peak_k).  Dense bytes are the GEMM
    operands and results (fp32); the FFN and head-projection flops are exact.
    ``issued``: price the wide (S2W) FFN GEMMs at the rate the path ISSUES them --
    in 'f32' mode six bf16 limb products per fp32-accurate product on the bf16 MFMA
    (2.5 PF/s / 6 = 417 TF/s fp32-equivalent) -- instead of the exact-f32 MFMA peak."""
    if gemm_dtype == "bf16":
        dense_peak = BF16_MFMA_PEAK_TFLOPS
    else:
        dense_peak = BF16_MFMA_PEAK_TFLOPS / 6 if issued else FP32_MFMA_PEAK_TFLOPS
    items = []
    layers = {"W2S": (rel_w, 300, 8, 8, 64), "S2W": (rel_s, 64, 6, 50, 300)}
    apps = ["W2S"] + ["S2W", "W2S"] * n_iter
    for i, kind in enumerate(apps):
        rel, d_in, H, D, d = layers[kind]
        HD = H * D
        items.append((f"edge_fwd_{kind}", edge_bytes_fwd(rel, H, D), 0.0, None))
        items.append((f"edge_bwd_{kind}", edge_bytes_bwd(rel, H, D), 0.0, None))
        n = rel.n_src
        proj = 2.0 * n * d_in * HD
        nb_grad = word_grad or i > 0          # app 0's neighbour is the frozen word embedding
        items.append((f"hproj_{kind}", 4.0 * (n * d_in + HD * d_in + n * HD) * (3 if nb_grad else 2),
                      proj * (3 if nb_grad else 2), FP32_MFMA_PEAK_TFLOPS))
        m, dh = rel.n_dst, 512
        # W2S (d = 64) FFN stays fp32 in every mode (one-launch kernel)
        peak = FP32_MFMA_PEAK_TFLOPS if kind == "W2S" else dense_peak
        ffn = 2.0 * m * d * dh
        items.append((f"ffn_{kind}", 4.0 * (m * d + m * dh) * 2 * 3, 6 * ffn, peak))
    # the deferred FFN weight gradients' split-K partial slabs (dense.gemm_dw_slabs): each
    # of dW1, dW2 of a layer writes and re-reads `splits` [d x 512] fp32 slabs, summed
    # by hsg_slab_reduce (these bytes belong to the step's dense work)
    for kind, (rel, d_in, H, D, d) in layers.items():
        splits = dw_slab_splits(rel.n_dst * apps.count(kind), d, 512)
        if splits > 1:
            items.append((f"ffn_dw_slabs_{kind}", 2 * 2 * 4.0 * splits * d * 512, 0.0, None))
    return items


DW_TILES = ((160, 128), (128, 160), (128, 128))


def dw_tiles(M, N):
    """Output tiles of one hsg_gemm_dw_slabs job (csrc/hsg_dw.hip pick_cfg: the tile
    with the least padded area, ties to the first), mirrored on the host so the byte
    count needs no HIP library (tests/test_abi.py pins it to hsg_gemm_dw_tiles)."""
    best = None
    for bm, bn in DW_TILES:
        t = (-(-M // bm), -(-N // bn))
        area = t[0] * bm * t[1] * bn
        if best is None or area < best[0]:
            best = (area, t[0] * t[1])
    return best[1]


def dw_slab_splits(K, d, dh):
    """K slices of a layer's FFN weight-gradient pair over K rows, mirrored on the host
    for the byte count: the product backward runs both gradients in one
    hsg_gemm_dw_slabs launch with dense.gemm_dw_slabs' rule -- two blocks per CU over
    the pair's tiles, at least 4 K tiles per slice, every slice non-empty -- and
    falls back to dense.gemm_slabs' 64 slices only when that declines (1: not split)."""
    kt = (K + 31) // 32
    tiles = dw_tiles(d, dh) + dw_tiles(dh, d)
    splits = max(1, min(max(1, (2 * 256) // max(tiles, 1)), kt // 4))
    per = (kt + splits - 1) // splits
    splits = (kt + per - 1) // per
    if splits >= 2:
        return splits
    from hetersumgraph_amd.dense import auto_splits
    if auto_splits(d, dh, K) < 2:
        return 1
    return max(2, min(64, kt))


def full_stack_floor(items):
    """(floor seconds, edge-floor s, dense-floor s, dense GFLOP)."""
    edge = sum(b / (HBM_PEAK_GBS * 1e9) for n, b, f, _ in items if n.startswith("edge_"))
    dense = sum(max(b / (HBM_PEAK_GBS * 1e9), f / (pk * 1e12) if f > 0 else 0.0)
                for n, b, f, pk in items if not n.startswith("edge_"))
    return edge + dense, edge, dense, sum(f for _, _, f, _ in items) / 1e9


def time_edge_kernels_in_step(step, zero, n_steps):
    """Average duration of every edge-kernel launch INSIDE eager training steps:
    HIP events recorded by the kernels' own dispatch packets on the launching stream
    (hipExtLaunchKernel via hsg_kclock_arm) for each hsg_gat_fwd and each
    (hsg_gat_bwd_dst + hsg_gat_bwd_src) pair or one-pass hsg_gat_bwd_src_g
    (hetersumgraph_amd._lib.KernelClock),
    so each launch runs with the caches its real predecessors in the step leave.
    Returns tag -> (mean ms, launches per step)."""
    from hetersumgraph_amd._lib import KernelClock
    with KernelClock() as clk:
        for _ in range(n_steps):
            zero()
            step()
        d = clk.durations_ms()
    return {t: (float(np.mean(v)), len(v) / n_steps) for t, v in d.items()}


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3
    FETCH_SIZE / WRITE_SIZE passes over in-step launches (tools/pmc_traffic.py), or
    None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
            return d["traffic_bytes"], os.path.relpath(path, ROOT), d
    except (OSError, KeyError, ValueError):
        return None, None, None


def time_dense_kernel(stack, n_rows, reps):
    """Average duration of the S2W FFN first GEMM (x W1^T + b1, ReLU;
    [n_w, 300] x [300, 512]) on the stack's own weights, on the path the step runs
    (hsg_gemm_f32_psw on the pre-split W1 in 'f32' mode, else hsg_gemm_*),
    back-to-back launches between HIP events on the launching stream.  Returns
    (ms, flops per launch, entry point name)."""
    from hetersumgraph_amd.dense import gemm, gemm_psw
    from hetersumgraph_amd.ffn import ffn_wsplit
    ffn = stack.sent2word.ffn
    w1, b1 = ffn.w_1.weight.detach().squeeze(-1).contiguous(), ffn.w_1.bias.detach()
    w2, b2 = ffn.w_2.weight.detach().squeeze(-1).contiguous(), ffn.w_2.bias.detach()
    x = torch.randn(n_rows, w1.shape[1], device=w1.device)
    out = x.new_empty(n_rows, w1.shape[0])
    ws = ffn_wsplit(x, w1, b1, w2, b2)
    if ws is not None:
        run = lambda: gemm_psw(x, ws[0], bias=b1, relu=True, out=out)
        name = "hsg_gemm_bf16_psw" if ws[0].mode == "bf16" else "hsg_gemm_f32_psw"
    else:
        run, name = (lambda: gemm(x, w1, b_t=True, bias=b1, relu=True, out=out)), "hsg_gemm_*"
    st = torch.cuda.current_stream()
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(reps):
        run()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, 2.0 * n_rows * w1.shape[0] * w1.shape[1], name


def dense_roofline(name, rows, useful_tf, flops, ms, dtype):
    """The S2W FFN GEMM against the peak of the MFMA it actually issues.
    'f32' mode runs hsg_gemm_f32_psw: fp32-accurate products as SIX bf16 limb
    products each on v_mfma_*_bf16, so the issued work is 6x the useful flops and
    the bound is the bf16 MFMA peak; 'bf16' mode issues the useful flops on the same
    peak.  ``fp32_equivalent`` keeps the useful rate against the exact-f32 MFMA peak
    (157.3 TF/s) for comparison with an fp32 GEMM."""
    products = 6 if dtype == "f32" and name == "hsg_gemm_f32_psw" else 1
    issued_tf = useful_tf * products
    out = {"kernel": f"{name} (S2W FFN x W1^T + b1, ReLU; {rows}x300 @ 300x512)", "bound": "mfma",
           "achieved": issued_tf, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": issued_tf / BF16_MFMA_PEAK_TFLOPS,
           "achieved_is": (f"issued bf16 MFMA FLOP/s ({products} bf16 limb products per fp32-accurate product)"
                           if products > 1 else "bf16 MFMA FLOP/s"),
           "flops_per_launch": flops, "issued_flops_per_launch": flops * products,
           "avg_launch_us": ms * 1e3}
    if products > 1:
        out["fp32_equivalent"] = {"achieved": useful_tf, "peak": FP32_MFMA_PEAK_TFLOPS,
                                  "frac": useful_tf / FP32_MFMA_PEAK_TFLOPS,
                                  "what": "useful (fp32) FLOP/s against the exact-f32 MFMA peak"}
    return out


# ------------------------------------------------------------- CPU baseline --
def cpu_threads():
    """(threads to use, host cores visible): every core this process may run on --
    the affinity mask, capped by the cgroup CPU quota when one is set (a container's
    CPU share; more threads than the quota only time-slice)."""
    visible = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    return (min(visible, quota) if quota else visible), visible, quota


def cpu_baseline(docs, args, stack):
    """The DGL-UDF-structured CPU port (oracle/dgl_udf.py) on the same workload's
    documents, on every core this process may use; median of ``--cpu-steps``
    fwd+bwd steps after one warm-up.  ``--cpu-docs`` (default: all of this rank's
    documents) bounds the sample."""
    from oracle import dgl_udf, fused
    threads, visible, quota = cpu_threads()
    torch.set_num_threads(threads)
    n_docs = len(docs) if args.cpu_docs <= 0 else min(args.cpu_docs, len(docs))
    sample = docs[:n_docs]
    offs = np.cumsum([0] + [d.n_nodes for d in sample])
    cat = lambda f: np.concatenate([f(d, o) for d, o in zip(sample, offs[:-1])])
    g = dgl_udf.UdfGraph(cat(lambda d, o: d.src + o), cat(lambda d, o: d.dst + o), cat(lambda d, o: d.unit),
                         cat(lambda d, o: d.tffrac), cat(lambda d, o: d.edtype))
    n_w, n_s = int((g.unit == 0).sum()), int((g.unit == 1).sum())
    rng = np.random.default_rng(5)
    Xw = torch.from_numpy((0.4 * rng.standard_normal((n_w, 300))).astype(np.float32))
    Xs = torch.from_numpy(rng.standard_normal((n_s, 64)).astype(np.float32))
    p1 = fused.as_params({k: v.cpu() for k, v in stack.word2sent.state_dict().items()}, torch.float32)
    p2 = fused.as_params({k: v.cpu() for k, v in stack.sent2word.state_dict().items()}, torch.float32)
    T = stack._TFembed.weight.detach().cpu().clone().requires_grad_()
    E = len(g.src)

    def step():
        Xs_ = Xs.clone().requires_grad_()
        s = dgl_udf.stack_step(g, Xw, Xs_, p1, p2, T, n_iter=args.n_iter, drop=args.dropout, training=True)
        s.sum().backward()

    step()  # warm-up
    times = []
    for _ in range(args.cpu_steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    return {"value": E / dt, "unit": "graph-edges/s", "cores": threads, "kind": "port",
            "host_cores_visible": visible, "cgroup_cpu_quota": quota,
            "sample": f"{n_docs} of the {len(docs)} {args.config} docs of this GPU's batch ({E} of "
                      f"{sum(len(d.src) for d in docs)} graph edges), median of {args.cpu_steps} fwd+bwd steps "
                      f"of the same stack (W2S + {args.n_iter}x(S2W, W2S), train mode), fp32, torch CPU on "
                      f"{threads} threads, {cpu_model()}; oracle/dgl_udf.py (DGL-0.4 UDF structure)",
            "ms_per_step": dt * 1e3, "step_ms_all": [t * 1e3 for t in times]}


class HipBench:
    """The measured path: the fused WSWGAT stack of libhsg.so on this rank's ROCm
    device, captured into a HIP graph.  ``main`` drives it through these seams --
    device, synchronisation, per-step events, the step itself and the in-step
    kernel measurements -- so that the multi-rank driver logic (barriers, max over
    ranks, the exchange, the JSON line, the CPU baseline on rank 0) is one code path
    for every world size; tests/bench_cpu_worker.py replays that logic over gloo on
    CPU with a stand-in step (test infrastructure, not a product path)."""

    graphs = True
    data = "synthetic (seeded CNN/DM-shaped graphs, random-init weights of the reference architecture)"

    def __init__(self, args, rank, world, local):
        self.args, self.rank, self.world = args, rank, world
        # one rank per GPU; ranks beyond the visible devices share them (only for the
        # single-GPU rehearsal of the multi-rank path with HSG_DIST_BACKEND=gloo)
        ndev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local % ndev)
        self.dev = torch.device("cuda", local % ndev)

    def dist_kwargs(self, backend):
        return {"device_id": self.dev} if backend == "nccl" else {}

    def load(self):
        from hetersumgraph_amd import _lib
        _lib.load()
        from hetersumgraph_amd.dense import set_gemm_dtype
        set_gemm_dtype(self.args.dtype)

    def synchronize(self):
        torch.cuda.synchronize()

    def events(self, n):
        st = torch.cuda.current_stream(self.dev)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
        return lambda i: evs[i].record(st), lambda i, j: evs[i].elapsed_time(evs[j])

    def build(self, G, docs):
        """(stack, step, zero, params): the timed unit on this rank's batch."""
        args, dev = self.args, self.dev
        G.to(dev)
        torch.manual_seed(args.seed)                       # identical replicas on every rank
        stack = Stack(args.dropout, args.n_iter).to(dev).train()
        rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
        gen = torch.Generator(device=dev).manual_seed(args.seed * 7 + self.rank)
        Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)      # word embeddings (frozen)
        Xs = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen).requires_grad_()   # encoder output
        R = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen)
        params = [p for p in stack.parameters() if p.requires_grad]
        from hetersumgraph_amd import rng as hsg_rng

        def step():
            hsg_rng.advance_all()          # fresh dropout masks every step (device-side: replays too)
            s = stack(G, Xw, Xs)
            s.backward(R)                  # d/ds of sum(s * R): the upstream gradient of the stack output

        def zero():
            # optimizer.zero_grad() (set_to_none): backward then writes fresh gradients
            for p in params:
                p.grad = None
            Xs.grad = None

        self.rel_w, self.rel_s, self.n_typed = rel_w, rel_s, rel_w.n_typed
        return stack, step, zero, params

    def capture(self, step, zero, allreduce, with_exchange):
        dev = self.dev
        s_side = torch.cuda.Stream(dev)
        s_side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s_side):
            for _ in range(2):
                zero()
                step()
                if with_exchange:
                    allreduce()
        torch.cuda.current_stream(dev).wait_stream(s_side)
        zero()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
            if with_exchange:
                allreduce()
        torch.cuda.synchronize()
        return g

    def kernel_report(self, stack, step, zero, ms_per_step):
        """The roofline objects of the JSON line: the S2W edge forward (the north-star
        kernel), every edge kernel of the step, the full-stack floor and the S2W FFN
        GEMM, all timed after the timed region."""
        args = self.args
        rel_w, rel_s = self.rel_w, self.rel_s
        # edge kernels timed inside eager steps (HIP events of their dispatches), after the
        # timed region so they cannot perturb it
        kt = time_edge_kernels_in_step(step, zero, args.kernel_steps)
        Hs, Ds = stack.sent2word.layer.num_heads, stack.sent2word.layer.head_dim
        Hw, Dw = stack.word2sent.layer.num_heads, stack.word2sent.layer.head_dim
        shapes = {"S2W": (rel_s, Hs, Ds), "W2S": (rel_w, Hw, Dw)}
        k_ms = kt[("gat_fwd", "S2W")][0]
        k_bytes = edge_bytes_fwd(rel_s, Hs, Ds)
        achieved = k_bytes / (k_ms * 1e-3) / 1e9
        e_bytes = e_ms = 0.0
        edge_rows = {}
        for (what, kind), (ms, per_step) in sorted(kt.items()):
            rel, H, D = shapes[kind]
            b = (edge_bytes_fwd if what == "gat_fwd" else edge_bytes_bwd)(rel, H, D)
            e_bytes += b * per_step
            e_ms += ms * per_step
            edge_rows[f"{what}_{kind}"] = {"avg_launch_us": ms * 1e3, "launches_per_step": per_step,
                                           "bytes_per_launch": b, "frac": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        traffic, traffic_src, traffic_rec = pmc_traffic() if args.config == "cfg2" else (None, None, None)
        items = step_work(rel_w, rel_s, args.n_iter, args.dtype)
        floor_s, edge_floor_s, dense_floor_s, gflop = full_stack_floor(items)
        floor_i, _, dense_floor_i, _ = full_stack_floor(step_work(rel_w, rel_s, args.n_iter, args.dtype, issued=True))
        d_ms, d_flops, d_name = time_dense_kernel(stack, rel_s.n_dst, args.kernel_reps)
        d_tf = d_flops / (d_ms * 1e-3) / 1e12
        rep = {
            "roofline": {"kernel": "hsg_gat_fwd (S2W: sentence->word, H=6 x D=50)", "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": k_bytes,
                         "bytes_formula": "SURVEY 8(d) B_f = 4 n_src (HD+H) + 8 n_dst + 4 + 5 E_T + 4 n_dst (HD+2H)",
                         "epilogue_bytes_per_launch": epilogue_bytes_fwd(rel_s, Hs, Ds),
                         "avg_launch_us": k_ms * 1e3,
                         "timing": f"HIP events recorded by the kernel's own dispatch packet on its stream "
                                   f"(hipExtLaunchKernel) inside {args.kernel_steps} eager training steps "
                                   "(in-step cache state); cross-check: rocprofv3 kernel trace of the same "
                                   "command under profiles/"},
            "edge_aggregate": {"bytes_per_step": e_bytes, "time_us_per_step": e_ms * 1e3,
                               "achieved": e_bytes / (e_ms * 1e-3) / 1e9, "unit": "GB/s",
                               "frac": e_bytes / (e_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernels": edge_rows},
            "full_stack": {"floor_us": floor_s * 1e6, "edge_floor_us": edge_floor_s * 1e6,
                           "dense_floor_us": dense_floor_s * 1e6, "dense_gflop_per_step": gflop,
                           "frac": floor_s / (ms_per_step * 1e-3),
                           "formula": "sum_k max(B_k/8 TB/s, F_k/peak_k) / t_step over the step's edge, head-"
                                      "projection and FFN work (bench.step_work)",
                           "floor_issued_us": floor_i * 1e6, "dense_floor_issued_us": dense_floor_i * 1e6,
                           "frac_issued": floor_i / (ms_per_step * 1e-3),
                           "frac_issued_is": "the same floor with the dense work priced at the rate the path issues "
                                             "it: the fp32-accurate GEMMs as 6 bf16 limb products each at the bf16 "
                                             "MFMA peak (2.5 PF/s), i.e. 417 TF/s fp32-equivalent, the exact-f32 "
                                             "kernels (head projection, narrow FFN) at 157 TF/s"},
            "roofline_dense": dense_roofline(d_name, rel_s.n_dst, d_tf, d_flops, d_ms, args.dtype),
        }
        if traffic_rec is not None:
            rep["roofline"]["traffic_detail"] = {k: traffic_rec[k] for k in ("fetch_bytes", "write_bytes", "launches")
                                                 if k in traffic_rec}
        return rep

    def e2e(self, G):
        dt = time_train_step(G, self.args.config, self.args.n_iter, self.args.e2e_steps, 3, self.dev)
        return {"value": G.number_of_edges() / dt, "unit": "graph-edges/s", "ms_per_step": dt * 1e3,
                "steps": self.args.e2e_steps,
                "what": "whole train.py iteration (HiGraph forward incl. CNN+LSTM sentence encoder, "
                        "cross-entropy, backward, Adam; eager, 1 GPU)"}


def main(backend_cls=HipBench):
    args = parse()
    # stdout carries exactly ONE JSON line (rank 0): anything libraries print there
    # (RCCL's version banner at communicator init, for one) goes to stderr instead
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    be = backend_cls(args, rank, world, local)
    # the data-parallel exchange runs whenever there is more than one rank; at one rank
    # HSG_DP_REHEARSAL=1 runs it anyway over a world-size-1 group (the driver's N-GPU
    # code path -- RCCL communicator, doc-weighted in-place all-reduce captured in the
    # step graph -- exercised on one GPU; tests/test_gpu_rccl.py)
    dp = world > 1 or os.environ.get("HSG_DP_REHEARSAL", "0") == "1"
    backend = None
    if dp:
        import torch.distributed as dist
        backend = os.environ.get("HSG_DIST_BACKEND", "nccl")       # nccl = RCCL over xGMI
        kw = be.dist_kwargs(backend)
        if world > 1:
            dist.init_process_group(backend, **kw)
        else:
            import tempfile
            fd, rdv = tempfile.mkstemp(prefix="hsg_rdv_")
            os.close(fd)
            os.unlink(rdv)
            dist.init_process_group(backend, init_method=f"file://{rdv}", rank=0, world_size=1, **kw)
    be.load()

    docs, G, E_global, frac = make_shard(args.config, rank, world, args.seed)
    E_total = G.number_of_edges()
    stack, step, zero, params = be.build(G, docs)

    def allreduce():
        # the data-parallel exchange: the doc-weighted gradient all-reduce over RCCL.
        # After the backward every gradient is final at once, so there is nothing to
        # overlap with: ONE flat bucket (7 MB at cfg2) pays one collective latency
        # instead of one per 2 MiB bucket (the eager train step overlaps its buckets
        # with the backward instead: parallel.GradientReducer).  The fused stack writes
        # every gradient into one flat buffer (stack._Grads), which is reduced in place:
        # one scale pass + one all-reduce, no concatenation or copy-back -- and no host
        # sync, so on RCCL it is captured into the step's graph
        from hetersumgraph_amd.parallel import allreduce_gradients, flat_gradients, reduce_flat
        flat = flat_gradients(params)
        if flat is not None:
            reduce_flat(flat, scale=frac)
        else:
            allreduce_gradients(params, scale=frac, bucket_bytes=1 << 30)

    # eager warm-up (builds relation caches, allocator pools)
    for _ in range(max(args.warmup, 2)):
        zero()
        step()
        if dp:
            allreduce()                # also the communicator's first collective, before any capture
    be.synchronize()

    use_graph = not args.no_graph and be.graphs
    graph = None
    # RCCL collectives are capturable: the exchange joins the step's graph (one replay
    # = step + exchange); gloo's are not, so a gloo rehearsal runs it eagerly after it
    capture_exchange = dp and backend == "nccl" and os.environ.get("HSG_CAPTURE_EXCHANGE", "1") != "0"
    if use_graph:
        for attempt in ((True, False) if capture_exchange else (False,)):
            try:
                graph = be.capture(step, zero, allreduce, attempt)
                capture_exchange = attempt
                break
            except Exception as exc:  # pragma: no cover - reported on stderr and in the JSON
                print(f"hip graph capture (exchange inside: {attempt}) failed: {exc!r}", file=sys.stderr)
                graph = None
        if graph is None:
            use_graph = capture_exchange = False
    else:
        capture_exchange = False

    def run_one():
        # replay == zero_grad(set_to_none) + forward + backward (+ the captured exchange):
        # the captured backward writes (does not accumulate into) the graph-owned .grad
        # tensors, and the captured all-reduce reduces them in place
        if graph is not None:
            graph.replay()
        else:
            zero()
            step()
        if dp and not capture_exchange:
            allreduce()

    for _ in range(args.warmup):
        run_one()
    if dp:
        import torch.distributed as dist
        dist.barrier()
    be.synchronize()
    # one event after every step on the launching stream: the per-step times give the
    # median (t_step is the median); the contract's value stays the timed
    # region's mean (K steps between barrier + synchronize)
    mark, between = be.events(args.steps + 1)
    t0 = time.perf_counter()
    mark(0)
    for i in range(args.steps):
        run_one()
        mark(i + 1)
    be.synchronize()
    if dp:
        dist.barrier()
    dt = time.perf_counter() - t0
    step_ms = [between(i, i + 1) for i in range(args.steps)]
    med_ms = float(np.median(step_ms))
    if dp:
        t = torch.tensor([dt, med_ms], dtype=torch.float64)
        if backend == "nccl":
            t = t.to(be.dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, med_ms = float(t[0].item()), float(t[1].item())
    ms_per_step = dt / args.steps * 1e3
    value = E_global / (dt / args.steps)
    from hetersumgraph_amd.parallel import flat_gradients
    dp_exchange = ("none (one rank)" if not dp else
                   ("one in-place all-reduce of the flat gradient buffer" if flat_gradients(params) is not None
                    else "bucketed all-reduce (concatenated copies)")
                   + (", captured in the step's HIP graph" if capture_exchange else ", eager after each step")
                   + f" ({backend}, world {world})")
    rep = be.kernel_report(stack, step, zero, ms_per_step)

    out = {
        "metric": "graph-edges/sec through WSWGAT fwd+bwd, CNN/DM-shaped batch; 1/2/4/8 GPU",
        "value": value,
        "unit": "graph-edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "median_ms_per_step": med_ms,
        "value_at_median": E_global / (med_ms * 1e-3),
        "step_timing": "value / ms_per_step: the timed region (K steps between barrier + synchronize) / K; "
                       "median_ms_per_step: median of the K per-step HIP-event intervals of the same steps "
                       "(BASELINE.md t_step), max over ranks",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": be.data,
        "config": {"workload": f"{args.config}: {model_name(args.config)} WSWGAT stack W2S + {args.n_iter}x(S2W, W2S) "
                               f"fwd+bwd, train mode, {workload_shape(args.config)}",
                   "gemm_operands": args.dtype,
                   "bf16_rows": ("S2W edge-layer output x = elu(h) + origin (the wide FFN's input: "
                                 "GEMM A operand, LayerNorm residual, dW1 operand), wide (S2W) FFN hidden H, "
                                 "its output y (LayerNorm input), dY, dH and the edge gate G rows; one RNE "
                                 "rounding each, GEMM operands rounded anyway"
                                 if args.dtype == "bf16" else "none"),
                   "f32_rows": ("LayerNorm outputs (the word / sentence states between applications), edge "
                                "softmax state (sigma, m, l), head projection, narrow (W2S) FFN, LayerNorm "
                                "statistics, parameters and gradients"
                                if args.dtype == "bf16" else "all"),
                   "docs_per_gpu": len(docs), "graph_edges_per_gpu": E_total,
                   "typed_edges_per_direction": be.n_typed,
                   "dropout": args.dropout, "parallelism": f"dp{world}", "dp_exchange": dp_exchange,
                   "hip_graph": bool(use_graph)},
    }
    out.update(rep)
    if world == 1 and not args.no_e2e:
        try:
            out["e2e_train_step"] = be.e2e(G)
        except Exception as exc:  # pragma: no cover - reported in the JSON
            out["e2e_train_step"] = {"error": repr(exc)}
    # the CPU baseline (every GPU count beside the CPU number) on rank 0 only,
    # after the timed region and the kernel timings, on rank 0's own shard -- the same
    # per-GPU workload at every world size; the other ranks wait at a barrier
    if rank == 0 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(docs, args, stack)
        except Exception as exc:  # pragma: no cover
            out["cpu_baseline"] = {"error": repr(exc)}
        if world > 1:
            out["cpu_baseline"]["sample"] = out["cpu_baseline"].get("sample", "") + (
                f"; rank 0's shard of the {world}-rank job, timed on rank 0's host cores after the timed "
                "region while the other ranks waited at a barrier")
    if dp:
        dist.barrier()
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
