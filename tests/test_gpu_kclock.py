"""The in-step kernel clock (hsg_kclock_arm, bench.py's measurement hook) leaves the
edge entry points reentrant (no global mutable state): an armed clock is
consumed only by launches from the arming thread onto the armed stream; other
streams and other threads launch as usual and leave it armed."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def _one_application():
    """A small S2W edge forward (gat_table_fwd) on the current stream."""
    import numpy as np
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.ops import LEAKY_SLOPE, gat_table_fwd
    rng = np.random.default_rng(0)
    d = synth.make_hsg_doc(rng, N=6, W=30, k=5)
    G = hg.batch([synth.to_graph(d, hg.DGLGraph)])
    G.to(torch.device("cuda"))
    rel = G.relation("S2W")
    H, D = 6, 50
    Z = torch.randn(rel.n_src, H * D, device="cuda")
    attn = torch.randn(H, 3 * D, device="cuda")
    T = torch.randn(10, 50, device="cuda")
    wf = torch.randn(H, D, 50, device="cuda")
    bf = torch.randn(H, D, device="cuda")
    org = torch.randn(rel.n_dst, H * D, device="cuda")

    def run():
        return gat_table_fwd(Z, attn, T, wf, bf, org, rel, H, D, LEAKY_SLOPE)[0]
    return run


def test_clock_is_stream_and_thread_bound():
    from hetersumgraph_amd._lib import load
    lib = load()
    run = _one_application()
    ref = run()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    main = torch.cuda.current_stream()
    e0.record(main)
    e1.record(main)
    lib.hsg_kclock_arm(main.cuda_stream, e0.cuda_event, e1.cuda_event)
    try:
        # another stream of this thread: not consumed
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):
            out_side = run()
        assert lib.hsg_kclock_pending() == 3
        # another thread (its own thread-local state): not consumed, and it sees none
        seen = []

        def worker():
            seen.append(lib.hsg_kclock_pending())
            with torch.cuda.stream(side):
                seen.append(run())
        t = threading.Thread(target=worker)
        t.start()
        t.join()
        assert seen[0] == 0
        assert lib.hsg_kclock_pending() == 3
        # the armed stream of this thread: consumed by the forward's single kernel
        out_main = run()
        assert lib.hsg_kclock_pending() == 0
    finally:
        lib.hsg_kclock_arm(None, None, None)
    torch.cuda.synchronize()
    assert e0.elapsed_time(e1) > 0
    for o in (out_side, seen[1], out_main):
        assert torch.equal(o, ref)


def test_clock_disarmed_when_entry_point_raises():
    """An entry point that raises between arming and launching must not leave the
    events armed: the wrapper's error path disarms them."""
    from hetersumgraph_amd import _lib, ops
    with _lib.KernelClock() as clk:
        tok = clk.start(("gat_fwd", "S2W"), torch.device("cuda"))
        assert _lib.load().hsg_kclock_pending() == 3
        ops._clock_abort(tok)
        assert _lib.load().hsg_kclock_pending() == 0
