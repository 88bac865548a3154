"""bench.py's secondary end-to-end line: one whole train.py iteration (HSumGraph /
HSumDocGraph forward with the sentence encoder, cross entropy, backward, Adam) runs
on a small synthetic batch and returns a positive step time."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("config", ["cfg2", "cfg4"])
def test_e2e_train_step_runs(config):
    import bench
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    docs = synth.make_batch_docs(config, seed=3, n_docs=3)
    G = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    dev = torch.device("cuda", 0)
    G.to(dev)
    dt = bench.time_train_step(G, config, 2, steps=2, warmup=1, dev=dev)
    assert np.isfinite(dt) and dt > 0
