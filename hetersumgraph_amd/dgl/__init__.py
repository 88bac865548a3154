"""``dgl`` drop-in namespace for the reference's call sites.

``import hetersumgraph_amd; hetersumgraph_amd.install_as_dgl()`` before the
reference's ``import dgl`` (train.py:26, HiGraph.py:26, module/dataloader.py:44)
routes DGLGraph / batch / unbatch / sum_nodes / init.zero_initializer to this
build's graph object, whose relations feed the HIP kernels.
"""
from ..graph import (ALL, BatchedDGLGraph, DGLGraph, batch, mean_nodes, sum_nodes,  # noqa: F401
                     unbatch)
from . import init  # noqa: F401
from . import data  # noqa: F401

__version__ = "0.4-compat"
