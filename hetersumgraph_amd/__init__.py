"""hetersumgraph_amd -- MI355X-native WSWGAT hot path of HeterSumGraph.

Public surface (drop-in for the reference's hot path):
  * ``module.GAT.WSWGAT`` / ``HiGraph.HSumGraph`` / ``HiGraph.HSumDocGraph``;
  * ``graph.DGLGraph`` + ``dgl`` namespace (``install_as_dgl``);
  * the C ABI of libhsg.so (include/hsg.h) via ``_lib``.
"""
import sys

__version__ = "0.1.0"


def install_as_dgl():
    """Make ``import dgl`` resolve to this build's DGL-0.4-compatible namespace."""
    from . import dgl as _dgl
    sys.modules["dgl"] = _dgl
    sys.modules["dgl.init"] = _dgl.init
    sys.modules["dgl.data"] = _dgl.data
    sys.modules["dgl.data.utils"] = _dgl.data.utils
    return _dgl
