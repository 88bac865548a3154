"""The C ABI: libhsg.so builds for gfx950, loads, and exports every symbol that
include/hsg.h declares, with the struct layout the ctypes binding assumes.
(No compute calls here -- those need a GPU and live in the -m gpu tests.)"""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hsg.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hsg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_bound_symbols():
    from hetersumgraph_amd import _lib
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    from hetersumgraph_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libhsg.so is not built (run python -m hetersumgraph_amd.build)")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert _lib.load() is not None
    assert "gfx950" in _lib.version()


def test_struct_layout():
    from hetersumgraph_amd._lib import HsgRel
    # 3 x int32 + pad to 8 + 7 pointers, then the work lists (round 6): 2 x int32 + 2
    # pointers (x86-64 SysV)
    assert ctypes.sizeof(HsgRel) == 16 + 7 * 8 + 8 + 2 * 8
    assert HsgRel.indptr.offset == 16
    assert HsgRel.n_dwork.offset == 72 and HsgRel.dwork.offset == 80 and HsgRel.swork.offset == 88


def test_code_object_is_gfx950():
    from hetersumgraph_amd import _lib
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_host_library_exports_graph_builder():
    """libhsg_host.so (g++, no HIP runtime) exports every symbol include/hsg_graph.h declares."""
    from hetersumgraph_amd import build, datapipe
    build.build_host(verbose=False)
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "hsg_graph.h")).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(hsg_[a-z0-9_]+)\s*\(", src)))
    assert names == ["hsg_graph_count", "hsg_graph_fill"]
    lib = ctypes.CDLL(datapipe.HOST_LIB)
    for name in names:
        assert hasattr(lib, name), name
    assert ctypes.sizeof(datapipe.HsgDocs) == 8 + 12 * 8


def test_host_mirror_of_dw_tiles():
    """bench.dw_tiles (the byte count's host mirror, no HIP call) equals the library's
    hsg_gemm_dw_tiles (a host-only query: no GPU needed) on the FFN shapes and a sweep."""
    import bench
    from hetersumgraph_amd import _lib
    lib = _lib.load()
    shapes = [(300, 512), (512, 300), (64, 512), (512, 64), (4, 4), (160, 128), (161, 129), (1024, 768)]
    shapes += [(m, n) for m in range(4, 700, 36) for n in range(4, 700, 52)]
    for m, n in shapes:
        assert bench.dw_tiles(m, n) == lib.hsg_gemm_dw_tiles(m, n), (m, n)
