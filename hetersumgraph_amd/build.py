"""In-tree build of libhsg.so for gfx950 (``python -m hetersumgraph_amd.build``).

hipcc cross-compiles without a GPU; the .so lands next to this file so that it
travels with the repository snapshot to the GPU box.  Each source compiles to its
own object in parallel (no cross-file device symbols, so no -fgpu-rdc), then one
link step.

``--dev`` (or HSG_DEV_BUILD=1) builds ``libhsg_dev.so`` instead, with HSG_DEV
defined (csrc/hsg_dev.h): the A/B switches read the environment and the rejected
variants are compiled in.  The tools load it through ``HSG_LIB_PATH``; the product
``libhsg.so`` carries the default kernels only.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("hsg_gat.hip", "hsg_attn.hip", "hsg_gemm.hip", "hsg_rows.hip", "hsg_hproj.hip", "hsg_relbuild.hip", "hsg_cnn.hip", "hsg_ffn.hip", "hsg_dw.hip")]
OUT = os.path.join(HERE, "libhsg.so")
OBJDIR = os.path.join(ROOT, "build", "obj")
DEV_OUT = os.path.join(HERE, "libhsg_dev.so")
DEV_OBJDIR = os.path.join(ROOT, "build", "obj_dev")
ARCH = os.environ.get("HSG_OFFLOAD_ARCH", "gfx950")
HEADERS = [os.path.join(ROOT, "include", "hsg.h")] + [os.path.join(HERE, "csrc", h) for h in
                                                      ("hsg_rng.h", "hsg_wsplit.h", "hsg_dev.h", "hsg_wave.h")]
# host-only graph builder (no HIP runtime: usable in DataLoader workers)
HOST_SOURCES = [os.path.join(HERE, "csrc", "hsg_graphbuild.cpp")]
HOST_HEADERS = [os.path.join(ROOT, "include", "hsg_graph.h")]
HOST_OUT = os.path.join(HERE, "libhsg_host.so")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build(dev=False):
    out = DEV_OUT if dev else OUT
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in SOURCES + HEADERS)


def _flags(dev=False):
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
            "-I", os.path.join(ROOT, "include")] + (["-DHSG_DEV"] if dev else [])


# per-file extra flags: the narrow-head projection wants plain v_fmac_f32 (SGPR weight
# operand) rather than SLP-packed v_pk_fma_f32, which issues slower on gfx950
FILE_FLAGS = {"hsg_hproj.hip": ["-fno-slp-vectorize"]}


def _obj(src, dev=False):
    return os.path.join(DEV_OBJDIR if dev else OBJDIR, os.path.basename(src).replace(".hip", ".o"))


def _compile(src, force, verbose, dev=False):
    obj = _obj(src, dev)
    if not force and os.path.exists(obj):
        t = os.path.getmtime(obj)
        if os.path.getmtime(src) <= t and all(os.path.getmtime(h) <= t for h in HEADERS):
            return obj
    cmd = [hipcc()] + _flags(dev) + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    return obj


def build_host(force=False, verbose=True):
    """libhsg_host.so with g++ (the native graph builder, include/hsg_graph.h)."""
    if not force and os.path.exists(HOST_OUT):
        t = os.path.getmtime(HOST_OUT)
        if all(os.path.getmtime(s) <= t for s in HOST_SOURCES + HOST_HEADERS):
            return HOST_OUT
    cmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-pthread",
           "-I", os.path.join(ROOT, "include"), "-o", HOST_OUT + ".tmp"] + HOST_SOURCES
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(HOST_OUT + ".tmp", HOST_OUT)
    return HOST_OUT


def build(force=False, verbose=True, dev=None):
    if dev is None:
        dev = os.environ.get("HSG_DEV_BUILD", "0") == "1"
    build_host(force=force, verbose=verbose)
    out = DEV_OUT if dev else OUT
    if not force and not needs_build(dev):
        return out
    os.makedirs(DEV_OBJDIR if dev else OBJDIR, exist_ok=True)
    jobs = min(len(SOURCES), os.cpu_count() or 1, 8)
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, verbose, dev), SOURCES))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, dev=True if "--dev" in sys.argv else None)
