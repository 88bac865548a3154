"""In-tree build of libhsg.so for gfx950 (``python -m hetersumgraph_amd.build``).

hipcc cross-compiles without a GPU; the .so lands next to this file so that it
travels with the repository snapshot to the GPU box.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("hsg_gat.hip", "hsg_attn.hip", "hsg_gemm.hip", "hsg_rows.hip", "hsg_hproj.hip", "hsg_relbuild.hip")]
OUT = os.path.join(HERE, "libhsg.so")
ARCH = os.environ.get("HSG_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + [os.path.join(ROOT, "include", "hsg.h"), os.path.join(HERE, "csrc", "hsg_rng.h")]
    return any(os.path.getmtime(s) > t for s in deps)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include"), "-o", OUT + ".tmp"] + SOURCES
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
