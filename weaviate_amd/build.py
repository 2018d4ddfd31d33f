"""Build the gfx950 shared library in-tree (weaviate_amd/libwvknn.so).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the CPU
container; the resulting .so travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libwvknn.so")
SOURCES = [
    os.path.join(HERE, "csrc", "runtime.hip"),
    os.path.join(HERE, "csrc", "kernels.hip"),
    os.path.join(HERE, "csrc", "bq_kernels.hip"),
    os.path.join(HERE, "csrc", "pq_kernels.hip"),
    os.path.join(HERE, "csrc", "kernels_bf3.hip"),
    os.path.join(HERE, "csrc", "rq_kernels.hip"),
    os.path.join(HERE, "csrc", "lsm_segment.hip"),
    os.path.join(HERE, "csrc", "batcher.hip"),
    os.path.join(HERE, "csrc", "gemv_kernels.hip"),
    os.path.join(HERE, "csrc", "qs_kernels.hip"),
    os.path.join(HERE, "csrc", "sq_kernels.hip"),
    os.path.join(HERE, "csrc", "wv_device.h"),
    os.path.join(REPO, "include", "wv_knn.h"),
]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",  # exact-order kernels: the only fused ops are explicit fmaf()
    "-fPIC",
    "-shared",
    "-Wno-unused-value",
    "-Wno-unused-result",
]


def needs_rebuild() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES if os.path.exists(s))


def build_library(force: bool = False, verbose: bool = True) -> str:
    if force or needs_rebuild():
        cmd = [HIPCC, *FLAGS, "-I" + os.path.join(REPO, "include"), SOURCES[0], "-o", LIB + ".tmp"]
        if verbose:
            print("[weaviate_amd] " + " ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def build_oracle(verbose: bool = True) -> None:
    """Test infrastructure: oracle/liboracle.so and, when the reference tree is
    present (CPU container only), oracle/_ref/libref.so."""
    odir = os.path.join(REPO, "oracle")
    subprocess.run(["make", "-s", "-C", odir], check=True)
    if os.path.isdir("/root/reference/adapters"):
        subprocess.run(["make", "-s", "-C", odir, "ref"], check=True)


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)
    build_oracle()
