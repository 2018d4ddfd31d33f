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
# translation units compiled in parallel (see csrc/rt_index.h) and linked into one library
UNITS = ["runtime.hip", "qs_runtime.hip", "qs_exact.hip", "qs_replay.hip", "quant_runtime.hip", "multi.hip"]
SOURCES = [os.path.join(HERE, "csrc", f) for f in (
    "runtime.hip", "qs_runtime.hip", "qs_exact.hip", "qs_replay.hip", "quant_runtime.hip", "multi.hip", "rt_index.h", "kernels.hip", "bq_kernels.hip",
    "pq_kernels.hip", "kernels_bf3.hip", "rq_kernels.hip", "lsm_segment.hip", "batcher.hip", "gemv_kernels.hip",
    "qs_kernels.hip", "q8_kernels.hip", "sq_kernels.hip", "vector_index.hip", "wv_device.h", "rq8_mfma.hip", "batch_row.h")] + [os.path.join(REPO, "include", "wv_knn.h")]
OBJDIR = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",  # exact-order kernels: the only fused ops are explicit fmaf()
    "-fPIC",
    "-Wno-unused-value",
    "-Wno-unused-result",
]


def needs_rebuild() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES if os.path.exists(s))


def unit_stale(u: str, obj: str) -> bool:
    """A unit's object is stale when the unit or a shared header (every source
    that is not another unit) is newer."""
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    others = {os.path.join(HERE, "csrc", x) for x in UNITS if x != u}
    return any(os.path.getmtime(s) > t for s in SOURCES if os.path.exists(s) and s not in others)


def build_library(force: bool = False, verbose: bool = True) -> str:
    if force or needs_rebuild():
        os.makedirs(OBJDIR, exist_ok=True)
        procs, objs = [], []
        for u in UNITS:
            obj = os.path.join(OBJDIR, u.replace(".hip", ".o"))
            objs.append(obj)
            if not force and not unit_stale(u, obj):
                continue
            cmd = [HIPCC, *FLAGS, "-I" + os.path.join(REPO, "include"), "-c", os.path.join(HERE, "csrc", u), "-o", obj]
            if verbose:
                print("[weaviate_amd] " + " ".join(cmd), file=sys.stderr)
            procs.append((u, subprocess.Popen(cmd)))
        failed = [u for u, p in procs if p.wait() != 0]
        if failed:
            raise subprocess.CalledProcessError(1, "hipcc " + " ".join(failed))
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", LIB + ".tmp"]
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
