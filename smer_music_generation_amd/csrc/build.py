"""Build libsmer_hip.so (gfx950) in-tree with hipcc.

    python -m smer_music_generation_amd.csrc.build      # or build() below

Each .hip/.cpp is compiled to an object under csrc/_build/ (skipped when
up to date) and linked into smer_music_generation_amd/libsmer_hip.so.
The host-only data pipeline loop (dataset.cpp, include/smer_data.h) is built
with g++ into smer_music_generation_amd/libsmer_data.so.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT = os.path.join(PKG, "libsmer_hip.so")
DATA_OUT = os.path.join(PKG, "libsmer_data.so")
OBJ = os.path.join(HERE, "_build")
SOURCES = ["abi.cpp", "gemm.hip", "attention.hip", "norm_embed.hip", "train_ops.hip", "decode_ops.hip"]
HEADERS = ["common.h", os.path.join("..", "..", "include", "smer_hip.h")]
ARCH = os.environ.get("SMER_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libsmer_hip.so)")


# No packed-FP32 VALU instructions (v_pk_fma_f32 / v_pk_mul_f32 /
# v_pk_add_f32) anywhere in the library: on gfx950 their results came out
# wrong in lanes 48-63 (one element of the register pair, a few ulps) while
# a workgroup of another kernel streamed LDS-DMA (global_load_lds) on the
# same CU -- the overlapped train step's LayerNorm backward beside the
# 128x128 weight gradient on the side stream (DESIGN.md section 8,
# tools/ck_log.py).  Without them every configuration repeats bit for bit,
# and the step is faster (the packed ops were an anti-lever beside MFMAs
# anyway).  tests/test_asm_hazards.py scans the built library for them.
NO_PACKED_F32 = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _flags():
    return ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH,
            "-Wno-unused-result", "-I" + os.path.join(ROOT, "include")] + NO_PACKED_F32


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _flags_changed():
    """True (and the stamp rewritten) when the compile flags differ from the
    ones the objects under _build/ were built with."""
    stamp = os.path.join(OBJ, "flags.txt")
    cur = " ".join([_hipcc()] + _flags())
    old = open(stamp).read() if os.path.exists(stamp) else None
    if old != cur:
        with open(stamp, "w") as f:
            f.write(cur)
        return True
    return False


def _compile(src, force=False):
    obj = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    deps = [os.path.join(HERE, src)] + [os.path.join(HERE, h) for h in HEADERS]
    if not force and not _newer(obj, deps):
        return obj
    cmd = [_hipcc()] + _flags() + ["-c", os.path.join(HERE, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (src, " ".join(cmd), r.stderr))
    return obj


def build_data(verbose=True):
    """libsmer_data.so: host C++ only (g++), no ROCm needed."""
    src = os.path.join(HERE, "dataset.cpp")
    hdr = os.path.join(ROOT, "include", "smer_data.h")
    if _newer(DATA_OUT, [src, hdr]):
        cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
        if not cxx:
            raise RuntimeError("no host C++ compiler (g++) for libsmer_data.so")
        cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-I" + os.path.join(ROOT, "include"),
               src, "-o", DATA_OUT]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("g++ failed for dataset.cpp:\n%s\n%s" % (" ".join(cmd), r.stderr))
    if verbose:
        print("built", DATA_OUT)
    return DATA_OUT


def build(verbose=True):
    build_data(verbose)
    os.makedirs(OBJ, exist_ok=True)
    force = _flags_changed()
    jobs = min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda f: _compile(f, force), SOURCES))
    if _newer(OUT, objs):
        cmd = [_hipcc(), "-shared", "-fPIC", "--offload-arch=" + ARCH] + objs + ["-o", OUT]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr))
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build()
    sys.exit(0)
