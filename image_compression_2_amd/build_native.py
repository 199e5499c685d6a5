"""Builds libic2ops.so in-tree (hipcc --offload-arch=gfx950), one object per .hip, linked -shared.

    python -m image_compression_2_amd.build_native [--force]

The .so lands next to this file so it travels with the repository snapshot to the GPU box.
Incremental: an object is rebuilt when its source or any header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")
# diagnostic variants build elsewhere (IC2_BUILD_DIR / IC2_LIB_OUT, e.g. with IC2_EXTRA_CFLAGS=-D...) and are loaded
# only under IC2_DEV=1 IC2_DEV_LIB=<path> (_native.py)
BUILD = os.environ.get("IC2_BUILD_DIR", os.path.join(HERE, "_build"))
LIB = os.environ.get("IC2_LIB_OUT", os.path.join(HERE, "libic2ops.so"))
ARCH = os.environ.get("IC2_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", "-Wno-unused-result",
          *os.environ.get("IC2_EXTRA_CFLAGS", "").split()]


def _newer(src_paths, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(p) > t for p in src_paths)


# per-file extras: the MFMA filtered-lrelu consumes every accumulator with VALU, so its MFMAs write VGPRs
# directly instead of AGPRs (saves one v_accvgpr_read per value)
FILE_FLAGS = {"flrelu_mfma.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
              # the backward FIR loops must unroll fully (register-resident taps; no scratch, no LDS promotion)
              "flrelu_bwd.hip": ["-mllvm", "-pragma-unroll-threshold=200000"]}


def _compile(src, headers, force):
    obj = os.path.join(BUILD, os.path.basename(src).replace(".hip", ".o"))
    if force or _newer([src] + headers, obj):
        cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h")))
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, headers, force), srcs))
    if force or _newer(objs, LIB):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print(f"[ic2] built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
