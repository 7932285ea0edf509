"""Build librlmd_amd.so (gfx950) in-tree with hipcc.

The .so is the product: a C-ABI shared library (include/rlmd_abi.h) loaded by
rlmd_amd/_abi.py with ctypes.  Objects are rebuilt when a source or header is
newer than the object, or when the compile command differs from the one the
object was built with (a per-object flags stamp): an experiment build's flags
never leak into the production library.
"""
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# experiment builds (A/B on one box): RLMD_BUILD_TAG=<tag> RLMD_EXTRA_FLAGS="-D..." writes
# tools/_abh/librlmd_amd_<tag>.so from objects in rlmd_amd/_build_<tag>; load it with RLMD_LIB_PATH
_TAG = os.environ.get("RLMD_BUILD_TAG", "")
EXTRA = os.environ.get("RLMD_EXTRA_FLAGS", "").split()
if EXTRA and not _TAG:
    raise RuntimeError("RLMD_EXTRA_FLAGS needs RLMD_BUILD_TAG: experiment flags never build the production "
                       "library (rlmd_amd/librlmd_amd.so)")
BUILD = os.path.join(HERE, "_build" + (f"_{_TAG}" if _TAG else ""))
LIB = (os.path.join(HERE, "..", "tools", "_abh", f"librlmd_amd_{_TAG}.so") if _TAG
       else os.path.join(HERE, "librlmd_amd.so"))
ARCH = os.environ.get("RLMD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["abi.hip", "env.hip", "replay.hip", "gemm.hip", "learn.hip", "act.hip", "rows.hip", "eval.hip", "shadow.hip", "lev.hip", "lev_sort.hip", "update.hip"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable"]
# env math must round where NumPy rounds (no FMA contraction); GEMM/learner may fuse
# act.hip as env.hip: the two acting kernels (act.hip, env.hip act_env_kernel) share
# rlmd_act_rows.h and must round alike (fused and two-launch steps are bit-equal)
PER_FILE = {"env.hip": ["-ffp-contract=off"], "act.hip": ["-ffp-contract=off"], "eval.hip": ["-ffp-contract=off"], "shadow.hip": ["-ffp-contract=off"],
            "lev_sort.hip": ["-ffp-contract=off"]}
DEFAULT_EXTRA = ["-ffp-contract=fast"]


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [
        os.path.join(HERE, "..", "include", "rlmd_abi.h")]


def _stamp_path(obj):
    return obj + ".flags"


def _stale(obj, src, deps, cmd):
    if not os.path.exists(obj):
        return True
    try:
        with open(_stamp_path(obj)) as f:
            if json.load(f) != cmd:
                return True
    except (OSError, ValueError):
        return True
    deps = deps + [os.path.abspath(__file__)]
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def _compile(src):
    obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
    path = os.path.join(CSRC, src)
    cmd = [HIPCC, *FLAGS, *PER_FILE.get(src, DEFAULT_EXTRA), *EXTRA, "-c", path, "-o", obj]
    if not _stale(obj, path, _headers(), cmd):
        return obj, None
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    with open(_stamp_path(obj), "w") as f:
        json.dump(cmd, f)
    return obj, None


def build(verbose=False, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    jobs = jobs or min(len(SOURCES), max(1, (os.cpu_count() or 4) // 2), 8)
    with ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(_compile, SOURCES))
    errs = [e for _, e in res if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in res]
    if not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
