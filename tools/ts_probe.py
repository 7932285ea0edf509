"""Experiment: s_memtime checkpoints inside the loss kernels (RLMD_TIMING build).

Build (here):  python tools/ts_probe.py build
Run (GPU box): python tools/ts_probe.py run
Prints, per checkpoint, the median cycle delta from the previous one over the
timed updates (thread 0 of the one-workgroup kernel).
"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_probe")
LIB = os.path.join(OUT, "librlmd_timing.so")


def build():
    from rlmd_amd import build as b

    b.build()
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "learn_ts.o")
    subprocess.check_call([b.HIPCC, *b.FLAGS, "-DRLMD_TIMING", "-c", os.path.join(b.CSRC, "learn.hip"), "-o", obj])
    objs = [os.path.join(b.BUILD, os.path.splitext(s)[0] + ".o") for s in b.SOURCES if s != "learn.hip"]
    subprocess.check_call([b.HIPCC, "-shared", f"--offload-arch={b.ARCH}", "-o", LIB, obj, *objs])
    print("built", LIB)


def run():
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts.restype = C.c_int
    lib.rlmd_debug_ts.argtypes = [C.POINTER(C.c_ulonglong)]
    from rlmd_amd.trainer import VecTrainer

    tr = VecTrainer("gbm", "A", 65536, algo="SAC", precision="bf16", warmup_steps=0, smoothing_window=0,
                    replay_capacity=1 << 20, k_updates=1, device="cuda:0")
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    rows = []
    buf = (C.c_ulonglong * 64)()
    for _ in range(30):
        tr.step()
        torch.cuda.synchronize()
        lib.rlmd_debug_ts(buf)
        rows.append(np.array(buf[:16], dtype=np.int64))
    a = np.stack(rows)
    d = np.diff(a[:, :13], axis=1)
    med = np.median(d, axis=0)
    for i, v in enumerate(med):
        print(f"ts{i}->ts{i + 1}: {v:10.0f} cycles")
    print("total", np.median(a[:, 12] - a[:, 0]))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
