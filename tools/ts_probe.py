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
LIB = os.path.join(OUT, f"librlmd_timing{os.environ.get('RLMD_TS_TAG', '')}.so")


def build():
    from rlmd_amd import build as b

    b.build()
    os.makedirs(OUT, exist_ok=True)
    timed = ("learn.hip", "rows.hip", "act.hip", "env.hip", "update.hip")
    tobjs = []
    for src in timed:
        obj = os.path.join(OUT, src.replace(".hip", "_ts.o"))
        extra = ["-DRLMD_TIMING_WINDOWS"] if "--windows" in sys.argv else []
        extra += ["-DRLMD_TIMING_DRAIN"] if "--drain" in sys.argv else []
        subprocess.check_call([b.HIPCC, *b.FLAGS, *b.PER_FILE.get(src, b.DEFAULT_EXTRA), "-DRLMD_TIMING", *extra, "-c",
                               os.path.join(b.CSRC, src), "-o", obj])
        tobjs.append(obj)
    objs = [os.path.join(b.BUILD, os.path.splitext(s)[0] + ".o") for s in b.SOURCES if s not in timed]
    subprocess.check_call([b.HIPCC, "-shared", f"--offload-arch={b.ARCH}", "-o", LIB, *tobjs, *objs])
    print("built", LIB)


def run():
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    for fn in ("rlmd_debug_ts", "rlmd_debug_ts_rows"):
        getattr(lib, fn).restype = C.c_int
        getattr(lib, fn).argtypes = [C.POINTER(C.c_ulonglong)]
    from rlmd_amd.trainer import VecTrainer

    td3 = "--td3" in sys.argv  # C3: Dice_SH_InvA, TD3 400/300, B = 200
    tr = VecTrainer("dice_sh" if td3 else "gbm", "A", 65536, algo="TD3" if td3 else "SAC", precision="bf16",
                    warmup_steps=0, smoothing_window=0, replay_capacity=1 << 20, k_updates=1, device="cuda:0")
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    rows, rrows = [], []
    buf = (C.c_ulonglong * 64)()
    rbuf = (C.c_ulonglong * 128)()
    for _ in range(30):
        tr.step()
        torch.cuda.synchronize()
        lib.rlmd_debug_ts(buf)
        lib.rlmd_debug_ts_rows(rbuf)
        rows.append(np.array(buf[:16], dtype=np.int64))
        rrows.append(np.array(rbuf[:128], dtype=np.int64))
    a = np.stack(rows)
    d = np.diff(a[:, :13], axis=1)
    med = np.median(d, axis=0)
    print("critic_loss_kernel:")
    for i, v in enumerate(med):
        print(f"  ts{i}->ts{i + 1}: {v:10.0f} cycles")
    print("  total", np.median(a[:, 12] - a[:, 0]))
    r = np.stack(rrows)
    def seq(name, idx):
        print(name + ":")
        for i, j in zip(idx[:-1], idx[1:]):
            print(f"  {i}->{j}: {np.median(r[:, j] - r[:, i]):10.0f} cycles")
        print("  total", np.median(r[:, idx[-1]] - r[:, idx[0]]))
    seq("fwd_rows target job 0", [0, 1, 2, 3, 4, 5])
    seq("fwd_rows job 0 policy MLP (staged -> layer 1 -> barrier -> layer 2 -> epilogue -> barrier -> heads)",
        [2, 6, 7, 8, 9, 10, 3])
    seq("fwd_rows job 0 target critic MLP (sampled -> same phases)", [4, 22, 23, 24, 25, 26, 5])
    seq("fwd_rows critic job 2", [60, 61, 63, 64, 65, 66, 67, 62])
    seq("abwd_rows", [96, 95, 97, 98, 99, 100, 101, 103, 104, 105, 108, 109, 106, 107, 110, 111])
    seq("cbwd_rows (0, 0, 0)", [112, 113, 114, 115, 116, 117, 118])
    seq("fwd_rows actor job 4", [80, 81, 87, 88, 89, 90, 91, 82, 83])
    t0 = r[:, 40:45].min(axis=1)
    print("fwd_rows job windows, block x = 0 (us from the first job start):")
    for y in range(5):
        s0, s1 = np.median(r[:, 40 + y] - t0) / 100, np.median(r[:, 45 + y] - t0) / 100
        print(f"  job {y}: {s0:7.2f} .. {s1:7.2f}  ({s1 - s0:6.2f} us)")


def run_act():
    """Per-workgroup timeline of fused_act_kernel over 65,536 rows (C2 SAC, and
    TD3 400/300 with --td3): block start spread, block spans, phase cycles."""
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts_act.restype = C.c_int
    lib.rlmd_debug_ts_act.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    from rlmd_amd.agent import DeviceAgent

    td3 = "--td3" in sys.argv
    algo, S, A, h1, h2 = ("TD3", 6, 2, 400, 300) if td3 else ("SAC", 5, 1, 256, 256)
    ag = DeviceAgent(algo, S, A, h1, h2, 512, 256, precision="bf16", device="cuda:0")
    n = 65536
    obs = torch.randn(n, S, device="cuda:0") * 1e-3
    out = torch.empty(n, A, device="cuda:0")
    nb = n // 64
    buf = (C.c_ulonglong * (8 * nb))()
    for it in range(5):
        ag.act(obs, mode=0, noise_ctr=it, out=out)
        torch.cuda.synchronize()
    t = np.array(buf[:], dtype=np.int64)
    lib.rlmd_debug_ts_act(buf, nb)
    t = np.array(buf[:], dtype=np.int64).reshape(nb, 8)
    st, en = t[:, 0] - t[:, 0].min(), t[:, 6] - t[:, 0].min()
    print(f"{algo} {h1}/{h2}: {nb} workgroups; realtime ticks (100 MHz = 10 ns)")
    print("  start  pct 0/25/50/75/100:", np.percentile(st, [0, 25, 50, 75, 100]))
    print("  end    pct 0/25/50/75/100:", np.percentile(en, [0, 25, 50, 75, 100]))
    print("  span   pct 0/25/50/75/100:", np.percentile(en - st, [0, 25, 50, 75, 100]))
    ph = np.diff(t[:, 1:6], axis=1)
    for i, name in enumerate(["stage", "layer1", "layer2", "epilogue"]):
        print(f"  {name:9s} cycles median {np.median(ph[:, i]):8.0f}  p90 {np.percentile(ph[:, i], 90):8.0f}")


def run_env():
    """Per-workgroup timeline of env_train_kernel (C2: 65,536 GBM lanes, 256
    blocks): block start spread, spans, block 0's phases (cycles)."""
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts_env.restype = C.c_int
    lib.rlmd_debug_ts_env.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    fused_mode = 0  # per env handle: set on the trainer below
    from rlmd_amd.trainer import VecTrainer

    fam = sys.argv[2] if len(sys.argv) > 2 else "gbm"
    tr = VecTrainer(fam, "A", 65536, algo="SAC", precision="bf16", warmup_steps=0, smoothing_window=0,
                    replay_capacity=1 << 20, k_updates=1, device="cuda:0")
    tr.set_fused(fused_mode)
    nb = 256
    buf = (C.c_ulonglong * (8 * nb))()
    spans, starts, ph = [], [], []
    for it in range(12):
        tr.step()
        torch.cuda.synchronize()
        lib.rlmd_debug_ts_env(buf, nb)
        t = np.array(buf[:], dtype=np.int64).reshape(nb, 8)
        if it < 2:
            continue
        st, en = t[:, 0] - t[:, 0].min(), t[:, 6] - t[:, 0].min()
        starts.append(np.percentile(st, [0, 50, 100]))
        spans.append(np.percentile(en - st, [0, 50, 100]))
        ph.append(np.diff(t[0, 1:6]))
    print("env_train_kernel: 256 blocks, realtime ticks (100 MHz = 10 ns)")
    print("  block start spread pct 0/50/100:", np.median(starts, 0))
    print("  block span         pct 0/50/100:", np.median(spans, 0))
    print("  block-0 phases (cycles) entry->draw, draw->step, step->stores, stores->end:", np.median(ph, 0))


def run_mkt():
    """eval_market_loop_kernel (C4's evaluation event, 100 lanes x 250 days): block
    0's phase cycles on day 10 (day start -> layer 1 -> layer 2 + heads -> action
    -> market step -> end-of-day barrier)."""
    import numpy as np
    import torch

    torch.zeros(1, device="cuda:0")

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts_env.restype = C.c_int
    lib.rlmd_debug_ts_env.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    from rlmd_amd.agent import DeviceAgent
    from rlmd_amd.trainer import market_evaluate

    rng = np.random.default_rng(3)
    prices = 100.0 * np.exp(np.cumsum(0.01 * rng.standard_normal((9167, 1)), axis=0))
    ag = DeviceAgent("SAC", 5, 1, 256, 256, 16, 8, precision="bf16", seed=1, device="cuda:0")
    starts = rng.integers(0, 9167 - 260, size=100)
    buf = (C.c_ulonglong * (8 * 7))()
    ph = []
    for it in range(8):
        market_evaluate(ag, prices, "A", 1, 250, starts, 5000, 10, 100, device="cuda:0")
        lib.rlmd_debug_ts_env(buf, 7)
        t = np.array(buf[:], dtype=np.int64).reshape(7, 8)
        if it >= 2:
            ph.append(np.diff(t[0, 0:6]))
    print("eval_market_loop_kernel block 0, day 10 (cycles): start->L1, L1->L2+heads, ->action, ->step, ->barrier")
    print("  ", np.median(ph, 0), "total", np.median(np.sum(ph, 1)))


def run_upd():
    """critic_update_kernel (C2, K = 1 per step): thread-0 stamps of tile (0, 0),
    tile (0, 1) and the first fc1 block, median cycles between stamps over 30 steps."""
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts_upd.restype = C.c_int
    lib.rlmd_debug_ts_upd.argtypes = [C.POINTER(C.c_ulonglong)]
    from rlmd_amd.trainer import VecTrainer

    algo = sys.argv[2] if len(sys.argv) > 2 else "SAC"
    env, inv = ("gbm", "A") if algo == "SAC" else ("dice_sh", "A")
    tr = VecTrainer(env, inv, 65536, algo=algo, precision="bf16", warmup_steps=0, smoothing_window=0,
                    replay_capacity=1 << 20, k_updates=1, device="cuda:0")
    buf = (C.c_ulonglong * 128)()
    rows = []
    for it in range(40):
        tr.step()
        torch.cuda.synchronize()
        lib.rlmd_debug_ts_upd(buf)
        if it >= 10:
            rows.append(np.array(buf[:], dtype=np.int64).reshape(8, 16))
    r = np.stack(rows)
    names = ["entry", "loads issued", "row loss", "rank + dq", "mfma / fc1 sums", "adam", "first-col extras", "end"]
    t0 = r[:, :6, 14].min(axis=1)
    for slot, label in enumerate(["tile (0,0)", "tile (0,1)", "fc1 block 0", "head wg 0", "critic 2 tile (0,0)",
                                  "last workgroup"]):
        t = r[:, slot]
        w0, w1 = np.median(t[:, 14] - t0) / 100, np.median(t[:, 15] - t0) / 100
        print(f"{label}: total {np.median(t[:, 7] - t[:, 0]):.0f} cycles, window {w0:6.2f} .. {w1:6.2f} us")
        prev = 0
        for i in range(1, 8):
            if np.all(t[:, i] == 0):
                continue
            print(f"  {names[prev]:>16s} -> {names[i]:<16s} {np.median(t[:, i] - t[:, prev]):8.0f}")
            prev = i


def run_aupd():
    """actor_update_kernel (C2, K = 1 per step): thread-0 cycle stamps of tiles (0, 0)
    and (0, 1), fc1 block 0 and the statistics workgroup, and their windows on the
    constant-rate clock (us from the earliest entry)."""
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts_aupd.restype = C.c_int
    lib.rlmd_debug_ts_aupd.argtypes = [C.POINTER(C.c_ulonglong)]
    from rlmd_amd.trainer import VecTrainer

    tr = VecTrainer("gbm", "A", 65536, algo="SAC", precision="bf16", warmup_steps=0, smoothing_window=0,
                    replay_capacity=1 << 20, k_updates=1, device="cuda:0")
    buf = (C.c_ulonglong * 128)()
    rows = []
    for it in range(40):
        tr.step()
        torch.cuda.synchronize()
        lib.rlmd_debug_ts_aupd(buf)
        if it >= 10:
            rows.append(np.array(buf[:], dtype=np.int64).reshape(8, 16))
    r = np.stack(rows)
    names = {0: "entry", 1: "stats branch passed", 2: "loads + rank", 3: "policy bwd / pre-arrive", 4: "arrived",
             5: "mfma / fc1 sums", 6: "adam", 7: "end"}
    t0 = r[:, :6, 14].min(axis=1)
    for slot, label in enumerate(["tile (0,0)", "tile (0,1)", "fc1 block 0", "stats part 0", "head wg 0",
                                  "stats part 1"]):
        t = r[:, slot]
        w0, w1 = np.median(t[:, 14] - t0) / 100, np.median(t[:, 15] - t0) / 100
        print(f"{label}: window {w0:6.2f} .. {w1:6.2f} us")
        prev = 0
        for i in range(1, 8):
            if np.all(t[:, i] == 0):
                continue
            print(f"  {names[prev]:>24s} -> {names[i]:<24s} {np.median(t[:, i] - t[:, prev]):8.0f}")
            prev = i


def run_actenv():
    """act_env_kernel per-workgroup timeline (C3 by default: 65,536 Dice_SH_InvA lanes,
    TD3 400/300; 'gbm' for C2): block spans and the sampling + env epilogue's share."""
    import numpy as np
    import torch

    from rlmd_amd import _abi

    _abi._LIB = _abi.load(LIB)
    lib = _abi._LIB
    lib.rlmd_debug_ts_actenv.restype = C.c_int
    lib.rlmd_debug_ts_actenv.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    fused_mode = 1  # per env handle: set on the trainer below
    from rlmd_amd.trainer import VecTrainer

    fam = sys.argv[2] if len(sys.argv) > 2 else "dice_sh"
    algo = "SAC" if fam == "gbm" else "TD3"
    tr = VecTrainer(fam, "A", 65536, algo=algo, precision="bf16", warmup_steps=0, smoothing_window=0,
                    replay_capacity=1 << 20, k_updates=0, device="cuda:0")
    tr.set_fused(fused_mode)
    nb = 1024
    buf = (C.c_ulonglong * (8 * nb))()
    rows = []
    for it in range(12):
        tr.step()
        torch.cuda.synchronize()
        lib.rlmd_debug_ts_actenv(buf, nb)
        if it >= 2:
            rows.append(np.array(buf[:], dtype=np.int64).reshape(nb, 8))
    r = np.stack(rows)
    t0 = r[:, :, 0].min(axis=1)[:, None]
    st, en, ep = (r[:, :, 0] - t0) / 100, (r[:, :, 6] - t0) / 100, (r[:, :, 7] - t0) / 100
    print(f"act_env_kernel {fam} {algo}: {nb} workgroups (us from the first entry)")
    print("  entry  pct 0/50/100:", np.percentile(st, [0, 50, 100]))
    print("  exit   pct 0/50/100:", np.percentile(en, [0, 50, 100]))
    print("  span   pct 0/50/100:", np.percentile(en - st, [0, 50, 100]))
    print("  epilogue (sampling + env) pct 0/50/100:", np.percentile(en - ep, [0, 50, 100]))
    ph = np.diff(r[:, :, 1:6], axis=2).reshape(-1, 4)
    print("  acting phases (cycles) median:", np.median(ph, 0))


if __name__ == "__main__":
    {"build": build, "run": run, "act": run_act, "env": run_env, "mkt": run_mkt, "upd": run_upd,
     "aupd": run_aupd, "actenv": run_actenv}[sys.argv[1]]()
