"""Full-size leverage sweep: lev/coin_flip.py's investor-1 run,
coin_smart_lev over 1e6 investors x 3e3 steps x 10 leverages (0.1..1.0), on one
MI355X.  Prints one JSON line: investor-steps-leverages per second over the
whole sweep (outcomes resident in HBM), each kernel's HIP-event time, and the
oracle (the reference's sort-per-step algorithm restated in NumPy) timed on a
bounded sample on the host cores."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rlmd_amd import lev  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--investors", type=int, default=1_000_000)
    ap.add_argument("--horizon", type=int, default=3000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kind", default="coin", choices=["coin", "dice", "dice_sh", "gbm", "coin_flip"])
    a = ap.parse_args()
    if a.kind == "coin_flip":
        return coin_flip_main(a)
    if a.kind != "coin":
        return sorted_main(a)
    dev = torch.device("cuda:0")
    inv, hor = a.investors, a.horizon
    g = torch.Generator(device=dev).manual_seed(420)
    ld = (hor + 63) // 64 * 64
    buf = torch.zeros((inv, ld), dtype=torch.uint8, device=dev)
    step = 1 << 17
    for i in range(0, inv, step):  # Bernoulli(0.5) outcomes, generated in slabs
        n = min(step, inv - i)
        buf[i:i + n, :hor] = (torch.rand((n, hor), generator=g, device=dev) < 0.5).to(torch.uint8)
    top = int(inv * 1e-4)
    args = (inv, hor, top, 100.0, 0.5, -0.4, 0.1, 1.0, 0.1)
    lev.coin_smart_lev(dev, (buf, hor), *args)  # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        data, data_T = lev.coin_smart_lev(dev, (buf, hor), *args)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    n_lev = data.shape[0]
    units = inv * hor * n_lev
    out = {"metric": "coin_smart_lev investor-steps-leverages/s", "value": units / (ms / 1e3), "unit": "1/s",
           "ms_per_sweep": ms, "config": {"investors": inv, "horizon": hor, "n_lev": n_lev, "top": top},
           "outcome_bytes": inv * ld, "finite_rows": int(torch.isfinite(data).all(dim=(1, 2)).sum())}
    if not a.no_cpu_baseline:
        from oracle import lev as olev

        o = buf[:20000, :200].cpu().numpy()
        t0 = time.perf_counter()
        olev.coin_smart_lev(o, 2, 100.0, 0.5, -0.4, 0.1, 1.0, 0.1)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 20000 * 200 * 10 / dt, "unit": "1/s", "cores": 1, "kind": "port",
                               "sample": "20000 investors x 200 steps x 10 leverages, sort per step (NumPy)"}
    print(json.dumps(out))


def sorted_main(a):
    """dice_smart_lev / dice_sh_smart_lev / gbm_smart_lev (rlmd_lev_sweep_sorted:
    a device radix sort per (step, leverage)) at the given size, 10 leverages
    (lev/dice_roll.py, dice_roll_sh.py, gbm.py grids 0.1..1.0)."""
    dev = torch.device("cuda:0")
    inv, hor = a.investors, a.horizon
    g = torch.Generator(device=dev).manual_seed(420)
    if a.kind == "gbm":
        o = (0.0540025395205692 - 0.1897916175617430 ** 2 / 2
             + 0.1897916175617430 * torch.randn((inv, hor), generator=g, device=dev))
    else:
        u = torch.rand((inv, hor), generator=g, device=dev)
        o = torch.where(u < 1 / 6, 0.0, torch.where(u < 2 / 6, 1.0, 2.0))
    top = int(inv * 1e-4)
    if a.kind == "dice":
        run = lambda: lev.dice_smart_lev(dev, o, inv, hor, top, 100.0, 0.5, -0.5, 0.05, 0.1, 1.0, 0.1)  # noqa
    elif a.kind == "dice_sh":
        run = lambda: lev.dice_sh_smart_lev(dev, o, inv, hor, top, 100.0, 0.5, -0.5, 0.05, -1.0, 5.0, -1.0,  # noqa
                                            0.1, 1.0, 0.1)
    else:
        run = lambda: lev.gbm_smart_lev(dev, o, inv, hor, top, 100.0, 0.1, 1.0, 0.1)  # noqa
    data, _ = run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        data, data_T = run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    n_lev = data.shape[0]
    out = {"metric": f"{a.kind}_smart_lev investor-steps-leverages/s", "value": inv * hor * n_lev / (ms / 1e3),
           "unit": "1/s", "ms_per_sweep": ms, "ms_per_step": ms / (hor - 1),
           "config": {"investors": inv, "horizon": hor, "n_lev": n_lev, "top": top}}
    if not a.no_cpu_baseline:
        from oracle import lev as olev

        oc = o[:20000, :100].cpu().numpy()
        t0 = time.perf_counter()
        if a.kind == "gbm":
            olev.gbm_smart_lev(oc, 2, 100.0, 0.1, 1.0, 0.1)
        elif a.kind == "dice":
            olev.dice_smart_lev(oc, 2, 100.0, 0.5, -0.5, 0.05, 0.1, 1.0, 0.1)
        else:
            olev.dice_sh_smart_lev(oc, 2, 100.0, 0.5, -0.5, 0.05, -1.0, 5.0, -1.0, 0.1, 1.0, 0.1)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 20000 * 100 * 10 / dt, "unit": "1/s", "cores": 1, "kind": "port",
                               "sample": "20000 investors x 100 steps x 10 leverages, sort per step (NumPy)"}
    print(json.dumps(out))


def coin_flip_main(a):
    """The whole of lev/coin_flip.py's experiment (:154-235) on the device at its
    own size (1e6 investors x 3e3 steps, Bernoulli(0.5), seed-independent
    synthetic outcomes): coin_fixed_final_lev over 20 leverages, coin_smart_lev
    over 10, coin_big_brain_lev for investor 2 (1 configuration) and investor 3
    (19 stop-losses x 6 retention ratios = 114 configurations; the reference's
    own coin_optimal_lev raises TypeError there, see rlmd_amd/lev.py).  Each
    call timed with events; one JSON line."""
    dev = torch.device("cuda:0")
    inv, hor = a.investors, a.horizon
    g = torch.Generator(device=dev).manual_seed(420)
    o = torch.empty((inv, hor), dtype=torch.uint8, device=dev)
    step = 1 << 17
    for i in range(0, inv, step):
        n = min(step, inv - i)
        o[i:i + n] = (torch.rand((n, hor), generator=g, device=dev) < 0.5).to(torch.uint8)
    top = int(inv * 1e-4)
    calls = {
        "coin_fixed_final_lev (20 levs)": lambda: lev.coin_fixed_final_lev(dev, o, top, 100.0, 0.5, -0.4, 0.05, 1.0,
                                                                           0.05),
        "coin_smart_lev (10 levs)": lambda: lev.coin_smart_lev(dev, o, inv, hor, top, 100.0, 0.5, -0.4, 0.1, 1.0, 0.1),
        "coin_big_brain_lev inv2 (1 cfg)": lambda: lev.coin_big_brain_lev(dev, o, inv, hor, top, 100.0, 0.5, -0.4,
                                                                           2.5, 0.1, 0.1, 0.1, 0.0, 0.0, 0.1),
        "coin_big_brain_lev inv3 (114 cfg)": lambda: lev.coin_big_brain_lev(dev, o, inv, hor, top, 100.0, 0.5, -0.4,
                                                                             2.5, 0.05, 0.95, 0.05, 0.7, 0.95, 0.05),
    }
    out = {"metric": "lev/coin_flip.py experiment wall time on one MI355X", "unit": "s",
           "config": {"investors": inv, "horizon": hor, "top": top}, "calls_ms": {}}
    total = 0.0
    for name, fn in calls.items():
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        out["calls_ms"][name] = ms
        total += ms
        first = r[0] if isinstance(r, tuple) else r
        out.setdefault("finite_frac", {})[name] = float(torch.isfinite(first).float().mean().item())
        del r, first
    out["value"] = total / 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
