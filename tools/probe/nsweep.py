"""N-sweep of one convergence workload at matched learner-update counts (as the C4
market sweep): the vectorised path at N lanes and K updates per
vector step for 96,000 updates, per seed the last-third (growth %/step, leverage),
appended to $RLMD_CONVERGE_LOG, then Mann-Whitney against the reference's five.

    RLMD_CONVERGE_LOG=gpurun_out/nsweep.jsonl python tools/probe/nsweep.py dice_sh_a_mse 1:1:0-7 8192:8:0-4
    (--updates=50000 first: another update count than the convergence test's 96,000)
"""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import numpy as np

    import converge
    import test_converge_gpu as t

    w = sys.argv[1]
    env, algo, loss, _, ms, _, _ = t.WORKLOADS[w]
    kw = t.WORKLOAD_KW.get(w, {})
    ref = t.ref_stats(lambda n: np.load(os.path.join(ROOT, "tests", "golden", n), allow_pickle=False), w)
    updates = t.STEPS * 8
    args = sys.argv[2:]
    precision = "bf16"
    while args and args[0].startswith("--"):
        if args[0].startswith("--updates="):  # e.g. the reference's own step count (one update per step)
            updates = int(args[0].split("=")[1])
        elif args[0].startswith("--precision="):
            precision = args[0].split("=")[1]
        args = args[1:]
    for spec in args:
        n, k, sr = spec.split(":")
        n, k = int(n), int(k)
        lo, hi = (int(v) for v in sr.split("-"))
        got = []
        for seed in range(lo, hi + 1):
            recs = converge.run(env, n, k, updates // k, eval_every=max(t.EVAL_EVERY * 8 // k, 1), seed=seed, algo=algo,
                                loss=loss, log=lambda s: None, multi_steps=ms, precision=precision, **kw)
            assert all(math.isfinite(r["eval_growth_pct"]) for r in recs)
            got.append((t._third(recs, "eval_growth_pct"), t._third(recs, "lev")))
            t.record(w + "_nsweep", lanes=n, k=k, seed=seed, updates=updates, precision=precision, growth_pct=got[-1][0],
                     lev=got[-1][1], lev_curve=[round(r["lev"], 3) for r in recs],
                     logtemp_curve=[round(r["log_alpha"], 3) for r in recs])
            print(f"{w} N={n} K={k} seed {seed}: growth {got[-1][0]:.3f} lev {got[-1][1]:.4f}", flush=True)
        pg, pl = t.mw_p(got, ref)
        print(f"{w} N={n} K={k}: Mann-Whitney p growth {pg:.3f} lev {pl:.3f}; lev median {np.median([x for _, x in got]):.3f}",
              flush=True)
        t.record(w + "_nsweep_test", lanes=n, k=k, updates=updates, precision=precision, p_growth=pg, p_lev=pl, n=len(got))


if __name__ == "__main__":
    main()
