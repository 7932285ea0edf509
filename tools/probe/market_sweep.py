"""C4 convergence N-sweep: VecTrainer on Market_InvA_D1 /
stooq_snp at matched learner-update counts, from the reference's single-stream
semantics (N = 1, K = 1: one env step and one update per vector step) up to
C4's own shape (8,192 lanes, K = 8).  Per run the last-third statistics of
tests/test_converge_gpu.py (growth %/step, eval_risk_log column-4 leverage).

    python tools/probe/market_sweep.py OUT.jsonl N:K[:replay[:shared[:fp32]]],... SEEDS [UPDATES]

shared > 0 gives lanes that share market slices in groups (see VecTrainer
market_slice_groups): the one controlled change that separates "many lanes"
from "many price slices per update"."""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import converge  # noqa: E402


def main():
    def beat():  # a line a minute: gpurun takes three silent minutes for a hang
        while True:
            time.sleep(60)
            print("heartbeat", time.strftime("%H:%M:%S"), flush=True)

    threading.Thread(target=beat, daemon=True).start()
    out = open(sys.argv[1], "a")
    cases = []
    for c in sys.argv[2].split(","):
        f = [int(x) for x in c.split(":")]
        cases.append((f[0], f[1], f[2] if len(f) > 2 and f[2] > 0 else 1 << 20, f[3] if len(f) > 3 else 0,
                      "fp32" if len(f) > 4 and f[4] else "bf16"))
    seeds = [int(s) for s in sys.argv[3].split(",")]
    updates = int(sys.argv[4]) if len(sys.argv) > 4 else 96000
    for lanes, k, replay, shared, prec in cases:
        for seed in seeds:
            t0 = time.perf_counter()
            ke = k if k > 0 else 8  # K = 0 (no learning): the C4 schedule's vector steps
            steps = updates // ke
            recs = converge.run("market", lanes, k, steps, eval_every=max(1000 // ke, 1), n_eval=100, seed=seed,
                                replay=replay, log=lambda s: None, slice_groups=shared, precision=prec)
            g = np.array([r["eval_growth_pct"] for r in recs])
            lv = np.array([r["lev"] for r in recs])
            n = len(g)
            sl = slice(n - n // 3, n)
            rec = {"lanes": lanes, "k": k, "replay": replay, "slice_groups": shared, "precision": prec, "seed": seed,
                   "updates": steps * k, "env_steps": steps * lanes, "wall_s": round(time.perf_counter() - t0, 1),
                   "growth_pct": float(g[sl].mean()), "lev": float(lv[sl].mean()),
                   "lev_curve": [round(float(x), 4) for x in lv], "growth_curve": [round(float(x), 4) for x in g]}
            out.write(json.dumps(rec) + "\n")
            out.flush()
            print(lanes, k, replay, shared, prec, seed, rec["wall_s"], round(rec["growth_pct"], 3), round(rec["lev"], 3),
                  flush=True)


if __name__ == "__main__":
    main()
