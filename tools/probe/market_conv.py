"""Market (C4) learning curves at several lane counts / replay sizes: where the
build's leverage goes against the reference's five market_env seeds."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import converge  # noqa: E402

out = open(sys.argv[1], "a")
cases = [(8192, 8, 12000, 1 << 23, 0), (8192, 8, 12000, 1 << 23, 1), (8192, 8, 12000, 1 << 22, 0),
         (1024, 8, 12000, 1 << 20, 0)]
for lanes, k, steps, replay, seed in cases:
    recs = converge.run("market", lanes, k, steps, eval_every=1000, seed=seed, replay=replay, log=lambda s: None)
    for r in recs:
        out.write(json.dumps({k2: r[k2] for k2 in ("lanes", "k", "replay", "step", "updates", "lev",
                                                   "eval_growth_pct", "eval_steps")}) + "\n")
    out.flush()
    print(lanes, k, replay, seed, [(r["updates"], round(r["lev"], 3), round(r["eval_growth_pct"], 2)) for r in recs],
          flush=True)
