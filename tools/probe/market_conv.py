"""Market (C4) learning curves at several lane counts / K: where the build's
leverage goes against the reference's five market_env seeds."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import converge  # noqa: E402

out = open(sys.argv[1], "a")
for lanes, k, steps in [(8192, 8, 12000), (1024, 8, 12000), (256, 8, 12000), (8192, 32, 3000)]:
    recs = converge.run("market", lanes, k, steps, eval_every=1000 if k == 8 else 250, seed=0, log=lambda s: None)
    for r in recs:
        out.write(json.dumps({k2: r[k2] for k2 in ("lanes", "k", "step", "updates", "lev", "eval_growth_pct",
                                                   "eval_steps", "action")}) + "\n")
    out.flush()
    print(lanes, k, [(r["updates"], round(r["lev"], 3), round(r["eval_growth_pct"], 2)) for r in recs], flush=True)
