"""Run several tools/converge.py configurations in one process (one torch import
on the GPU box) and append every evaluation record as a JSON line.

    python tools/converge_batch.py OUT.jsonl "env=gbm,algo=SAC,k=8,seed=0" "env=dice_sh_a,algo=TD3,k=0" ...
Keys: env, algo, loss, k, seed, lanes, steps, replay, precision, eval_every, warmup, smoothing, ms (n-step
returns), stored (reference | prestep: the replay rows' s), sg (market slice_groups), n_eval.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import converge  # noqa: E402


def parse(spec):
    d = dict(env="gbm", algo="SAC", loss="MSE", k=8, seed=0, lanes=65536, steps=12000, replay=1 << 20,
             precision="bf16", eval_every=250, warmup=1000, smoothing=2000, schedule="updates", ms=1,
             stored="reference", sg=0, n_eval=4096)
    for kv in spec.split(","):
        k, v = kv.split("=")
        d[k] = v if k in ("env", "algo", "loss", "precision", "schedule", "stored") else int(float(v))
    return d


def main():
    out = open(sys.argv[1], "a")
    for spec in sys.argv[2:]:
        d = parse(spec)
        t0 = time.perf_counter()
        recs = converge.run(d["env"], d["lanes"], d["k"], d["steps"], precision=d["precision"],
                            warmup=d["warmup"], smoothing=d["smoothing"], eval_every=d["eval_every"], seed=d["seed"],
                            replay=d["replay"], algo=d["algo"], loss=d["loss"], log=lambda s: None,
                            schedule=d["schedule"], multi_steps=d["ms"], stored_state=d["stored"],
                            slice_groups=d["sg"], n_eval=d["n_eval"])
        for r in recs:
            r["spec"] = spec
            out.write(json.dumps(r) + "\n")
        out.flush()
        third = recs[-max(len(recs) // 3, 1):]
        lev = sum(r["lev"] for r in third) / len(third)
        g = sum(r["eval_growth_pct"] for r in third) / len(third)
        print(f"{spec}: last-third lev {lev:.4f} growth {g:.3f} %/step ({time.perf_counter() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
