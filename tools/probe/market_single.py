"""C4's single-stream control (tools/converge.market_single) for a few seeds,
with the last-third statistics of tests/test_converge_gpu.py: separates the
vectorised loop's data regime from the learner."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import converge  # noqa: E402


def main():
    def beat():  # a line a minute: gpurun takes three silent minutes for a hang
        while True:
            time.sleep(60)
            print("heartbeat", time.strftime("%H:%M:%S"), flush=True)

    threading.Thread(target=beat, daemon=True).start()
    out = open(sys.argv[1], "a")
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    for seed in [int(s) for s in (sys.argv[3] if len(sys.argv) > 3 else "0,1,2").split(",")]:
        t0 = time.perf_counter()
        g, lv = converge.market_single(seed, steps)
        n = len(g)
        sl = slice(n - n // 3, n)
        rec = {"seed": seed, "steps": steps, "wall_s": time.perf_counter() - t0, "growth_pct": float(g[sl].mean()),
               "lev": float(lv[sl].mean()), "lev_curve": [float(x) for x in lv]}
        out.write(json.dumps(rec) + "\n")
        out.flush()
        print(seed, round(rec["wall_s"], 1), round(rec["growth_pct"], 3), round(rec["lev"], 3), flush=True)


if __name__ == "__main__":
    main()
