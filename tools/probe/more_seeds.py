"""More build seeds for the Mann-Whitney convergence checks (tests/test_converge_gpu.py):
the test's run on seeds [lo, hi) for each named workload, records appended to
$RLMD_CONVERGE_LOG, and the Mann-Whitney p of these seeds against the reference's five.

    RLMD_CONVERGE_LOG=gpurun_out/more_seeds.jsonl python tools/probe/more_seeds.py 5 15 dice_sh dice_sh_a_mse
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import numpy as np

    import test_converge_gpu as t

    lo, hi = int(sys.argv[1]), int(sys.argv[2])

    def golden(name):  # the test fixture's loader
        return np.load(os.path.join(ROOT, "tests", "golden", name), allow_pickle=False)

    for w in sys.argv[3:]:
        _, _, seeds = t.build_medians(w, 8, seeds=list(range(lo, hi)))
        pg, pl = t.mw_p(seeds, t.ref_stats(golden, w))
        print(f"{w}: seeds {lo}..{hi - 1} Mann-Whitney p growth {pg:.3f} lev {pl:.3f}", flush=True)
        t.record(w + "_extra", seeds=[lo, hi], p_growth=pg, p_lev=pl, n=len(seeds))


if __name__ == "__main__":
    main()
