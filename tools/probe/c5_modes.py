"""More build seeds for C5's bimodal convergence (GBM_InvA, TD3, 5-step returns):
the test's run (tests/test_converge_gpu.py build_medians) on seeds beyond its five,
each seed's last-third (growth %/step, leverage) appended to $RLMD_CONVERGE_LOG,
then the upper-mode count over all seeds run here against the reference's 3 of 5.

    RLMD_CONVERGE_LOG=gpurun_out/c5_modes.jsonl python tools/probe/c5_modes.py 5 20
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import test_converge_gpu as t

    lo, hi = int(sys.argv[1]), int(sys.argv[2])
    _, _, seeds = t.build_medians("gbm_td3_n5", 8, seeds=list(range(lo, hi)))
    n_up = t.c5_upper_count(seeds)
    print(f"C5 upper mode: {n_up} of {len(seeds)} build seeds {lo}..{hi - 1}", flush=True)
    t.record("gbm_td3_n5_extra", seeds=[lo, hi], upper_mode=n_up, n=len(seeds))


if __name__ == "__main__":
    main()
