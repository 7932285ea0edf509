"""Log files written by the build's host path, for F9 (make_golden.aggregate_fixtures)
and tests/test_logs_cpu.py.  Imports nothing from the reference."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

AGG_INPUTS = {"n_trials": 2, "n_cumsteps": 3000, "eval_freq": 1000, "n_eval": 10, "algo": "SAC", "s_dist": "N",
              "loss_fn": "MSE", "critic_mean_type": "E", "buffer": 1e6, "multi_steps": 1}


def write_build_logs(root):
    """The build's run_experiment (host path) with the deterministic stub trainer of
    tests/stub_trainer.py: Coin_InvA/B/C n=1, the reference's results layout
    (test_agent False).  Shared with tests/test_logs_cpu.py."""
    import functools

    repo = os.path.dirname(os.path.dirname(HERE))
    if repo not in sys.path:
        sys.path.insert(0, repo)
    import importlib.util

    from rlmd_amd.experiment import run_experiment

    # by file path: the reference's own tests/ package shadows this repo's here
    spec = importlib.util.spec_from_file_location("rlmd_stub_trainer", os.path.join(repo, "tests", "stub_trainer.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    StubTrainer = mod.StubTrainer

    paths = []
    for inv, rdim in (("A", 4), ("B", 5), ("C", 6)):
        a = AGG_INPUTS
        path, _ = run_experiment(env="coin", investor=inv, n_trials=a["n_trials"], n_cumsteps=a["n_cumsteps"],
                                 eval_freq=a["eval_freq"], n_eval=a["n_eval"], buffer=int(a["buffer"]), seed=3,
                                 log_every=500, results_root=root, test_agent=False, checkpoint=False,
                                 trainer_factory=functools.partial(StubTrainer, risk_dim=rdim))
        paths.append(path)
    return paths
