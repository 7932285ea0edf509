"""bench.py's N-rank launch path on CPU (`--dry-run`: a host stand-in trainer,
gloo over 127.0.0.1, no HIP library).

`python bench.py --gpus 2` without a launcher goes through spawn_ranks (two
child rank processes with RANK / WORLD_SIZE / MASTER_* set), the per-rank
multi-step n (parse_multi_steps, C5's "one n per GPU"), the barrier-bracketed
timed region (timed_region), the max-over-ranks reduction and all_gather
(whole_job -> reduce_ranks), and rank 0's single JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", *args], capture_output=True,
                       text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


def test_two_ranks_spawned_with_per_rank_multi_steps():
    steps, lanes = 6, 128
    out = _run("--gpus", "2", "--steps", str(steps), "--warmup", "2", "--lanes", str(lanes),
               "--multi-steps", "3,5", "--config", "c5")
    assert out["n_gpus"] == 2
    assert out["config"]["multi_steps_per_rank"] == [3, 5]
    assert out["config"]["global_lanes"] == 2 * lanes
    # value = env steps of every rank / the max-over-ranks wall time
    assert out["value"] == pytest.approx(2 * lanes * steps / out["t_max_s"], rel=1e-12)
    assert out["ms_per_step"] == pytest.approx(1e3 * out["t_max_s"] / steps, rel=1e-12)
    # rank 1's stand-in sleeps 4 ms per step, rank 0's 2 ms: the max is rank 1's
    assert out["t_max_s"] >= steps * 0.004
    assert out["t_max_s"] >= out["rank0_elapsed_s"]


def test_single_rank_default():
    out = _run("--steps", "3", "--warmup", "1", "--lanes", "64")
    assert out["n_gpus"] == 1 and out["config"]["multi_steps_per_rank"] == [1]
    assert out["value"] == pytest.approx(64 * 3 / out["t_max_s"], rel=1e-12)


def test_gpus_world_mismatch_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_seed_processes_protocol():
    """--seed-procs: one child process per seed (SeedProcs / seed_worker), built
    and warmed on "run", started together on "go"; the group's rate is T x
    lanes x n_t over the span from the first start to the last end."""
    lanes = 64
    out = _run("--steps", "3", "--warmup", "1", "--lanes", str(lanes), "--seed-procs", "1,2,3")
    sp = out["seeds_per_gpu_processes"]
    assert sorted(sp) == ["1", "2", "3"]
    for T, r in sp.items():
        assert len(r["per_seed_ms_per_step"]) == int(T)
        assert r["env_steps_per_s"] == pytest.approx(int(T) * lanes * 5 / r["span_s"], rel=1e-12)
        # the seeds overlap: the span is shorter than their own step times end to
        # end (self-calibrated, so a loaded host that slows every step still passes)
        serial = sum(ms * 5 / 1e3 for ms in r["per_seed_ms_per_step"])
        assert r["span_s"] < 0.9 * serial or int(T) == 1
