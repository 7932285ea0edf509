"""Headline benchmark: env steps/s of the vectorised GBM + SAC loop on MI355X.

Workload (BASELINE.json configs[1]): GBM_InvA (n_gambles=1,
S=5, A=1), 65,536 lanes per GPU, SAC 256/256 with bf16 MFMA GEMMs (f32 master
weights / Adam), mini-batch B=512 / top-k 256, on-device replay of 1,048,576
transitions per GPU, K learner updates per vector step (UTD stated in the
output).  One "step" = one fused vector step: policy acting for every lane,
the env step + replay insert + auto-reset kernel, then K learn() updates.
Timing is steady state: the reference's per-lane warm-up (1e3 random-action
steps) and smoothing window (2e3) are start-up phases and are disabled here,
so every timed step runs the (more expensive) policy path.

Multi-GPU (one process per GPU, torchrun): independent seeds per rank, no
data-path collective; one RCCL all_gather of each rank's episode-log slab at
logging time; value = lanes * steps * world / max-over-ranks time ("weak").

Output: ONE JSON line on rank 0 (see the harness contract), with
  roofline      the fused env-step kernel against HBM (live HIP-event timing),
  roofline_mfma the learner (MFMA) phase against the bf16 dense peak,
  cpu_baseline  the CPU oracle port of the same loop on the host cores.
"""
import argparse
import glob
import json
import statistics
import math
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md)


def env_bytes_per_step(S, A, n_assets=0, fused=False):
    """Algorithmic HBM bytes of one lane-step of the env step + replay insert.

    fused (the env step in the acting kernel's epilogue, its marginal cost):
    SURVEY §8(d)'s count, 8A + 12S + 35 = 103 B at C2 — action 4A, f64 wealth
    read + write 16, i32 time read + write 8, obs write 4S, reward 4, two flag
    bytes, and the replay row (2S + A + 1) * 4 + 1.  The observation the row's
    s comes from is read by the acting body, which the marginal excludes.
    separate (env_train_kernel): the same plus the obs read 4S it does itself.
    Market adds the two f64 price gathers per asset (P_t, P_0): 16 n_assets."""
    return 8 * A + 12 * S + 35 + (0 if fused else 4 * S) + 16 * n_assets


def act_flops_per_row(S, A, H1, H2, algo):
    """Policy forward MACs x 2 per acting row (heads: mu + log-scale for SAC)."""
    return 2.0 * (S * H1 + H1 * H2 + (2 if algo == "SAC" else 1) * A * H2)


def sac_update_flops(S, A, H1, H2, B):
    """Dense MLP FLOPs of one SAC update (2 per MAC), as launched:
    target: actor fwd(B) + 2 target-critic fwd(B); critics: 2 fwd + 2 bwd (dW, dX);
    actor: actor fwd + 2 critic fwd + 2 critic bwd-to-input + actor bwd (dW, dX)."""
    X = S + A
    actor_mac = S * H1 + H1 * H2 + 2 * A * H2
    critic_mac = X * H1 + H1 * H2 + H2
    fwd = actor_mac + 2 * critic_mac          # target path
    fwd += 2 * critic_mac                      # critics on (s, a)
    bwd_c = 2 * (critic_mac + H1 * H2 + H2)    # dW (all layers) + dX (layers 2..3) per critic
    fwd += actor_mac + 2 * critic_mac          # actor update forward
    bwd_a = 2 * (H2 + H1 * H2 + H1 * A)        # critics to the action input
    bwd_a += actor_mac + (H1 * H2 + 2 * A * H2)  # actor dW + dX
    return 2.0 * B * (fwd + bwd_c + bwd_a)


def td3_update_flops(S, A, H1, H2, B, actor_every=2):
    """Dense MLP FLOPs of one TD3 update (algo_td3.py:363-531): target actor fwd
    + 2 target-critic fwd; both critics fwd + bwd (dW all layers, dX layers 2..3);
    every `actor_every` updates: actor fwd, critic_1 fwd + bwd to the action,
    actor bwd (dW + dX)."""
    X = S + A
    actor_mac = S * H1 + H1 * H2 + A * H2
    critic_mac = X * H1 + H1 * H2 + H2
    per = actor_mac + 2 * critic_mac + 2 * critic_mac + 2 * (critic_mac + H1 * H2 + H2)
    act = actor_mac + critic_mac + (H2 + H1 * H2 + H1 * A) + actor_mac + H1 * H2 + A * H2
    return 2.0 * B * (per + act / actor_every)


def stooq_snp_prices():
    """tools/market_data/stooq_snp.npy (9167 x 1 S&P 500 daily closes, the C4
    workload of SURVEY §8d) from the committed data fixture
    tests/golden/stooq_snp.npz (tests/golden/make_market_data.py copies it out
    of the reference; the GPU box has no /root/reference)."""
    import numpy as np

    with np.load(os.path.join(ROOT, "tests", "golden", "stooq_snp.npz"), allow_pickle=False) as z:
        return np.ascontiguousarray(z["prices"], dtype=np.float64)


# BASELINE.json configs as single-GPU workloads.  C2 is the
# headline; the others run with --config.  Market (C4): train 1000 / test 250
# days, obs_days 1, shuffle 5 (train) / 3 (eval), gap 5..20 (rl_market.py:54-62).
CONFIGS = {
    "c2": dict(env="gbm", investor="A", n=1, algo="SAC", lanes=65536, replay=1 << 20, multi_steps=1,
               workload="C2: GBM_InvA n_gambles=1 (S=5,A=1), SAC 256/256, replay 1M/GPU"),
    "c3": dict(env="dice_sh", investor="A", n=1, algo="TD3", lanes=65536, replay=1 << 20, multi_steps=1,
               workload="C3: Dice_SH_InvA (key 18, S=6,A=2), TD3 400/300, B=200/k=100, replay 1M/GPU"),
    "c4": dict(env="market", investor="A", n=1, algo="SAC", lanes=8192, replay=1 << 20, multi_steps=1,
               workload="C4: Market_InvA_D1 on stooq_snp (9167 S&P 500 daily closes), "
                        "train 1000 d, shuffle 5, SAC 256/256, 8192 lanes/GPU on one shared slice stream "
                        "(one seed shard per GPU)"),
    "c5": dict(env="gbm", investor="A", n=1, algo="TD3", lanes=65536, replay=1 << 24, multi_steps=5,
               workload="C5: GBM_InvA, TD3 400/300, multi-step n=5 (A), replay 16,777,216 transitions/GPU"),
}


def cpu_baseline(lanes, k_updates, seconds, threads, replay=1 << 20, S=5, A=1, H=256, B=512, topk=256, seed=420):
    """The same loop on the host: CPU oracle (oracle/envs.py + oracle/learn.py,
    the restatement pinned to the reference) — NumPy env over all lanes,
    torch-CPU policy forward, a replay ring of `replay` transitions (the C2
    1,048,576) filled lane-major each vector step, and K torch-CPU SAC updates
    per vector step on B distinct uniform ring rows (replay.py:356-364)."""
    import numpy as np
    import torch

    from oracle import envs as oe
    from oracle import learn as ol
    from rlmd_amd.agent import reference_init

    torch.set_num_threads(threads)
    # the clock starts once the ring holds more than B rows (learn() returns NaN
    # placeholders before that, algo_sac.py:380-396): every timed step updates
    env = oe.OracleVecEnv(oe.GBM, oe.INV_A, lanes, 1, seed=seed)
    init = reference_init("SAC", S, A, H, H, seed=seed)
    lay, n = ol.layout("SAC", S, A, H, H)
    names = {nm: [x[0] for x in lay[nm]] for nm in ("actor", "critic_1", "critic_2")}
    p = ol.flatten({nm: dict(zip(names[nm], [t.numpy() for t in init[nm]])) for nm in names}, lay, n)
    t = ol.flatten({nm: dict(zip(names[nm], [t.numpy() for t in init["target_" + nm]])) for nm in names}, lay, n)
    learner = ol.OracleLearner("SAC", S, A, H, H, B, topk, "MSE", p, t)
    rng = np.random.default_rng(seed)
    obs = env.reset()
    cap = max(replay, lanes)
    ring_s, ring_s2 = np.zeros((cap, S), np.float32), np.zeros((cap, S), np.float32)
    ring_a, ring_r, ring_d = np.zeros((cap, A), np.float32), np.zeros(cap, np.float32), np.zeros(cap, bool)
    mem = 0
    steps, t0 = 0, None
    while True:
        with torch.no_grad():
            Pn = learner.nets(learner.P)
            eps = torch.from_numpy(rng.standard_normal((lanes, A)).astype(np.float32))
            act = learner.policy(Pn["actor"], torch.from_numpy(obs.astype(np.float32)), eps)[0].numpy()
        ns, r, d, _ = env.step(act)
        rows = (mem + np.arange(lanes)) % cap
        ring_s[rows], ring_a[rows], ring_r[rows] = obs, act, r
        ring_s2[rows], ring_d[rows] = ns, d[:, 1]
        mem += lanes
        obs = ns.copy()
        if d[:, 0].any():
            obs[d[:, 0]] = env.reset(d[:, 0])[d[:, 0]]
        filled = min(mem, cap)
        if filled <= B:
            continue
        if t0 is None:
            t0 = time.perf_counter()
        for _ in range(k_updates):
            idx = rng.choice(filled, B, replace=False)
            learner.learn(ring_s[idx], ring_a[idx], ring_r[idx], ring_s2[idx], ring_d[idx],
                          rng.standard_normal((B, A)).astype(np.float32), rng.standard_normal((B, A)).astype(np.float32))
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": lanes * steps / el, "steps": steps, "elapsed_s": el, "unit": "env steps/sec", "cores": threads,
            "kind": "port",
            "sample": f"{steps} vector steps x {lanes} GBM lanes, SAC 256/256 fp32, K={k_updates} updates "
                      f"of B={B} per vector step from a {cap}-row ring (oracle/envs.py + oracle/learn.py on "
                      f"torch-CPU, {threads} thread(s)), {el:.1f} s"}


def cpu_baseline_seeds(lanes, k_updates, seconds, procs, replay=1 << 20):
    """one independent seed per host core — `procs` single-threaded
    worker processes (bench.py --cpu-worker, started as children: they never touch
    the GPU) each run the cpu_baseline loop on their own seed at the full lane count;
    value = all workers' env steps / the longest worker's time."""
    import subprocess

    env = dict(os.environ, OMP_NUM_THREADS="1", MKL_NUM_THREADS="1", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", "--cpu-seconds", str(seconds),
           "--k-updates", str(k_updates), "--lanes", str(lanes), "--replay", str(replay)]
    ps = [subprocess.Popen(cmd + ["--seed", str(420 + i)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           env=env, text=True) for i in range(procs)]
    res = []
    try:
        for i, pr in enumerate(ps):
            try:
                out, err = pr.communicate(timeout=seconds * 4 + 300)
            except subprocess.TimeoutExpired:
                raise RuntimeError(f"cpu baseline worker {i} timed out")
            if pr.returncode != 0:
                tail = "\n".join((err or "").strip().splitlines()[-12:])
                raise RuntimeError(f"cpu baseline worker {i} failed (rc {pr.returncode}):\n{tail}")
            res.append(json.loads(out.strip().splitlines()[-1]))
    finally:  # on any failure, end the workers still running
        for pr in ps:
            if pr.poll() is None:
                pr.kill()
                pr.wait()
    steps = sum(r["steps"] for r in res)
    el = max(r["elapsed_s"] for r in res)
    what = "the reference's loop semantics: 1 env, 1 update per env step" if lanes == 1 and k_updates == 1 else \
        f"{lanes} GBM lanes, K={k_updates} updates of B=512 per vector step"
    return {"value": lanes * steps / el, "unit": "env steps/sec", "cores": procs, "kind": "port",
            "sample": f"{procs} independent seeds, one single-threaded process per host core, each {what}, "
                      f"SAC 256/256 fp32 from a {max(replay, lanes)}-row ring (oracle/envs.py + oracle/learn.py on "
                      f"torch-CPU): {steps} vector steps in total, longest worker {el:.1f} s"}


def load_traffic(kernel, config, lanes):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    written for it (profiles/<round>_pmc_env.json, tools/pmc_summary.py, from
    separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this same bench command).
    kernel: "act_env_marginal" (the fused kernel minus the acting kernel: the env
    step's marginal traffic) or "env_train_kernel" (the separate env kernel).
    Only a summary of the same kernel, config and lane count is used; the newest
    round wins (r03 > r02b > r02a > r02)."""
    best = None
    for path in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_env.json")):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        kid = d.get("kernel_id") or ("act_env_marginal" if d.get("kernel", "").startswith("act_env_kernel")
                                     else "env_train_kernel")
        if kid != kernel or d.get("config", "c2") != config or d.get("lanes") != lanes:
            continue
        tag = os.path.basename(path)[:-len("_pmc_env.json")]
        m = re.match(r"r(\d+)([a-z]*)", tag)
        key = (int(m.group(1)), len(m.group(2)) > 0, m.group(2)) if m else (0, False, tag)
        if best is None or key > best[0]:
            best = (key, d, tag)
    if best is None:
        return None
    return {"hbm_bytes_per_launch": best[1]["hbm_bytes_per_launch"], "source": f"profiles/{best[2]}_pmc_env.json",
            "kernel": best[1].get("kernel")}


def reduce_ranks(elapsed, ep_stats, steps, world, device, extra=()):
    """Logging-time exchange across ranks (the only collective of the run): the
    max-over-ranks wall time, and one all_gather of every rank's log slab
    [episodes, sum final reward, sum length, steps seen, env steps timed,
    *extra] (extra: e.g. the rank's multi-step n).
    RCCL ("nccl") on the GPU box; tests/test_multirank_cpu.py runs it on gloo."""
    import torch
    import torch.distributed as dist

    el_t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    slab = torch.cat([ep_stats.to(device=device, dtype=torch.float64),
                      torch.tensor([steps, *extra], dtype=torch.float64, device=device)])
    if _dist_on():
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
        gathered = [torch.empty_like(slab) for _ in range(world)]
        dist.all_gather(gathered, slab)
        slab_all = torch.stack(gathered)
    else:
        slab_all = slab[None]
    return float(el_t.item()), slab_all


def _dist_on():
    """A process group is up: world > 1, or RLMD_BENCH_FORCE_DIST=1 at world 1
    (the nccl path's rendezvous, barriers, all_reduce and all_gather exercised
    over RCCL on a one-GPU box)."""
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def spawn_ranks(n):
    """`bench.py --gpus N` started without a launcher: start N rank processes
    (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their env) as
    children of this process, which has not touched the GPU, and exit with the
    worst return code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def parse_multi_steps(spec, rank, default):
    """--multi-steps "5" or a per-rank list "3,5,7" (C5: one n per GPU, rank r
    takes entry r mod len)."""
    if spec is None:
        return default
    vals = [int(v) for v in str(spec).split(",") if v.strip()]
    return vals[rank % len(vals)]


def timed_steps(tr, steps, k=None):
    """Mean wall ms per vector step over `steps` steps at K = k (rank-local)."""
    import torch

    for _ in range(3):
        tr.step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(k)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


def timed_region(tr, steps, warmup, world, sync, on_start=None):
    """`warmup` untimed steps, then exactly `steps` timed steps bracketed by a
    barrier + device synchronize on both sides (the harness contract); returns
    this rank's wall seconds."""
    import torch.distributed as dist

    for _ in range(warmup):
        tr.step()
    sync()
    if _dist_on():
        dist.barrier()
    if on_start is not None:
        on_start()
        sync()
        if _dist_on():
            dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    sync()
    if _dist_on():
        dist.barrier()
    return time.perf_counter() - t0


def whole_job(elapsed, tr, lanes, steps, world, device, ms_n):
    """Whole-job value: the env steps every rank timed / the max-over-ranks
    wall time (reduce_ranks, the run's one collective); plus each rank's
    multi-step n as the ranks report it."""
    t_max, slab_all = reduce_ranks(elapsed, tr.flush_stats().double(), float(lanes * steps), world, device,
                                   extra=(float(ms_n),))
    total_steps = float(slab_all[:, 4].sum().item())
    return t_max, total_steps / t_max, [int(v) for v in slab_all[:, 5].tolist()]


class DryTrainer:
    """--dry-run stand-in for VecTrainer (no HIP library, no GPU): a fixed host
    sleep per vector step, longer on higher ranks, so the N-rank plumbing
    (spawn_ranks, rendezvous, per-rank multi-step n, barrier-bracketed timing,
    max-over-ranks, all_gather, the JSON line) runs on CPU over gloo
    (tests/test_bench_cli_cpu.py)."""

    def __init__(self, rank, step_s=0.002):
        self.rank, self.step_s, self.t = rank, step_s, 0

    def step(self, k=None):
        time.sleep(self.step_s * (1 + self.rank))
        self.t += 1

    def flush_stats(self):
        import torch

        return torch.tensor([0.0, 0.0, 0.0, float(self.t)])


def dry_run(args):
    """The N-rank launch path of main() with DryTrainer: gloo on the host,
    rank 0 prints the headline fields it would print for the real loop,
    labelled DRY-RUN (never a measurement)."""
    # the per-seed processes start now, before this process opens the GPU (they
    # wait on stdin until the headline and its companions are done)
    procs_spec = args.seed_procs if args.seed_procs is not None else ("1,2,3,4" if args.config in ("c2", "c4") else "")
    procs_T = [int(v) for v in procs_spec.split(",") if v.strip()]
    seed_procs = None
    if procs_T and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        child = ["--config", args.config, "--k-updates", str(args.k_updates), "--precision", args.precision,
                 "--loss", args.loss, "--warmup", str(args.warmup), "--slice-groups", str(args.slice_groups)]
        if args.lanes:
            child += ["--lanes", str(args.lanes)]
        if args.replay:
            child += ["--replay", str(args.replay)]
        seed_procs = SeedProcs(max(procs_T), child, hw_queues=args.seed_proc_queues)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    cfg = CONFIGS[args.config]
    N = args.lanes or cfg["lanes"]
    ms_n = parse_multi_steps(args.multi_steps, rank, cfg["multi_steps"])
    procs_T = [int(v) for v in (args.seed_procs or "").split(",") if v.strip()]
    sp = SeedProcs(max(procs_T), ["--dry-run", "--warmup", "1"]) if procs_T and world == 1 else None
    tr = DryTrainer(rank)
    elapsed = timed_region(tr, args.steps, args.warmup, world, lambda: None)
    t_max, value, ms_per_rank = whole_job(elapsed, tr, N, args.steps, world, torch.device("cpu"), ms_n)
    per_proc = {}
    if sp is not None:
        per_proc = {str(T): sp.round(T, 5, N) for T in procs_T}
        assert sp.close() == 0
    if rank == 0:
        print(json.dumps({"metric": "DRY-RUN (host stand-in trainer; not a measurement)", "value": value,
                          "unit": "env steps/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1e3 * t_max / args.steps, "t_max_s": t_max,
                          "rank0_elapsed_s": elapsed, "scaling": "weak", "seeds_per_gpu_processes": per_proc,
                          "config": {"config": args.config, "lanes_per_gpu": N, "global_lanes": N * world,
                                     "multi_steps_per_rank": ms_per_rank}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


class SeedProcs:
    """Several seeds per GPU as one PROCESS per seed (§8e "GPU g runs seeds
    {g, g+G, ...}"): each seed process gets its own HIP hardware queues, which
    SeedGroup's streams inside one process share (4 queues per process; two busy
    seeds placed on one queue serialise).  The children are started
    before this process opens the GPU (subprocess children of a process that has
    not initialised HIP) and wait on stdin; each builds its trainer when first
    asked to run.  One round of T seeds: "run" to children 0..T-1 (build or reuse
    the trainer, warm up, synchronize, answer "ready"), then "go" to all of them
    together (n_t timed steps bracketed by synchronize, answer with the
    wall-clock start and end); the group's rate is T x lanes x n_t over the span
    from the first start to the last end."""

    def __init__(self, n, argv, hw_queues=1):
        """hw_queues: GPU_MAX_HW_QUEUES of each seed process (its trainer runs on one
        stream; 1 keeps the processes' queues within what the hardware scheduler
        maps at once)."""
        import subprocess

        self.procs = []
        for i in range(n):
            env = dict(os.environ)
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
                env.pop(k, None)
            if hw_queues:
                env["GPU_MAX_HW_QUEUES"] = str(int(hw_queues))
            self.procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--seed-worker",
                                                "--seed", str(420 + 1000 * (i + 1))] + argv, env=env,
                                               stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1))

    def _ask(self, procs, msg):
        for p in procs:
            p.stdin.write(msg + "\n")
            p.stdin.flush()
        out = []
        for p in procs:
            line = p.stdout.readline()
            if not line:
                raise RuntimeError(f"seed process exited (rc {p.poll()})")
            out.append(json.loads(line))
        return out

    def round(self, T, n_t, lanes):
        ps = self.procs[:T]
        self._ask(ps, f"run {n_t} {T}")
        res = self._ask(ps, "go")
        span = max(r["t1"] for r in res) - min(r["t0"] for r in res)
        return {"env_steps_per_s": T * lanes * n_t / span, "span_s": span,
                "per_seed_ms_per_step": [1e3 * (r["t1"] - r["t0"]) / n_t for r in res]}

    def close(self):
        for p in self.procs:
            try:
                p.stdin.write("exit\n")
                p.stdin.flush()
            except OSError:
                pass
        return max((p.wait() for p in self.procs), key=abs, default=0)


def seed_worker(args):
    """One seed process of SeedProcs: the headline workload's trainer (own lanes,
    replay and learner, seed --seed) driven by stdin commands."""
    tr = None
    n_t = 0
    for line in sys.stdin:
        cmd = line.split()
        if not cmd or cmd[0] == "exit":
            break
        import torch

        sync = (lambda: None) if args.dry_run else torch.cuda.synchronize
        if cmd[0] == "run":
            n_t, T = int(cmd[1]), int(cmd[2]) if len(cmd) > 2 else 1
            if tr is None:
                tr = DryTrainer(0) if args.dry_run else make_trainer(args, torch.device("cuda", 0), args.seed)
            if not args.dry_run:
                # the CU share of one of T seeds (rlmd_agent_set_cu_budget, as SeedGroup
                # gives its seeds): the layer-2 column split stays off where T
                # learners' grids would queue for the same CUs
                from rlmd_amd import _abi

                ncu = torch.cuda.get_device_properties(0).multi_processor_count
                _abi.check(_abi.lib().rlmd_agent_set_cu_budget(tr.agent.h, max(ncu // max(T, 1), 1)))
            for _ in range(max(args.warmup, 3)):
                tr.step()
            sync()
            print(json.dumps({"ready": True}), flush=True)
        elif cmd[0] == "go":
            t0 = time.time()
            for _ in range(n_t):
                tr.step()
            sync()
            print(json.dumps({"t0": t0, "t1": time.time()}), flush=True)
    return 0


def make_trainer(args, dev, seed, **over):
    """The configuration's trainer as the headline builds it (steady state:
    warm-up and smoothing off)."""
    from rlmd_amd.trainer import VecTrainer

    cfg = CONFIGS[args.config]
    N = args.lanes or cfg["lanes"]
    replay = args.replay or cfg["replay"]
    ms_n = over.pop("multi_steps", cfg["multi_steps"])
    if ms_n > 1:
        replay = (replay // N) * N
    kw = market_kwargs(args.slice_groups) if cfg["env"] == "market" else {}
    kw.update(over)
    return VecTrainer(env=cfg["env"], investor=cfg["investor"], n_lanes=N, n_gambles=cfg["n"], algo=cfg["algo"],
                      loss=args.loss, k_updates=args.k_updates, replay_capacity=replay, seed=seed, warmup_steps=0,
                      smoothing_window=0, precision=args.precision, device=dev, init_seed=seed, multi_steps=ms_n,
                      dynamics="A", **kw)


def market_kwargs(slice_groups=1):
    """C4's market env: stooq_snp, train 1000 d (obs_days 1), shuffle 5, the
    start draw excluding train + test + gap days (rl_market.py:54-62).  The lanes
    trade one shared shuffled slice stream (slice_groups = 1): the reference's
    single-stream data regime (one time_slice + shuffle_data per episode,
    rl_market.py:202-214), vectorised over the lanes' policy noise.  Independent
    slices per lane (0) learn a leverage outside the reference's."""
    return dict(prices=stooq_snp_prices(), obs_days=1, time_length=1000, shuffle_days=5,
                sample_days=1000 + 250 + 1 + 20 - 1, slice_groups=slice_groups)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--lanes", type=int, default=None)
    ap.add_argument("--k-updates", type=int, default=8)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--replay", type=int, default=None)
    ap.add_argument("--loss", default="MSE", help="critic loss (C3 sweeps MSE/HUB/MAE/HSC)")
    ap.add_argument("--multi-steps", default=None, help="n-step returns; a comma list gives one n per rank (C5)")
    ap.add_argument("--k-sweep", default="1,8,32,64",
                    help="K values timed after the headline region (env steps/s and updates/s each); '' = off")
    ap.add_argument("--no-companion", action="store_true", help="skip the fp32 companion measurement")
    ap.add_argument("--seeds-per-gpu", default=None,
                    help="independent seeds per GPU timed after the headline (SeedGroup: one stream per seed); "
                         "default '2,3,4' (C2, C4), '2,4' otherwise; '' = off")
    ap.add_argument("--seed-streams", default="cu,pool",
                    help="SeedGroup stream kind(s) for --seeds-per-gpu, comma list: pool (torch's stream pool), "
                         "hip (library streams), cu (CU-masked streams: a hardware queue each), cu_split "
                         "(CU-masked, a 1/T interleaved CU share each); the first is the reported seeds_per_gpu")
    ap.add_argument("--seed-procs", default=None,
                    help="independent seeds per GPU as one process each (own HIP queues), timed after the headline; "
                         "default '1,2,3,4' (C2, C4), '' otherwise; '' = off")
    ap.add_argument("--seed-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--seed-proc-queues", type=int, default=1,
                    help="GPU_MAX_HW_QUEUES of each --seed-procs process (0: inherit)")
    ap.add_argument("--slice-groups", type=int, default=1,
                    help="C4: lanes l, l' with l %% G == l' %% G trade the same shuffled slices; 1 (default) = one "
                         "shared stream, the reference's data regime; 0 = every lane its own")
    ap.add_argument("--variants", default=None,
                    help="BASELINE config variants timed after the headline, one trainer each: C3 the critic losses "
                         "(default 'MSE,HUB,MAE,HSC'), C5 the multi-step n (default '3,5,7'); '' = off")
    ap.add_argument("--eval-every", type=int, default=1000,
                    help="vector steps between evaluations (eval_freq 1e3, main.py); amortised into value")
    ap.add_argument("--event-stride", type=int, default=5,
                    help="time every n-th env-kernel dispatch of the timed region with attached HIP events (each "
                         "attached pair costs the stream ~11 us at C2: stamping every step would tax the headline)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="the N-rank launch path with a host stand-in trainer (gloo, no GPU): plumbing test only")
    ap.add_argument("--cpu-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--seed", type=int, default=420, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_worker:  # one seed of the per-core CPU baseline (never imports the GPU library)
        r = cpu_baseline(args.lanes or 65536, args.k_updates, args.cpu_seconds, 1, replay=args.replay or (1 << 20),
                         seed=args.seed)
        print(json.dumps(r), flush=True)
        return 0

    if args.seed_worker:
        return seed_worker(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if args.dry_run:
        return dry_run(args)
    # the CPU baseline runs first, before this process opens the GPU: its worker
    # processes import torch, and the box counts every process holding the device
    cpu_lines = None
    if not args.no_cpu_baseline and int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.config == "c2":
        cfg0 = CONFIGS[args.config]
        n0, rep0 = args.lanes or cfg0["lanes"], args.replay or cfg0["replay"]
        allc = min(16, os.cpu_count() or 1)  # this GPU's host-core share on the box
        # both worker pools first: the in-process runs import torch, which opens the
        # device, and the box allows 16 processes on it (the pool's 16 + this one)
        pool = cpu_baseline_seeds(n0, args.k_updates, args.cpu_seconds, allc, replay=rep0)
        # BASELINE.md's plan: the reference's own loop semantics (one env, UTD = 1,
        # single stream), one seed per core and on one core
        pool1 = cpu_baseline_seeds(1, 1, args.cpu_seconds, allc, replay=rep0)
        cpu_lines = (pool, cpu_baseline(n0, args.k_updates, args.cpu_seconds, 1, replay=rep0), pool1,
                     cpu_baseline(1, 1, args.cpu_seconds, 1, replay=rep0))

    # the per-seed processes start now, before this process opens the GPU (they
    # wait on stdin until the headline and its companions are done)
    procs_spec = args.seed_procs if args.seed_procs is not None else ("1,2,3,4" if args.config in ("c2", "c4") else "")
    procs_T = [int(v) for v in procs_spec.split(",") if v.strip()]
    seed_procs = None
    if procs_T and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        child = ["--config", args.config, "--k-updates", str(args.k_updates), "--precision", args.precision,
                 "--loss", args.loss, "--warmup", str(args.warmup), "--slice-groups", str(args.slice_groups)]
        if args.lanes:
            child += ["--lanes", str(args.lanes)]
        if args.replay:
            child += ["--replay", str(args.replay)]
        seed_procs = SeedProcs(max(procs_T), child, hw_queues=args.seed_proc_queues)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # more ranks than GPUs (a rehearsal of the N-rank path on a smaller box): the
    # ranks share the GPUs round-robin and exchange over gloo on the host; the
    # line says so ("rehearsal"), it is never a scaling measurement
    ndev = torch.cuda.device_count()
    shared = world > 1 and ndev < world
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    force_dist = os.environ.get("RLMD_BENCH_FORCE_DIST") == "1"
    if world > 1 or force_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from rlmd_amd import _abi
    from rlmd_amd.trainer import VecTrainer
    import ctypes as C

    cfg = CONFIGS[args.config]
    N, K = args.lanes or cfg["lanes"], args.k_updates
    replay = args.replay or cfg["replay"]
    ms_n = parse_multi_steps(args.multi_steps, rank, cfg["multi_steps"])
    kw = {}
    if cfg["env"] == "market":
        kw = market_kwargs(args.slice_groups)
    if ms_n > 1:
        replay = (replay // N) * N  # per-lane rings: capacity a multiple of the lanes
    tr = VecTrainer(env=cfg["env"], investor=cfg["investor"], n_lanes=N, n_gambles=cfg["n"], algo=cfg["algo"],
                    loss=args.loss, k_updates=K, replay_capacity=replay, seed=420 + rank, warmup_steps=0,
                    smoothing_window=0, precision=args.precision, device=dev, init_seed=420 + rank,
                    multi_steps=ms_n, dynamics="A", **kw)
    # inside the timed region only the events attached to the env kernel's own
    # dispatch are recorded (profile mode 2), on every event_stride-th step: the
    # phase markers around acting and learning cost the stream ~25 us per C2 step
    # (5 %) and an attached pair ~11 us (2.4 %), so the phase times come from a
    # separate pass after the headline and the live kernel timing samples the region
    def _prof_on():
        tr.profile(2)
        tr.profile_stride(max(args.event_stride, 1))

    elapsed = timed_region(tr, args.steps, args.warmup, world, torch.cuda.synchronize, on_start=_prof_on)
    # medians of the sampled launches: a mean of 10 attached-event samples moved by
    # one slow dispatch (another tenant's work on the box, a late event) by 10 %+
    env_s = tr.profile_samples(1)
    env_ms = statistics.median(env_s) if env_s else 0.0
    env_mean_ms = statistics.mean(env_s) if env_s else 0.0
    env_samples = len(env_s)
    tr.profile_stride(1)
    tr.profile(1)  # the phase pass (untimed)
    for _ in range(10):
        tr.step()
    ms, cnt = tr.profile_read()
    tr.profile(0)
    learn_ms = ms[2] / max(cnt[2], 1)
    act_ms = ms[0] / max(cnt[0], 1)
    fused = tr.last_fused()
    # evaluation (eval_multiplicative / eval_market, 100 episodes) every eval_every
    # vector steps, timed on its own and amortised into the timed region
    ev = (lambda: tr.evaluate_market(n_eval=100, test_days=250)) if cfg["env"] == "market" else \
        (lambda: tr.evaluate(n_eval=100, max_steps=100))
    ev()
    torch.cuda.synchronize()
    te = time.perf_counter()
    ev()
    torch.cuda.synchronize()
    eval_s = time.perf_counter() - te
    if args.eval_every > 0:
        elapsed += eval_s * args.steps / args.eval_every
    t_max, value, ms_per_rank = whole_job(elapsed, tr, N, args.steps, world,
                                          torch.device("cpu") if shared else dev, ms_n)

    # after the headline region (rank-local, no collective): K sweep at the same
    # lanes, and the fp32 companion (the reference's arithmetic) at the headline K
    sweep = {}
    for kk in [int(v) for v in args.k_sweep.split(",") if v.strip()]:
        ms_k = timed_steps(tr, max(5, min(args.steps, 20)), kk)
        sweep[str(kk)] = {"ms_per_step": ms_k, "env_steps_per_s": N * 1e3 / ms_k,
                          "updates_per_s": kk * 1e3 / ms_k, "utd_updates_per_env_step": kk / N}
    tr.step(K)
    # several independent seeds per GPU (§8e "GPU g runs seeds {g, g+G, ...}"):
    # T whole trainers on T streams, the per-GPU throughput of a trial sweep
    seeds_spec = args.seeds_per_gpu if args.seeds_per_gpu is not None else ("2,3,4" if args.config in ("c2", "c4") else "2,4")
    per_mode = {}
    stream_modes = [m.strip() for m in args.seed_streams.split(",") if m.strip()]
    if world == 1:
        from rlmd_amd.trainer import SeedGroup

        for mode, T in [(m, int(v)) for m in stream_modes for v in seeds_spec.split(",") if v.strip()]:
            grp = SeedGroup([420 + 1000 * i for i in range(T)], device=dev, env=cfg["env"], investor=cfg["investor"],
                            n_lanes=N, n_gambles=cfg["n"], algo=cfg["algo"], loss=args.loss, k_updates=K,
                            replay_capacity=replay, warmup_steps=0, smoothing_window=0, precision=args.precision,
                            multi_steps=ms_n, dynamics="A", streams=mode, **kw)
            for _ in range(5):
                grp.step()
            grp.synchronize()
            n_t = max(10, min(args.steps, 30))
            t0 = time.perf_counter()
            for _ in range(n_t):
                grp.step()
            grp.synchronize()
            dt = time.perf_counter() - t0
            per_mode.setdefault(mode, {})[str(T)] = {
                "env_steps_per_s": T * N * n_t / dt, "updates_per_s": T * K * n_t / dt,
                "ms_per_group_step": 1e3 * dt / n_t,
                "vs_one_seed": (T * N * n_t / dt) / (N * 1e3 / (1e3 * t_max / args.steps))}
            del grp
    per_proc = {}
    if seed_procs is not None:
        one = N * 1e3 / (1e3 * t_max / args.steps)
        for T in procs_T:
            r = seed_procs.round(T, max(10, min(args.steps, 30)), N)
            per_proc[str(T)] = dict(r, vs_one_seed=r["env_steps_per_s"] / one)
        seed_procs.close()
    # BASELINE.json names variants of C3 (critic-loss sweep MSE/HUB/MAE/HSC,
    # tools/critic_loss.py:143-205) and C5 (n = 3/5/7, tools/replay.py:251-332):
    # each is timed as its own trainer (same lanes, K, ring), with its learn
    # phase's MFMA fraction from a phase pass
    variants = {}
    if world == 1 and args.config in ("c3", "c5"):
        spec = args.variants if args.variants is not None else ("MSE,HUB,MAE,HSC" if args.config == "c3" else "3,5,7")
        for v in [x.strip() for x in spec.split(",") if x.strip()]:
            loss_v, ms_v = (v.upper(), ms_n) if args.config == "c3" else (args.loss, int(v))
            rep_v = (replay // N) * N if ms_v > 1 else replay
            trv = VecTrainer(env=cfg["env"], investor=cfg["investor"], n_lanes=N, n_gambles=cfg["n"], algo=cfg["algo"],
                             loss=loss_v, k_updates=K, replay_capacity=rep_v, seed=430 + len(variants), warmup_steps=0,
                             smoothing_window=0, precision=args.precision, device=dev, init_seed=430 + len(variants),
                             multi_steps=ms_v, dynamics="A", **kw)
            for _ in range(args.warmup):
                trv.step()
            ms_v_step = timed_steps(trv, max(10, min(args.steps, 30)))
            trv.profile(1)
            for _ in range(10):
                trv.step()
            pms, pcnt = trv.profile_read()
            trv.profile(0)
            lms = pms[2] / max(pcnt[2], 1)
            upd_v = sac_update_flops if cfg["algo"] == "SAC" else td3_update_flops
            fl = K * upd_v(trv.env.state_dim, trv.env.action_dim, trv.agent.h1, trv.agent.h2, trv.batch)
            variants[v] = {"critic_loss": loss_v, "multi_steps": ms_v, "env_steps_per_s": N * 1e3 / ms_v_step,
                           "ms_per_step": ms_v_step, "learn_ms_per_step": lms,
                           "learn_mfma_frac": fl / (lms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS if lms > 0 else None}
            del trv
    companion = None
    if not args.no_companion and world == 1 and args.precision == "bf16":
        tr32 = VecTrainer(env=cfg["env"], investor=cfg["investor"], n_lanes=N, n_gambles=cfg["n"],
                          algo=cfg["algo"], loss=args.loss, k_updates=K, replay_capacity=replay, seed=421,
                          warmup_steps=0, smoothing_window=0, precision="fp32", device=dev, init_seed=421,
                          multi_steps=ms_n, dynamics="A", **kw)
        for _ in range(args.warmup):
            tr32.step()
        ms32 = timed_steps(tr32, args.steps)
        companion = {"dtype": "fp32", "value": N * 1e3 / ms32, "unit": "env steps/sec", "ms_per_step": ms32,
                     "k_updates_per_vector_step": K, "note": "same workload, fp32 GEMM operands (exact-f32 MFMA); "
                                                            "eval not amortised"}
        del tr32

    S, A = tr.env.state_dim, tr.env.action_dim
    n_assets = cfg["n"] if cfg["env"] == "market" else 0
    pmc = load_traffic("act_env_marginal" if fused else "env_train_kernel", args.config, N)
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    H1, H2 = tr.agent.h1, tr.agent.h2
    lib = _abi.lib()
    if fused:
        # the env step lives in the acting kernel's epilogue: its cost is the fused
        # kernel minus the standalone acting kernel on the same rows (both timed by
        # events attached to the kernels' own dispatches), and, for comparison, the
        # separate env kernel of unfused steps
        fused_ms = env_ms
        tr.profile(1)
        for i in range(20):  # 65,536-row launches back to back (reported beside, not used)
            tr.agent.act(tr.obs, mode=0, noise_ctr=1_000_000 + i, out=tr.actions)
        b2b = tr.profile_samples(0)
        act_b2b_ms = statistics.median(b2b) if b2b else 0.0
        # the acting-only reference inside whole train steps (unfused: acting kernel,
        # env kernel, K updates), events attached to both kernels' own dispatches:
        # the acting kernel then starts from the cache state act_env_kernel sees
        # (after the previous step's updates), which back-to-back launches do not
        tr.set_fused(0)
        tr.profile(3)
        for _ in range(20):
            tr.step()
        a_s, e_s = tr.profile_samples(0), tr.profile_samples(1)
        tr.profile(0)
        tr.set_fused(1)
        act_only_ms = statistics.median(a_s) if a_s else 0.0
        act_samples = len(a_s)
        sep_env_ms = statistics.median(e_s) if e_s else 0.0
        env_bytes = env_bytes_per_step(S, A, n_assets, fused=True) * N
        marginal_ms = max(fused_ms - act_only_ms, 1e-6)
        achieved = env_bytes / (marginal_ms * 1e-3) / 1e9
        sep_bytes = env_bytes_per_step(S, A, n_assets) * N
        act_fl = act_flops_per_row(S, A, H1, H2, cfg["algo"]) * N
        roofline = {"kernel": "act_env_kernel: env step + replay insert + auto-reset in the acting kernel's epilogue",
                    "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": pmc and pmc["source"],
                    "algorithmic_bytes_per_launch": env_bytes, "avg_launch_ms": marginal_ms,
                    "timing": f"marginal: act_env_kernel (kernel-attached HIP events on every {args.event_stride}-th "
                              f"step of the timed region: median of {env_samples} launches) minus the acting-only kernel "
                              f"on the same rows inside whole unfused train steps (kernel-attached events, median of {act_samples} "
                              "launches after the timed region)",
                    "fused_kernel_ms": fused_ms, "fused_kernel_mean_ms": env_mean_ms, "act_only_kernel_ms": act_only_ms,
                    "act_only_back_to_back_ms": act_b2b_ms,
                    "separate_env_kernel": {"avg_launch_ms": sep_env_ms, "algorithmic_bytes_per_launch": sep_bytes,
                                            "achieved": sep_bytes / (sep_env_ms * 1e-3) / 1e9,
                                            "frac": sep_bytes / (sep_env_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                            "note": "env_train_kernel of the same unfused steps (RLMD_NO_FUSED_ENV "
                                                    "path), 20 steps after the timed region"}}
        roofline_fused = {"kernel": "act_env_kernel (whole kernel)", "bound": "mfma",
                          "achieved": act_fl / (fused_ms * 1e-3) / 1e12, "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": act_fl / (fused_ms * 1e-3) / 1e12 / BF16_PEAK_TFLOPS, "avg_launch_ms": fused_ms,
                          "algorithmic_flops_per_launch": act_fl,
                          "hbm_GBs": (env_bytes + 0.0) / (fused_ms * 1e-3) / 1e9}
    else:
        env_bytes = env_bytes_per_step(S, A, n_assets) * N
        achieved = env_bytes / (env_ms * 1e-3) / 1e9
        roofline = {"kernel": "env_train_kernel (fused env step + replay insert + reset)",
                    "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": pmc and pmc["source"],
                    "algorithmic_bytes_per_launch": env_bytes, "avg_launch_ms": env_ms,
                    "timing": f"HIP events attached to every {args.event_stride}-th env_train_kernel dispatch of the "
                              f"timed region ({env_samples} launches; hipExtLaunchKernelGGL start/stop: the "
                              "dispatch's own begin/end)"}
        roofline_fused = None
    upd = sac_update_flops if cfg["algo"] == "SAC" else td3_update_flops
    flops = K * upd(S, A, H1, H2, tr.batch)
    mfma_tf = flops / (learn_ms * 1e-3) / 1e12 if learn_ms > 0 else None

    if rank == 0:
        out = {
            "metric": "env steps/sec (whole node), 64k-parallel GBM+SAC at 1/2/4/8 MI355X",
            "value": value, "unit": "env steps/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * t_max / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "real: stooq_snp daily closes" if cfg["env"] == "market" else "synthetic",
            "config": {"workload": cfg["workload"], "config": args.config, "critic_loss": args.loss,
                       "replay_per_gpu": replay, "multi_steps": ms_n, "multi_steps_per_rank": ms_per_rank,
                       "eval_ms_per_event": 1e3 * eval_s, "eval_every_vector_steps": args.eval_every,
                       "lanes_per_gpu": N, "global_lanes": N * world, "k_updates_per_vector_step": K,
                       "mini_batch": tr.batch, "topk": tr.topk, "utd_updates_per_env_step": K / N,
                       "parallelism": f"independent seeds x{world} (no data-path collective)"
                                      + (f"; REHEARSAL: {world} ranks sharing {ndev} GPU(s) over gloo" if shared else ""),
                       "fused_act_env": fused,
                       "phase_ms_per_step": {"act": act_ms, "env_kernel": env_ms, "learn_k": learn_ms}},
            "updates_per_s": K * args.steps * world / t_max,
            "seeds_per_gpu": {"note": "T independent seeds of this workload on one GPU (SeedGroup: own lanes, "
                                      "replay and learner per seed, one HIP stream each), per-GPU totals; eval not "
                                      "amortised", "streams": stream_modes[0], **per_mode[stream_modes[0]],
                              "other_streams": {m: per_mode[m] for m in stream_modes[1:]} or None}
            if per_mode else None,
            "seeds_per_gpu_processes": {"note": "T independent seeds of this workload on one GPU, one process each "
                                                "(own HIP hardware queues; the process-per-seed alternative to "
                                                "SeedGroup's streams); per-GPU totals over the span from the first "
                                                "seed's start to the last one's end; vs_one_seed against the "
                                                "headline's one seed; eval not amortised", **per_proc}
            if per_proc else None,
            "k_sweep": sweep,
            "variants": {"note": "BASELINE.json's variants of this config, each its own trainer (same lanes, K, "
                                 "ring), timed after the headline; eval not amortised", **variants} if variants else None,
            "fp32_companion": companion,
            "roofline": roofline,
            "roofline_fused_kernel": roofline_fused,
            "roofline_mfma": {"kernel": f"learn phase (K {cfg['algo']} updates, all kernels)", "bound": "mfma",
                              "achieved": mfma_tf, "peak": BF16_PEAK_TFLOPS if args.precision == "bf16" else 157.3,
                              "unit": "TFLOP/s", "frac": (mfma_tf or 0) / (BF16_PEAK_TFLOPS if args.precision == "bf16" else 157.3),
                              "algorithmic_flops_per_step": flops, "avg_phase_ms": learn_ms},
        }
        if cpu_lines is not None:
            # all host cores of this GPU's share (16 on the box), one seed each; and one core
            out["cpu_baseline"], out["cpu_baseline_1core"] = cpu_lines[:2]
            out["cpu_baseline_utd1"] = {"all_cores": cpu_lines[2], "1core": cpu_lines[3]}
        else:
            out["cpu_baseline"] = None
        if force_dist and world == 1:
            out["process_group"] = f"{dist.get_backend()} at world 1 (RLMD_BENCH_FORCE_DIST)"
        print(json.dumps(out), flush=True)
    if _dist_on():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
