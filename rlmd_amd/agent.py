"""SAC / TD3 agents with the reference's interface, learning on the MI355X.

``Agent_sac(inputs)`` / ``Agent_td3(inputs)`` take the reference's ``inputs``
dict (main.py:144-259 + the driver's additions, rl_multiplicative.py:70-113)
and expose its methods: ``store_transistion`` (sic), ``select_next_action``,
``eval_next_action``, ``learn``, ``save_models``, ``load_models`` and
``memory.mem_idx`` (algos/algo_sac.py:82-632, algos/algo_td3.py:84-580).
Parameters are f32 torch tensors on the GPU (one flat buffer per role, with
per-layer views for state_dict compatibility); ``learn()`` runs entirely in
librlmd_amd.so (rlmd_agent_learn) — no torch autograd, no host round trips
inside an update.
"""
import ctypes as C
import math
import os

import numpy as np
import torch

from . import _abi
from ._abi import check, ptr, stream_ptr
from .envs import _StateKeyed

HEADS = {"SAC": ("pi", "log_scale"), "TD3": ("mu",)}
_AGENT_SEEDS = _StateKeyed(b"agent")
def private_agent_seed():
    """The Philox key of an agent built without one (acting noise, the update's
    policy noise, replay indices).  The reference draws these from torch's and
    NumPy's generators, so they follow the driver's torch.manual_seed /
    np.random.seed: the key hashes both generators' states (read, not advanced).
    Agent construction draws the initial parameters from torch's generator
    (reference_init), so consecutive agents see different states."""
    return _AGENT_SEEDS()


def layer_names(algo, net):
    heads = ("q_value",) if net.startswith("critic") else HEADS[algo]
    names = ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"]
    for h in heads:
        names += [h + ".weight", h + ".bias"]
    return names


def layer_shapes(algo, net, S, A, h1, h2):
    inp = S + A if net.startswith("critic") else S
    out = 1 if net.startswith("critic") else A
    shp = [(h1, inp), (h1,), (h2, h1), (h2,)]
    for _ in (("q_value",) if net.startswith("critic") else HEADS[algo]):
        shp += [(out, h2), (out,)]
    return shp


def reference_init(algo, S, A, h1, h2, seed=None):
    """Initial parameters exactly as the reference builds them: nn.Linear default
    init, nets constructed in algo_sac.py:144-149 order (actor, target_actor,
    critic_1, target_critic_1, critic_2, target_critic_2 — targets independent,
    SURVEY §8a-A11).  Returns {net: [tensors]} on CPU."""
    gen_state = None
    if seed is not None:
        gen_state = torch.random.get_rng_state()
        torch.manual_seed(seed)
    out = {}
    try:
        for net in ("actor", "target_actor", "critic_1", "target_critic_1", "critic_2", "target_critic_2"):
            base = net.replace("target_", "")
            shapes = layer_shapes(algo, base, S, A, h1, h2)
            tensors = []
            for i in range(0, len(shapes), 2):
                lin = torch.nn.Linear(shapes[i][1], shapes[i][0])
                tensors += [lin.weight.detach().clone(), lin.bias.detach().clone()]
            out[net] = tensors
    finally:
        if gen_state is not None:
            torch.random.set_rng_state(gen_state)
    return out


# inputs["s_dist"] (algo_sac.py:100, :207-218): the SAC policy's sampler
POLICY_DIST = {"N": _abi.DIST_N, "L": _abi.DIST_L, "MVN": _abi.DIST_MVN}


class DeviceAgent:
    """The learner state on the device + its librlmd_amd handle."""

    def __init__(self, algo, S, A, h1, h2, batch, topk, loss="MSE", precision="fp32", seed=0,
                 gamma=0.99, tau=5e-3, lr_actor=None, lr_critic=None, lr_temp=3e-4, reward_scale=1.0,
                 max_action=0.99, log_scale_min=-20.0, log_scale_max=2.0, reparam_noise=1e-6,
                 log_noise=1e-6, cauchy_scale=1.0, initial_logtemp=0.0, policy_noise=0.1,
                 target_policy_noise=0.2, target_policy_clip=0.5, actor_update_interval=None,
                 target_critic_update=None, target_actor_update=2, temp_update_interval=1,
                 actor_topk=True, policy_dist="N", init=None, init_seed=None, device="cuda:0"):
        sac = algo == "SAC"
        self.algo, self.S, self.A, self.h1, self.h2 = algo, S, A, h1, h2
        self.batch, self.topk, self.device = batch, topk, torch.device(device)
        cfg = _abi.AgentCfg()
        cfg.algo = _abi.SAC if sac else _abi.TD3
        cfg.state_dim, cfg.action_dim, cfg.h1, cfg.h2 = S, A, h1, h2
        cfg.batch, cfg.topk = batch, topk
        cfg.loss_type = _abi.LOSSES.index(loss.upper())
        cfg.precision = {"fp32": _abi.FP32, "bf16": _abi.BF16}[precision]
        cfg.actor_update_interval = actor_update_interval or (1 if sac else 2)
        cfg.target_critic_update = target_critic_update or (1 if sac else 2)
        cfg.target_actor_update = target_actor_update
        cfg.temp_update_interval = temp_update_interval
        cfg.actor_topk = 1 if actor_topk else 0
        cfg.policy_dist = POLICY_DIST[policy_dist]
        cfg.gamma, cfg.tau = gamma, tau
        cfg.lr_actor = lr_actor or (3e-4 if sac else 1e-3)
        cfg.lr_critic = lr_critic or (3e-4 if sac else 1e-3)
        cfg.lr_temp, cfg.reward_scale, cfg.max_action = lr_temp, reward_scale, max_action
        cfg.log_scale_min, cfg.log_scale_max = log_scale_min, log_scale_max
        cfg.reparam_noise, cfg.log_noise = reparam_noise, log_noise
        cfg.cauchy_scale, cfg.initial_logtemp = cauchy_scale, initial_logtemp
        cfg.policy_noise = policy_noise * max_action
        cfg.target_policy_noise = target_policy_noise * max_action
        cfg.target_policy_clip = target_policy_clip * max_action
        cfg.seed = seed
        self.cfg = cfg
        n, oa, o1, o2 = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(_abi.lib().rlmd_agent_layout(C.byref(cfg), C.byref(n), C.byref(oa), C.byref(o1), C.byref(o2)))
        self.n_params = n.value
        self.offsets = {"actor": oa.value, "critic_1": o1.value, "critic_2": o2.value}
        dev = self.device
        self.params = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        self.target = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        self.grads = torch.zeros(_abi.GRAD_SPLITS, self.n_params, dtype=torch.float32, device=dev)
        self.adam_m = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        self.adam_v = torch.zeros(self.n_params, dtype=torch.float32, device=dev)
        init = init if init is not None else reference_init(algo, S, A, h1, h2, init_seed)
        for net in ("actor", "critic_1", "critic_2"):
            for v, t in zip(self.views(net, self.params), init[net]):
                v.copy_(t)
            for v, t in zip(self.views(net, self.target), init["target_" + net]):
                v.copy_(t)
        h = C.c_void_p()
        check(_abi.lib().rlmd_agent_create(C.byref(cfg), ptr(self.params), ptr(self.target), ptr(self.grads),
                                           ptr(self.adam_m), ptr(self.adam_v), C.byref(h)))
        self.h = h
        self.stats = torch.full((1, 16), float("nan"), dtype=torch.float32, device=dev)
        self._seen = self._versions()

    def _versions(self):
        # torch bumps a tensor's version on every in-place write, through any view
        # (state_dict() entries, slices); the device's own updates do not touch it
        return (self.params._version, self.target._version)

    def sync_written(self):
        """Mark the compute copies stale if the parameters or targets were written on
        the torch side since the last call (every act / learn / train step calls it,
        so a write through state_dict() without params_written() is still seen)."""
        v = self._versions()
        if v != self._seen:
            self._seen = v
            check(_abi.lib().rlmd_agent_params_written(self.h))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _abi._LIB is not None:
            _abi.lib().rlmd_agent_destroy(h)
            self.h = None

    def views(self, net, flat):
        shapes = layer_shapes(self.algo, net, self.S, self.A, self.h1, self.h2)
        o = self.offsets[net]
        out = []
        for shp in shapes:
            k = int(np.prod(shp))
            out.append(flat[o:o + k].view(shp))
            o += k
        return out

    def state_dict(self, net, target=False):
        flat = self.target if target else self.params
        return dict(zip(layer_names(self.algo, net), self.views(net, flat)))

    def act(self, obs, mode=0, noise_ctr=0, eps=None, out=None):
        # every tensor handed to the C ABI stays referenced until the call returns
        obs = obs.to(device=self.device, dtype=torch.float32).contiguous()
        n = obs.shape[0]
        out = torch.empty(n, self.A, dtype=torch.float32, device=self.device) if out is None else out
        e = None if eps is None else eps.to(device=self.device, dtype=torch.float32).contiguous()
        self.sync_written()
        check(_abi.lib().rlmd_agent_act(self.h, ptr(obs), n, ptr(out), mode, noise_ctr, ptr(e), stream_ptr()))
        return out

    def learn(self, replay, k=1):
        if self.stats.shape[0] < k:
            self.stats = torch.full((k, 16), float("nan"), dtype=torch.float32, device=self.device)
        self.sync_written()
        check(_abi.lib().rlmd_agent_learn(self.h, replay.h, k, ptr(self.stats), stream_ptr()))
        return self.stats[:k]

    def learn_batch(self, s, a, r, s2, done, eps_a, eps_b=None, eff=None):
        # keep every argument tensor alive until the call has enqueued its work:
        # a temporary freed early is recycled by the caching allocator for the
        # next argument's host->device copy
        f = lambda x: None if x is None else x.to(self.device, torch.float32).contiguous()
        args = [f(s), f(a), f(r), f(s2), done.to(self.device, torch.uint8).contiguous(),
                None if eff is None else eff.to(self.device, torch.int32).contiguous(), f(eps_a), f(eps_b)]
        self.sync_written()
        check(_abi.lib().rlmd_agent_learn_batch(self.h, *[ptr(x) for x in args], ptr(self.stats), stream_ptr()))
        return self.stats[0]

    def status(self, stream=None):
        """(flags, nan_update) from rlmd_status_poll: bit 0 NaN in a mini-batch's
        q / target, bit 1 NaN in the critic statistics (the reference's
        test_live_learning guards); nan_update = learn counter at first set."""
        f, u = C.c_int32(), C.c_int32()
        check(_abi.lib().rlmd_status_poll(self.h, C.byref(f), C.byref(u), stream_ptr(stream)))
        return f.value, u.value

    def save(self, prefix):
        """The reference's checkpoint files: <prefix>_{actor,critic_1,critic_2}.pt
        (networks_sac.py:87-88, :287-292), state dicts with its layer names."""
        for net in ("actor", "critic_1", "critic_2"):
            torch.save({k: v.detach().cpu() for k, v in self.state_dict(net).items()}, f"{prefix}_{net}.pt")

    def load(self, prefix):
        for net in ("actor", "critic_1", "critic_2"):
            sd = torch.load(f"{prefix}_{net}.pt", weights_only=True)
            for k, v in self.state_dict(net).items():
                v.copy_(sd[k])
        self.params_written()

    def params_written(self):
        """Call after writing parameters through state_dict() / the flat tensors:
        the device re-derives its MFMA compute copies before the next act / learn
        (sync_written() also catches torch-side writes by their version counters)."""
        self._seen = self._versions()
        check(_abi.lib().rlmd_agent_params_written(self.h))

    def scalars(self):
        out = (C.c_double * 5)()
        check(_abi.lib().rlmd_agent_scalars(self.h, out))
        return {"cauchy": (out[0], out[1]), "log_alpha": out[2], "learn_step_cntr": int(out[3]),
                "nan_flag": int(out[4])}


class ReplayMemory:
    """On-device ring (rlmd_replay_*) with the reference's mem_idx attribute.

    multi_steps > 1 selects the n-step history sampling of tools/replay.py
    (:93-332) over `lanes` independent transition streams; dynamics "A" sums the
    discounted rewards, anything else multiplies them (replay.py:280-283)."""

    def __init__(self, capacity, S, A, device="cuda:0", multi_steps=1, lanes=1, dynamics="A", gamma=0.99):
        h = C.c_void_p()
        check(_abi.lib().rlmd_replay_create(int(capacity), S, A, C.byref(h)))
        self.h, self.capacity, self.S, self.A, self.device = h, int(capacity), S, A, torch.device(device)
        self.multi_steps = int(multi_steps)
        if self.multi_steps > 1:
            check(_abi.lib().rlmd_replay_set_multistep(h, int(lanes), self.multi_steps,
                                                       1 if str(dynamics) == "A" else 0, float(gamma)))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _abi._LIB is not None:
            _abi.lib().rlmd_replay_destroy(h)
            self.h = None

    @property
    def mem_idx(self):
        m = C.c_int64()
        check(_abi.lib().rlmd_replay_mem_idx(self.h, C.byref(m)))
        return m.value

    def store_exp(self, state, action, reward, next_state, done):
        dev = self.device
        f = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32).reshape(-1, self.S if x is not action else self.A), device=dev)
        s, s2 = f(state), f(next_state)
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(-1, self.A), device=dev)
        n = s.shape[0]
        r = torch.as_tensor(np.asarray(reward, dtype=np.float32).reshape(n), device=dev)
        d = torch.as_tensor(np.asarray(done, dtype=np.uint8).reshape(n), device=dev)
        check(_abi.lib().rlmd_replay_insert(self.h, n, ptr(s), ptr(a), ptr(r), ptr(s2), ptr(d), stream_ptr()))

    def gather(self, rows):
        """sample_exp's gather for given ring rows: (s, a, r, s', done, eff)."""
        dev = self.device
        rows = torch.as_tensor(rows, dtype=torch.int64, device=dev)
        n = rows.numel()
        s, s2 = torch.empty(n, self.S, device=dev), torch.empty(n, self.S, device=dev)
        a, r = torch.empty(n, self.A, device=dev), torch.empty(n, device=dev)
        d, eff = torch.empty(n, dtype=torch.uint8, device=dev), torch.empty(n, dtype=torch.int32, device=dev)
        check(_abi.lib().rlmd_replay_gather(self.h, n, ptr(rows), ptr(s), ptr(a), ptr(r), ptr(s2), ptr(d), ptr(eff),
                                            stream_ptr()))
        return s, a, r, s2, d.bool(), eff


def _loss_code(name):
    return name.upper()


class _Agent:
    """Common part of Agent_sac / Agent_td3 (reference interface)."""

    algo = None

    def __init__(self, inputs, device=None, precision="fp32", seed=None):
        sac = self.algo == "SAC"
        seed = private_agent_seed() if seed is None else seed
        device = device or ("cuda:0" if torch.cuda.is_available() else None)
        if device is None:
            raise _abi.RlmdError("rlmd_amd agents need a GPU (no CPU fallback)")
        self.inputs = inputs
        S = int(sum(inputs["input_dims"]))
        A = int(inputs["num_actions"])
        pre = "sac" if sac else "td3"
        h1, h2 = int(inputs[f"{pre}_layer_1_units"]), int(inputs[f"{pre}_layer_2_units"])
        self.batch_size = int(inputs["mini_batch_size"])
        self.optimise_count = int(inputs["batch_size"][inputs["algo"]])
        self.max_action = float(inputs["max_action"])
        self.num_actions = A
        kw = dict(gamma=inputs["discount"], max_action=self.max_action, log_noise=float(inputs["log_noise"]),
                  cauchy_scale=float(inputs["cauchy_scale"]), actor_topk=inputs["actor_percentile"] != 100)
        if sac:
            kw.update(tau=inputs["sac_target_update_rate"], lr_actor=inputs["sac_actor_learn_rate"],
                      lr_critic=inputs["sac_critic_learn_rate"], lr_temp=inputs["sac_temp_learn_rate"],
                      reward_scale=float(inputs["reward_scale"]),
                      log_scale_min=float(inputs["log_scale_min"]), log_scale_max=float(inputs["log_scale_max"]),
                      reparam_noise=float(inputs["reparam_noise"]), policy_dist=str(inputs.get("s_dist", "N")),
                      initial_logtemp=float(inputs["initial_logtemp"]),
                      actor_update_interval=int(inputs["sac_actor_step_update"]),
                      temp_update_interval=int(inputs["sac_temp_step_update"]),
                      target_critic_update=int(inputs["sac_target_critic_update"]))
        else:
            kw.update(tau=inputs["td3_target_update_rate"], lr_actor=inputs["td3_actor_learn_rate"],
                      lr_critic=inputs["td3_critic_learn_rate"], policy_noise=inputs["policy_noise"],
                      target_policy_noise=inputs["target_policy_noise"],
                      target_policy_clip=inputs["target_policy_clip"],
                      actor_update_interval=int(inputs["td3_actor_step_update"]),
                      target_actor_update=int(inputs["td3_target_actor_update"]),
                      target_critic_update=int(inputs["td3_target_critic_update"]))
        self.dev = DeviceAgent(self.algo, S, A, h1, h2, self.batch_size, self.optimise_count,
                               loss=inputs["loss_fn"], precision=precision, seed=seed, device=device, **kw)
        buf = int(min(inputs["buffer"], inputs["n_cumsteps"]))  # replay.py:75-78
        self.memory = ReplayMemory(buf, S, A, device=device, multi_steps=int(inputs.get("multi_steps", 1)),
                                   dynamics=inputs.get("dynamics", "A"), gamma=float(inputs["discount"]))
        self._act_ctr = 0
        self._batch_ctr = 0
        self.file_prefix = None
        if all(k in inputs for k in ("env_id", "dynamics", "s_dist", "loss_fn", "critic_mean_type", "n_cumsteps",
                                     "n_trials", "trial", "multi_steps")):
            # algo_sac.py:121-141: ./results/<dyna>models/<env_id>/ + save_directory(results=False)
            from . import logs

            self.file_prefix = logs.save_directory(inputs, results=False)
            os.makedirs(os.path.dirname(self.file_prefix), exist_ok=True)

    # -- reference methods --------------------------------------------------
    def store_transistion(self, state, action, reward, next_state, done):
        self.memory.store_exp(state, action, reward, next_state, done)

    def select_next_action(self, state):
        s = torch.as_tensor(np.asarray(state, dtype=np.float32).reshape(1, -1))
        self._act_ctr += 1
        return self.dev.act(s, mode=0, noise_ctr=self._act_ctr)[0].cpu().numpy()

    def eval_next_action(self, state):
        s = torch.as_tensor(np.asarray(state, dtype=np.float32).reshape(1, -1))
        return self.dev.act(s, mode=1)[0].cpu().numpy()

    def learn(self):
        if self.memory.mem_idx <= self.batch_size:
            loss = [np.nan] * 11
            logtemp = np.float32(self.dev.scalars()["log_alpha"]) if self.algo == "SAC" else np.nan
            return loss, logtemp, [np.nan] * 4
        st = self.dev.learn(self.memory, 1)[0].cpu().numpy().astype(np.float64)
        loss = [float(x) for x in st[:11]]
        logtemp = np.float32(st[11]) if self.algo == "SAC" else np.nan
        return loss, logtemp, [float(x) for x in st[12:16]]

    def _mini_batch(self):
        """algo_sac.py:238-262: one mini-batch of B distinct uniform ring rows,
        sampled and gathered on the device (rlmd_replay_sample): (states,
        actions, rewards, next_states, dones, effective n-step counts)."""
        dev, B, S, A = self.dev.device, self.batch_size, self.dev.S, self.dev.A
        m = self.memory
        idx = torch.empty(B, dtype=torch.int64, device=dev)
        s, s2 = torch.empty(B, S, device=dev), torch.empty(B, S, device=dev)
        a, r = torch.empty(B, A, device=dev), torch.empty(B, device=dev)
        d, eff = torch.empty(B, dtype=torch.uint8, device=dev), torch.empty(B, dtype=torch.int32, device=dev)
        self._batch_ctr += 1
        check(_abi.lib().rlmd_replay_sample(m.h, B, int(self.dev.cfg.seed) ^ 0xBA7C4, self._batch_ctr, ptr(idx),
                                            ptr(s), ptr(a), ptr(r), ptr(s2), ptr(d), ptr(eff), stream_ptr()))
        return s, a, r, s2, d.bool(), eff

    def _multi_step_target(self, *args, **kw):
        """algo_sac.py:300-367: the target is formed inside the fused learn()
        kernels on the device (fwd_rows target jobs + the critic-loss epilogue),
        never materialised for the host; kept for the reference's hasattr contract
        (tests/test_input_agent.py:587-734)."""
        raise NotImplementedError("the target is fused into learn() (rlmd_agent_learn)")

    def _update_critic_parameters(self, *args, **kw):
        """algo_sac.py:597-615: the Polyak update runs inside the device Adam step of
        every learn(); kept for the reference's hasattr contract."""
        raise NotImplementedError("Polyak averaging is fused into learn() (rlmd_agent_learn)")

    def _prefix(self):
        return self.file_prefix or os.path.join(".", "rlmd_amd_model")

    def _ckpt(self, net):
        return f"{self._prefix()}_{net}.pt"

    def save_models(self):
        self.dev.save(self._prefix())

    def load_models(self, prefix=None):
        """algo_sac.py:625-632; prefix: another file stem (the driver's `continue`
        loads the previous trial's checkpoints)."""
        self.dev.load(self._prefix() if prefix is None else prefix)


class Agent_sac(_Agent):
    algo = "SAC"


class Agent_td3(_Agent):
    algo = "TD3"
