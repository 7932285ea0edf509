"""ctypes binding of librlmd_amd.so (include/rlmd_abi.h).

The shared library is the product; this module only declares its C ABI.  It
fails loudly: importing the package without the built .so raises, and every
non-zero return code raises ``RlmdError`` with ``rlmd_last_error()``.  There
is no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librlmd_amd.so")

# enums (rlmd_abi.h)
COIN, DICE, GBM, DICE_SH, MARKET = range(5)
INV_A, INV_B, INV_C, INV_INSURED = range(4)
SAC, TD3 = 0, 1
STATUS_NAN_BATCH, STATUS_NAN_STATS = 1, 2
FP32, BF16 = 0, 1
DIST_N, DIST_L, DIST_MVN = 0, 1, 2
LOSSES = ["MSE", "HUB", "MAE", "HSC", "CAU", "TCAU", "CIM", "MSE2", "MSE4", "MSE6"]
GEMM_FWD, GEMM_BWD_X, GEMM_BWD_W = 0, 1, 2
GRAD_SPLITS = 4  # RLMD_GRAD_SPLITS


class RlmdError(RuntimeError):
    pass


class EnvCfg(C.Structure):
    _fields_ = [("family", C.c_int32), ("investor", C.c_int32), ("n_lanes", C.c_int32),
                ("n_gambles", C.c_int32), ("obs_days", C.c_int32), ("time_length", C.c_int32),
                ("action_days", C.c_int32), ("shuffle_days", C.c_int32),
                ("sample_days", C.c_int32), ("slice_groups", C.c_int32), ("seed", C.c_uint64)]


class AgentCfg(C.Structure):
    _fields_ = [("algo", C.c_int32), ("state_dim", C.c_int32), ("action_dim", C.c_int32),
                ("h1", C.c_int32), ("h2", C.c_int32), ("batch", C.c_int32), ("topk", C.c_int32),
                ("loss_type", C.c_int32), ("precision", C.c_int32),
                ("actor_update_interval", C.c_int32), ("target_critic_update", C.c_int32),
                ("target_actor_update", C.c_int32), ("temp_update_interval", C.c_int32),
                ("actor_topk", C.c_int32), ("policy_dist", C.c_int32),
                ("gamma", C.c_float), ("tau", C.c_float), ("lr_actor", C.c_float),
                ("lr_critic", C.c_float), ("lr_temp", C.c_float), ("reward_scale", C.c_float),
                ("max_action", C.c_float), ("log_scale_min", C.c_float),
                ("log_scale_max", C.c_float), ("reparam_noise", C.c_float),
                ("log_noise", C.c_float), ("cauchy_scale", C.c_float),
                ("initial_logtemp", C.c_float), ("policy_noise", C.c_float),
                ("target_policy_noise", C.c_float), ("target_policy_clip", C.c_float),
                ("seed", C.c_uint64)]


class TrainCfg(C.Structure):
    _fields_ = [("cum_step", C.c_int64), ("warmup_steps", C.c_int32),
                ("smoothing_window", C.c_int32), ("abs_warmup", C.c_int32),
                ("k_updates", C.c_int32)]


P = C.c_void_p
I32, I64, U64 = C.c_int32, C.c_int64, C.c_uint64
SIGNATURES = {
    "rlmd_last_error": (C.c_char_p, []),
    "rlmd_device_sync": (C.c_int, []),
    "rlmd_stream_create": (C.c_int, [P]),
    "rlmd_stream_create_cu": (C.c_int, [P, I32, P]),
    "rlmd_stream_destroy": (C.c_int, [P]),
    "rlmd_env_create": (C.c_int, [C.POINTER(EnvCfg), P, I64, C.POINTER(P)]),
    "rlmd_env_destroy": (C.c_int, [P]),
    "rlmd_env_dims": (C.c_int, [P, C.POINTER(I32), C.POINTER(I32), C.POINTER(I32), C.POINTER(I32)]),
    "rlmd_env_reset": (C.c_int, [P, P, P, P]),
    "rlmd_env_step": (C.c_int, [P, P, P, P, P, P, P, P]),
    "rlmd_env_step_f64": (C.c_int, [P, P, P, P, P, P, P, P]),
    "rlmd_env_lane_state": (C.c_int, [P, P, P]),
    "rlmd_eval_rollout": (C.c_int, [P, P, I32, I64, I32, I32, P, P, P, P, P]),
    "rlmd_eval_stats": (C.c_int, [P, P, P, I32, I32, I32, P, P]),
    "rlmd_replay_create": (C.c_int, [I64, I32, I32, C.POINTER(P)]),
    "rlmd_replay_destroy": (C.c_int, [P]),
    "rlmd_replay_insert": (C.c_int, [P, I64, P, P, P, P, P, P]),
    "rlmd_replay_mem_idx": (C.c_int, [P, C.POINTER(I64)]),
    "rlmd_replay_read": (C.c_int, [P, I64, I64, P, P, P, P, P, P]),
    "rlmd_replay_sample": (C.c_int, [P, I32, U64, U64, P, P, P, P, P, P, P, P]),
    "rlmd_replay_set_multistep": (C.c_int, [P, I32, I32, I32, C.c_double]),
    "rlmd_replay_gather": (C.c_int, [P, I32, P, P, P, P, P, P, P, P]),
    "rlmd_agent_layout": (C.c_int, [C.POINTER(AgentCfg), C.POINTER(I64), C.POINTER(I64),
                                    C.POINTER(I64), C.POINTER(I64)]),
    "rlmd_agent_create": (C.c_int, [C.POINTER(AgentCfg), P, P, P, P, P, C.POINTER(P)]),
    "rlmd_agent_destroy": (C.c_int, [P]),
    "rlmd_agent_act": (C.c_int, [P, P, I64, P, I32, U64, P, P]),
    "rlmd_agent_learn": (C.c_int, [P, P, I32, P, P]),
    "rlmd_agent_learn_batch": (C.c_int, [P, P, P, P, P, P, P, P, P, P, P]),
    "rlmd_agent_scalars": (C.c_int, [P, P]),
    "rlmd_agent_params_written": (C.c_int, [P]),
    "rlmd_status_poll": (C.c_int, [P, C.POINTER(I32), C.POINTER(I32), P]),
    "rlmd_train_step": (C.c_int, [P, P, P, C.POINTER(TrainCfg), P, P, P, P, P]),
    "rlmd_train_reset": (C.c_int, [P, P, P]),
    "rlmd_train_flush_stats": (C.c_int, [P, P]),
    "rlmd_train_episode_log": (C.c_int, [P, C.c_int32]),
    "rlmd_train_set_fused": (C.c_int, [P, C.c_int32]),
    "rlmd_train_last_fused": (C.c_int, [P]),
    "rlmd_train_set_stored_state": (C.c_int, [P, C.c_int32]),
    "rlmd_train_stored_state": (C.c_int, [P]),
    "rlmd_train_episode_drain": (C.c_int, [P, P, C.c_int64, P, P, P]),
    "rlmd_env_lane_start": (C.c_int, [P, P]),
    "rlmd_env_write_prices": (C.c_int, [P, P, I64, I64, P]),
    "rlmd_shadow_means": (C.c_int, [P, I32, I32, C.c_float, C.c_float, P, I32, P]),
    "rlmd_shadow_equiv": (C.c_int, [P, P, P, P, C.c_double, I64, P, P]),
    "rlmd_lev_workspace_bytes": (I64, [I64, I32]),
    "rlmd_lev_sorted_workspace_bytes": (I64, [I64, I32]),
    "rlmd_lev_sweep_sorted": (C.c_int, [I32, P, I64, I32, I64, I64, C.c_float, P, P, I32, P, I64, P, P, P]),
    "rlmd_lev_brain_workspace_bytes": (I64, [I64, I32]),
    "rlmd_lev_brain": (C.c_int, [I32, P, I64, I32, I64, I64, C.c_float, P, C.c_float, P, I32, P, I64, P, P]),
    "rlmd_lev_final_sorted": (C.c_int, [I32, P, I64, I32, I64, I64, C.c_float, P, P, I32, P, I64, P, P, P]),
    "rlmd_lev_coin_sweep": (C.c_int, [P, I64, I32, I64, I64, C.c_float, C.c_float, C.c_float, P, I32, P, I64, P, P,
                                       P]),
    "rlmd_eval_market": (C.c_int, [P, P, P, C.c_int64, C.c_int32, C.c_int32, P, P, P, P, P, P, P]),
    "rlmd_profile_enable": (C.c_int, [P, I32]),
    "rlmd_profile_read": (C.c_int, [P, P, P]),
    "rlmd_profile_stride": (C.c_int, [P, I32]),
    "rlmd_profile_samples": (C.c_int, [P, I32, P, C.c_int64, P]),
    "rlmd_agent_set_cu_budget": (C.c_int, [P, I32]),
    "rlmd_gemm": (C.c_int, [I32, I32, I32, I32, I32, I32, P, I32, P, I32, P, P, I32, P, I32, P, P]),
}


def header_symbols():
    """Function names declared in include/rlmd_abi.h (for the export test)."""
    import re

    hdr = os.path.join(HERE, "..", "include", "rlmd_abi.h")
    txt = open(hdr).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char\*)\s+(rlmd_\w+)\(", txt, re.M)))


def load(path=LIB_PATH):
    if not os.path.exists(path):
        raise RlmdError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP extension is required; there is no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        # RLMD_LIB_PATH: another build of the same ABI (tools/ab_build.py A/B runs)
        _LIB = load(os.environ.get("RLMD_LIB_PATH", LIB_PATH))
    return _LIB


def check(rc):
    if rc != 0:
        raise RlmdError(lib().rlmd_last_error().decode())
    return rc


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    assert t.is_contiguous(), "rlmd ABI expects contiguous tensors"
    return C.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)
