"""The reference's run tables for the multiplicative and market paths.

``GYM_ENVS`` holds the rows of main.py:40-139 this build runs (keys 8-26:
coin / dice / GBM / Dice_SH / SNP and USEI markets): [env_id, state_dim,
action_dim, warm-up steps].  ``INPUTS`` holds main.py:144-259's learning and
model parameters that the multiplicative / market drivers read, with the
reference's defaults.  ``input_initialisation`` is tools/utils.py:80-106.
Keys keep the reference's names (including its spellings) so a reference
``inputs`` dict can be passed through unchanged.
"""
from typing import Dict, List

GYM_ENVS: Dict[str, list] = {
    "8": ["Coin_InvA", 5, 1, 1e3],
    "9": ["Coin_InvB", 5, 2, 1e3],
    "10": ["Coin_InvC", 5, 3, 1e3],
    "11": ["Dice_InvA", 5, 1, 1e3],
    "12": ["Dice_InvB", 5, 2, 1e3],
    "13": ["Dice_InvC", 5, 3, 1e3],
    "14": ["GBM_InvA", 5, 1, 1e3],
    "15": ["GBM_InvB", 5, 2, 1e3],
    "16": ["GBM_InvC", 5, 3, 1e3],
    "17": ["Dice_SH_INSURED", 6, 1, 1e3],
    "18": ["Dice_SH_InvA", 6, 2, 1e3],
    "19": ["Dice_SH_InvB", 6, 3, 1e3],
    "20": ["Dice_SH_InvC", 6, 4, 1e3],
    "21": ["SNP_InvA", 5, 1, 1e3],
    "22": ["SNP_InvB", 5, 2, 1e3],
    "23": ["SNP_InvC", 5, 3, 1e3],
    "24": ["EI_InvA", 7, 3, 1e3],
    "25": ["EI_InvB", 7, 4, 1e3],
    "26": ["EI_InvC", 7, 5, 1e3],
}

INPUTS: dict = {
    # multiplicative execution (main.py:153-162)
    "n_trials_mul": 10, "n_cumsteps_mul": 5e4, "eval_freq_mul": 1e3, "n_eval_mul": 1e2,
    "max_eval_steps_mul": 1e2, "smoothing_window_mul": 2e3, "actor_percentile_mul": 50,
    "critic_percentile_mul": 50, "n_gambles": [1],
    # market execution (main.py:165-186)
    "market_dir": "./tools/market_data/", "n_trials_mkt": 10, "n_cumsteps_mkt": 1e5, "eval_freq_mkt": 1e3,
    "n_eval_mkt": 1e2, "smoothing_window_mkt": 2e3, "actor_percentile_mkt": 50, "critic_percentile_mkt": 50,
    "action_days": 1, "train_days": 1e3, "test_days": 250, "train_shuffle_days": 5, "test_shuffle_days": 3,
    "gap_days_min": 5, "gap_days_max": 20, "past_days": [1],
    # learning variables (main.py:201-218)
    "gpu": "cuda:0", "buffer_gpu": True, "buffer": 1e6, "discount": 0.99, "trail": 50, "cauchy_scale": 1,
    "r_abs_zero": None, "continue": False, "critic_mean_type": "E", "shadow_low_mul": 1e0,
    "shadow_high_mul": 1e1,
    # SAC (main.py:222-236)
    "sac_actor_learn_rate": 3e-4, "sac_critic_learn_rate": 3e-4, "sac_temp_learn_rate": 3e-4,
    "sac_layer_1_units": 256, "sac_layer_2_units": 256, "sac_actor_step_update": 1, "sac_temp_step_update": 1,
    "sac_target_critic_update": 1, "sac_target_update_rate": 5e-3, "initial_logtemp": 0, "reward_scale": 1,
    "log_scale_min": -20, "log_scale_max": 2, "reparam_noise": 1e-6,
    # TD3 (main.py:239-250)
    "td3_actor_learn_rate": 1e-3, "td3_critic_learn_rate": 1e-3, "td3_layer_1_units": 400,
    "td3_layer_2_units": 300, "td3_actor_step_update": 2, "td3_target_actor_update": 2,
    "td3_target_critic_update": 2, "td3_target_update_rate": 5e-3, "policy_noise": 0.1,
    "target_policy_noise": 0.2, "target_policy_clip": 0.5,
    # shared (main.py:253-259)
    "sample_dist": {"SAC": "N", "TD3": "N"}, "batch_size": {"SAC": 256, "TD3": 100},
    "grad_step": {"SAC": 1, "TD3": 1}, "log_noise": 1e-6,
}


def input_initialisation(inputs: dict, envs: List[int], algo: List[str], critic: List[str],
                         multi_steps: List[int]) -> dict:
    """tools/utils.py:80-106: the run lists folded into the inputs dict."""
    return {"test_agent": False, "envs": envs, "ENV_KEY": None, "algo_name": [a.upper() for a in algo],
            "critic_loss": [c.upper() for c in critic], "bootstraps": multi_steps, **inputs}


def env_dynamics(gym_envs: Dict[str, list]):
    """tools/utils.py:109-140 for the keys this build knows: (multi_key, sh_key,
    market_key)."""
    first = lambda name: [int(k) for k, v in gym_envs.items() if v[0] == name][0]
    return first("Coin_InvA"), first("Dice_SH_INSURED"), first("SNP_InvA")
