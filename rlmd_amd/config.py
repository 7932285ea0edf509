"""The reference's run tables for the multiplicative and market paths.

``GYM_ENVS`` holds the rows of main.py:40-139 this build runs (keys 8-26:
coin / dice / GBM / Dice_SH / SNP and USEI markets): [env_id, state_dim,
action_dim, warm-up steps].  ``INPUTS`` holds main.py:144-259's learning and
model parameters that the multiplicative / market drivers read, with the
reference's defaults.  ``input_initialisation`` is tools/utils.py:80-106.
Keys keep the reference's names (including its spellings) so a reference
``inputs`` dict can be passed through unchanged.
"""
import os
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


# ---------------------------------------------------------------------------
# Start-up validation: tests/test_input_agent.py learning_tests (:51-406) and
# env_tests (:409-584), restated for the keys and drivers this build runs.
# A bad value raises AssertionError with the reference's message before any
# device work, as main.py:277-280 runs them.  The additive / guidance sections
# are checked only when their keys are present (those drivers are out of scope).
# ---------------------------------------------------------------------------
_TB, _TD, _TF = "variable must be of type bool", "variable must be of type dict", "variable must be of type float"
_TFI, _TI = "variable must be of type float for int", "variable must be of type int"
_TL, _TS = "variable must be of type list", "variable must be of type str"
_GTE0, _GT0 = "quantity must be greater than or equal to 0", "quantity must be greater than 0"
_GTE1 = "quantity must be greater than or equal to 1"
LOSSES = ["MSE", "HUB", "MAE", "HSC", "CAU", "TCAU", "CIM", "MSE2", "MSE4", "MSE6"]


def _num(x):
    return isinstance(x, (float, int)) and not isinstance(x, bool)


def _two_digits(name, v):
    # "n_cumsteps must consist of only 2 leading non-zero digits" (str(5e4)[2:] = "000.0")
    assert set(list(str(v)[2:])).issubset(set(["0", "."])), f"{name} must consist of only 2 leading non-zero digits"


def _unique_pos_ints(name, xs, what):
    assert isinstance(xs, list), _TL
    assert all(isinstance(x, int) and not isinstance(x, bool) for x in xs), _TI
    assert len(xs) >= 1, f"{name} must have at least one {what}"
    assert len(xs) == len(set(xs)), f"{name} must contain only unique elements"
    assert all(x >= 1 for x in xs), f"{name} must be a list of (non-zero) positive integers"


def _schedule(inputs, sfx, steps_key="max_eval_steps"):
    """The per-driver execution block (…_add / _mul / _mkt / _gud)."""
    for k in (f"n_trials_{sfx}", f"n_cumsteps_{sfx}", f"eval_freq_{sfx}", f"n_eval_{sfx}"):
        assert _num(inputs[k]), _TFI
        assert int(inputs[k]) >= 1, _GTE1
    _two_digits(f"n_cumsteps_{sfx}", inputs[f"n_cumsteps_{sfx}"])
    assert int(inputs[f"eval_freq_{sfx}"]) <= int(inputs[f"n_cumsteps_{sfx}"]), \
        f"eval_freq_{sfx} must be less than or equal to n_cumsteps_{sfx}"
    if f"{steps_key}_{sfx}" in inputs:
        assert _num(inputs[f"{steps_key}_{sfx}"]), _TFI
        assert int(inputs[f"{steps_key}_{sfx}"]) >= 1, _GTE1
    if f"smoothing_window_{sfx}" in inputs:
        assert _num(inputs[f"smoothing_window_{sfx}"]), _TFI
        assert int(inputs[f"smoothing_window_{sfx}"]) >= 0, _GTE0
    for k in (f"actor_percentile_{sfx}", f"critic_percentile_{sfx}"):
        assert _num(inputs[k]), _TFI
        assert 0 < inputs[k] <= 100, f"{k} must be within (0, 100] interval"


def learning_tests(inputs: dict) -> None:
    """tests/test_input_agent.py:51-406 (learning, execution and hyper-parameter
    checks of the folded inputs dict)."""
    assert isinstance(inputs, dict), _TD
    # training input tests (:61-92)
    assert isinstance(inputs["test_agent"], bool), _TB
    assert isinstance(inputs["algo_name"], list), _TL
    assert set(inputs["algo_name"]).issubset({"SAC", "TD3"}), \
        "algo_name must be a list containing only 'SAC' and/or 'TD3'"
    assert 1 <= len(inputs["algo_name"]) <= 2, "only upto two possible algorithms selectable"
    assert len(inputs["algo_name"]) == len(set(inputs["algo_name"])), "algo_name must contain only unique elements"
    assert isinstance(inputs["critic_loss"], list), _TL
    assert set(inputs["critic_loss"]).issubset(set(LOSSES)), \
        "critic_loss must be a list containing 'MSE', 'HUB', 'MAE', 'HSC', 'CAU', 'TCAU', 'CIM', 'MSE2', 'MSE4', " \
        "and/or 'MSE6'"
    assert 1 <= len(inputs["critic_loss"]) <= 10, "only ten possible critic_loss functions selectable"
    assert len(inputs["critic_loss"]) == len(set(inputs["critic_loss"])), \
        "critic_loss must contain only unique elements"
    _unique_pos_ints("bootstraps (multi-steps)", inputs["bootstraps"], "multi-step")
    # execution blocks (:94-292); additive / guidance only when configured
    if "n_trials_add" in inputs:
        _schedule(inputs, "add")
    _schedule(inputs, "mul")
    _unique_pos_ints("n_gambles (number of gambles)", inputs["n_gambles"], "count of gambles")
    md = inputs["market_dir"]
    assert isinstance(md, (str, bytes, os.PathLike)), _TS
    assert md[0:2] == "./" and md[-1] == "/", "market_dir file path must be in a sub-directory relative to main.py"
    _schedule(inputs, "mkt")
    assert _num(inputs["action_days"]), _TFI
    assert int(inputs["action_days"]) >= 1, _GTE1
    for k in ("train_days", "test_days"):
        assert _num(inputs[k]), _TFI
        assert int(inputs[k]) > 0, _GT0
    for k, d in (("train_shuffle_days", "train_days"), ("test_shuffle_days", "test_days")):
        assert isinstance(inputs[k], int), _TI
        assert int(inputs[k]) >= 1, _GTE1
        assert inputs[k] <= int(inputs[d]), f"{k} must be less than or equal to {d.replace('days', 'years')}"
    for k in ("gap_days_min", "gap_days_max"):
        assert isinstance(inputs[k], int), _TI
        assert int(inputs[k]) >= 0, _GTE0
    assert int(inputs["gap_days_min"]) <= int(inputs["gap_days_max"]), \
        "gap_days_max must be greater than or equal to gap_days_min"
    _unique_pos_ints("past_days (observed days)", inputs["past_days"], "count of days")
    if "n_trials_gud" in inputs:
        _schedule(inputs, "gud")
    # learning variable tests (:296-333)
    assert isinstance(inputs["gpu"], str), _TS
    if inputs["gpu"] != "cpu":
        assert inputs["gpu"][0:5] == "cuda:"
        assert int(inputs["gpu"][-1]) >= 0, _GTE0
    assert isinstance(inputs["buffer_gpu"], bool), _TB
    assert _num(inputs["buffer"]), _TFI
    _two_digits("buffer", inputs["buffer"])
    assert int(inputs["buffer"]) >= 1, _GTE1
    for sfx in ("add", "mul", "mkt", "gud"):
        if f"n_cumsteps_{sfx}" in inputs:
            assert inputs["buffer"] >= int(inputs[f"n_cumsteps_{sfx}"]), \
                f"buffer must be greater than or equal to n_cumsteps_{sfx} training steps"
    assert 0 <= inputs["discount"] < 1, "discount must be within [0, 1) interval"
    assert _num(inputs["trail"]), _TFI
    assert int(inputs["trail"]) >= 1, _GTE1
    assert _num(inputs["cauchy_scale"]), _TFI
    assert inputs["cauchy_scale"] > 0, _GT0
    assert _num(inputs["r_abs_zero"]) or inputs["r_abs_zero"] is None, "r_abs_zero must be either real number or None"
    assert isinstance(inputs["continue"], bool), _TB
    # critic loss aggregation (:336-343)
    assert inputs["critic_mean_type"] == "E", "critic_mean_type must be 'E' ('S' not currently possible)"
    assert _num(inputs["shadow_low_mul"]), _TFI
    assert inputs["shadow_low_mul"] >= 0, _GTE0
    assert _num(inputs["shadow_high_mul"]), _TFI
    assert inputs["shadow_high_mul"] > 0, _GT0
    # SAC (:346-374) and TD3 (:377-402) hyper-parameters
    for k in ("sac_actor_learn_rate", "sac_critic_learn_rate", "sac_temp_learn_rate", "sac_target_update_rate",
              "td3_actor_learn_rate", "td3_critic_learn_rate", "td3_target_update_rate", "policy_noise",
              "target_policy_noise", "target_policy_clip"):
        assert _num(inputs[k]), _TFI
        assert inputs[k] > 0, _GT0
    for k in ("sac_layer_1_units", "sac_layer_2_units", "sac_actor_step_update", "sac_temp_step_update",
              "sac_target_critic_update", "td3_layer_1_units", "td3_layer_2_units", "td3_actor_step_update",
              "td3_target_actor_update", "td3_target_critic_update"):
        assert _num(inputs[k]), _TFI
        assert int(inputs[k]) >= 1, _GTE1
    for k in ("initial_logtemp", "log_scale_min", "log_scale_max"):
        assert _num(inputs[k]), _TFI
    assert inputs["log_scale_min"] < inputs["log_scale_max"], "SAC scale limits must be valid"
    assert isinstance(inputs["reparam_noise"], float), _TF
    assert 1e-7 < inputs["reparam_noise"] < 1e-5, "SAC reparam_noise must be a real number in the vicinity of 1e-6"
    # shared algorithm parameters (:405-434)
    sd = inputs["sample_dist"]
    assert isinstance(sd, dict), _TD
    assert set(sd.keys()).issubset({"SAC", "TD3"}), "must contain the two main algorithms"
    assert sd["SAC"] in ("N", "L", "MVN"), "SAC sample_dist must be either 'N' (normal = Gaussian) or 'L' " \
                                           "(2x exponential = Laplace), or 'MVN' (multi-variate normal)"
    assert isinstance(sd["TD3"], str), _TS
    assert sd["TD3"] in ("N", "L"), "TD3 sample_dist must be either 'N' (normal = Gaussian) or 'L' " \
                                    "(2x exponential = Laplace)"
    for k in ("batch_size", "grad_step"):
        assert isinstance(inputs[k], dict), _TD
        assert set(inputs[k].keys()).issubset({"SAC", "TD3"}), "must contain the two main algorithms"
        for a in ("TD3", "SAC"):
            assert _num(inputs[k][a]), _TFI
            assert int(inputs[k][a]) >= 1, _GTE1
    assert isinstance(inputs["log_noise"], float), _TF
    assert 1e-7 < inputs["log_noise"] < 1e-5, "log_noise must be a real number in the vicinity of 1e-6"


def env_tests(gym_envs: Dict[str, list], inputs: dict, load_market=None) -> None:
    """tests/test_input_agent.py:409-584: the selected keys' table rows, warm-up
    and evaluation cadence against their driver's budget, and that each market
    key's price table is long enough for train + gap + test at every past_days.
    load_market(key) -> prices [days, assets] (default: main.load_market_data)."""
    assert isinstance(gym_envs, dict), _TD
    assert all(isinstance(int(env), int) for env in gym_envs), \
        "all environment keys must be strings that are convertible to integers"
    keys = [int(env) for env in gym_envs]
    assert isinstance(inputs["envs"], list), _TL
    assert set(inputs["envs"]).issubset(set(keys)), "environments must be selected from gym_envs dict keys"
    assert inputs["ENV_KEY"] is None
    multi_key, _, market_key = env_dynamics(gym_envs)
    for key in inputs["envs"]:
        row = gym_envs[str(key)]
        assert isinstance(row, list), _TL
        assert len(row) == 4, "environment {} list musst be of length 4".format(key)
        assert isinstance(row[0], str), _TS
        assert all(_num(x) for x in row[1:]), \
            "environment {} details must be a list of the form [string, int>0, int>0, real>0]".format(key)
        assert int(row[1]) >= 1, "environment {} must have at least one state".format(key)
        assert int(row[2]) >= 1, "environment {} must have at least one action".format(key)
        sfx = "mul" if key < market_key else "mkt"
        assert int(row[3]) >= 0, _GTE0
        assert int(row[3]) < int(inputs[f"n_cumsteps_{sfx}"]), \
            "environment {}: warm-up must be less than total training steps".format(key)
        assert int(2 * inputs[f"eval_freq_{sfx}"]) <= int(inputs[f"n_cumsteps_{sfx}"]), \
            "environment {}: 2x evaluation frequency must be less than or equal to total training steps".format(key)
    for key in inputs["envs"]:
        if key < market_key:
            continue
        if load_market is None:
            from .main import load_market_data

            data = load_market_data(key, gym_envs, inputs)
        else:
            data = load_market(key)
        time_length = data.shape[0]
        for days in inputs["past_days"]:
            sample_length = int(int(inputs["action_days"]) * (int(inputs["train_days"]) + int(inputs["test_days"]))
                                + int(inputs["gap_days_max"]) + days - 1)
            assert time_length >= sample_length, \
                "ENV_KEY {}: total time {} period with {} day(s) observed and {} day(s) action spacing must be " \
                "greater than sample length = {}".format(key, time_length, days, int(inputs["action_days"]),
                                                        sample_length)
