"""Host side of the reference interface (CPU): the method / attribute contract
the reference enforces with hasattr (tests/test_input_agent.py:587-734 for the
agents, tests/test_input_envs.py for the envs), the run tables, and the
driver's host arithmetic (action window, NaN guard)."""
import numpy as np
import pytest


def test_agent_method_contract():
    from rlmd_amd.agent import Agent_sac, Agent_td3

    for cls in (Agent_sac, Agent_td3):
        for m in ("store_transistion", "select_next_action", "eval_next_action", "_mini_batch",
                  "_multi_step_target", "learn", "_update_critic_parameters", "save_models", "load_models"):
            assert callable(getattr(cls, m, None)), f"{cls.__name__} lacks {m}"


def test_env_class_contract():
    from rlmd_amd import envs
    from rlmd_amd.config import GYM_ENVS

    for key, (name, S, A, warm) in GYM_ENVS.items():
        if name.startswith(("SNP", "EI")):
            assert any(n.startswith("Market_Inv" + name.split("_Inv")[1]) for n in envs.ENV_CLASSES)
            continue
        cls = envs.ENV_CLASSES[name]
        for m in ("reset", "step"):
            assert callable(getattr(cls, m))
        assert warm == 1e3


def test_input_initialisation_and_tables():
    from rlmd_amd.config import GYM_ENVS, INPUTS, env_dynamics, input_initialisation

    inp = input_initialisation(dict(INPUTS), [8], ["sac"], ["mse"], [1])
    assert inp["algo_name"] == ["SAC"] and inp["critic_loss"] == ["MSE"] and inp["bootstraps"] == [1]
    assert inp["test_agent"] is False and inp["ENV_KEY"] is None
    assert env_dynamics(GYM_ENVS) == (8, 17, 21)
    # main.py's dims for the multiplicative keys
    assert GYM_ENVS["17"][1:3] == [6, 1] and GYM_ENVS["20"][1:3] == [6, 4]


def test_action_window():
    """tools/utils.py:330-373: float64 window, identity during the warm-up."""
    from rlmd_amd.scripts.rl_multiplicative import action_window

    a = np.array([0.9], dtype=np.float32)
    assert action_window(a, 0.99, -0.99, 500, 2000, 1000) is a
    w = action_window(a, np.float32(0.99), np.float32(-0.99), 1001, 2000, 1000)
    width = (np.sin(np.pi * (1001 / 2000 - 0.5)) + 1) / 2
    assert w.dtype == np.float64
    assert w[0] == np.float64(np.float32(0.99)) * width
    w2 = action_window(np.array([-0.9]), 0.99, -0.99, 2000, 2000, 1000)
    assert w2[0] == -0.9


def test_nan_guard():
    from rlmd_amd.scripts.rl_multiplicative import NaNLearning, critic_learning

    loss = [1.0] * 11
    critic_learning(600, 512, loss)
    critic_learning(100, 512, [np.nan] * 11)  # before the first real update: no check
    loss[9] = np.nan
    with pytest.raises(NaNLearning):
        critic_learning(600, 512, loss)
    loss = [1.0] * 11
    loss[6] = np.nan  # the shadow-mean slots are not part of the guard
    critic_learning(600, 512, loss)
