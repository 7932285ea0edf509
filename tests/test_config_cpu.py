"""Start-up validation (rlmd_amd.config.learning_tests / env_tests), the
reference's tests/test_input_agent.py:51-406 and :409-584: the default inputs
pass; each bad value below raises AssertionError before any device work, as
main.py:277-280 runs the checks.  main.run calls both first."""
import numpy as np
import pytest

from rlmd_amd import config as c


def folded(envs=(8,), algo=("SAC",), critic=("MSE",), ms=(1,), **over):
    return c.input_initialisation(dict(c.INPUTS, **over), list(envs), list(algo), list(critic), list(ms))


def test_defaults_pass():
    inp = folded(envs=[8, 14, 18], algo=["SAC", "TD3"], critic=c.LOSSES, ms=[1, 3, 5])
    c.learning_tests(inp)
    c.env_tests(c.GYM_ENVS, inp)


BAD = [
    # (override, message fragment)  — test_input_agent.py line of the check
    (dict(algo_name=["PPO"]), "algo_name must be a list"),                          # :64-66
    (dict(algo_name=["SAC", "SAC"]), "unique"),                                     # :70-72
    (dict(critic_loss=["L1"]), "critic_loss must be a list"),                       # :74-76
    (dict(bootstraps=[0]), "positive integers"),                                    # :88-90
    (dict(bootstraps=[1.5]), "type int"),                                           # :79
    (dict(n_cumsteps_mul=12345), "2 leading non-zero digits"),                      # :121-123
    (dict(eval_freq_mul=1e6), "eval_freq_mul must be less than"),                   # :127-129
    (dict(actor_percentile_mul=0), "(0, 100]"),                                     # :136-138
    (dict(n_gambles=[1, 1]), "unique"),                                             # :150-152
    (dict(market_dir="/abs/data/"), "sub-directory relative"),                      # :161-163
    (dict(train_shuffle_days=2000), "train_shuffle_days must be less than"),        # :198-200
    (dict(gap_days_min=30), "gap_days_max must be greater"),                        # :209-211
    (dict(past_days=[]), "at least one"),                                           # :217-219
    (dict(gpu="gpu0"), None),                                                       # :260
    (dict(buffer=1e3), "buffer must be greater than or equal"),                     # :280-291
    (dict(discount=1.0), "discount must be within"),                                # :292-294
    (dict(cauchy_scale=0), "greater than 0"),                                       # :298
    (dict(r_abs_zero="x"), "r_abs_zero"),                                           # :299-301
    (dict(critic_mean_type="S"), "critic_mean_type"),                               # :305-307
    (dict(sac_actor_learn_rate=0), "greater than 0"),                               # :314
    (dict(log_scale_min=3), "SAC scale limits"),                                    # :335-337
    (dict(reparam_noise=1e-3), "reparam_noise"),                                    # :339-341
    (dict(td3_layer_1_units=0), "greater than or equal to 1"),                      # :350
    (dict(target_policy_clip=-0.5), "greater than 0"),                              # :369
    (dict(sample_dist={"SAC": "X", "TD3": "N"}), "SAC sample_dist"),                # :378-382
    (dict(sample_dist={"SAC": "N", "TD3": "MVN"}), "TD3 sample_dist"),              # :384-386
    (dict(batch_size={"SAC": 0, "TD3": 100}), "greater than or equal to 1"),        # :393
    (dict(log_noise=1), "type float"),                                              # :403
]


@pytest.mark.parametrize("over,msg", BAD, ids=[next(iter(o)) + str(i) for i, (o, _) in enumerate(BAD)])
def test_learning_tests_reject(over, msg):
    inp = folded()
    inp.update(over)
    with pytest.raises(AssertionError) as e:
        c.learning_tests(inp)
    if msg:
        assert msg in str(e.value), str(e.value)


def test_env_tests_reject():
    with pytest.raises(AssertionError, match="selected from gym_envs"):
        c.env_tests(c.GYM_ENVS, folded(envs=[3]))                       # :424-426 (additive key)
    inp = folded(envs=[8])
    inp["ENV_KEY"] = 8
    with pytest.raises(AssertionError):
        c.env_tests(c.GYM_ENVS, inp)                                    # :428
    with pytest.raises(AssertionError, match="warm-up must be less"):
        c.env_tests(c.GYM_ENVS, folded(envs=[14], n_cumsteps_mul=1e3))  # :454-458
    with pytest.raises(AssertionError, match="2x evaluation frequency"):
        c.env_tests(c.GYM_ENVS, folded(envs=[18], n_cumsteps_mul=1.5e3, eval_freq_mul=1e3))
    bad = dict(c.GYM_ENVS, **{"8": ["Coin_InvA", 0, 1, 1e3]})
    with pytest.raises(AssertionError, match="at least one state"):
        c.env_tests(bad, folded(envs=[8]))                              # :446-448


def test_env_tests_market_length():
    """:497-581: a market table too short for train + gap + test at past_days."""
    inp = folded(envs=[21], past_days=[1, 5])
    short = lambda key: np.ones((1000 + 250 + 20 + 1, 1))  # enough for obs 1 only
    with pytest.raises(AssertionError, match="greater than sample length"):
        c.env_tests(c.GYM_ENVS, inp, load_market=short)
    c.env_tests(c.GYM_ENVS, folded(envs=[21], past_days=[1]), load_market=short)


def test_main_run_checks_first():
    from rlmd_amd.main import run

    with pytest.raises(AssertionError, match="algo_name"):
        run([8], algo=["PPO"], log=None)
