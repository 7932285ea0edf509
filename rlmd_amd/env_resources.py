"""Host-side market slicing of the single-stream market driver.

tools/env_resources.py:203-291 (the functions scripts/rl_market.py calls per
episode): ``time_slice`` draws an episode's start row, ``shuffle_data``
permutes the extract's rows inside consecutive blocks (the tail block too),
``observed_market_state`` reads the observation of one time step.  They draw
from NumPy's global generator in the reference's order (one ``randint`` per
slice, one ``permutation`` per block), so a seeded run consumes the stream as
the reference does.  The vectorised loop does the same on the device (Philox
starts and in-block Fisher-Yates, env.hip ``market_row``).
"""
import numpy as np


def time_slice(prices, extract_days, action_days, sample_days):
    """(prices[start : start + extract_days * action_days + 1], start) with
    start ~ U{0, ..., days - sample_days - 1} (env_resources.py:229-254)."""
    start = np.random.randint(0, prices.shape[0] - sample_days)
    return prices[start:start + extract_days * action_days + 1], start


def shuffle_data(prices, interval_days):
    """Rows permuted independently inside each block of interval_days, then the
    remainder block (env_resources.py:257-291); float64 output."""
    n = prices.shape[0]
    out = np.empty((n, prices.shape[1]))
    full = n // interval_days
    for b in range(full):
        lo = b * interval_days
        out[lo:lo + interval_days] = np.random.permutation(prices[lo:lo + interval_days])
    if n % interval_days:
        out[full * interval_days:] = np.random.permutation(prices[full * interval_days:])
    return out


def observed_market_state(market_extract, time_step, action_days, obs_days):
    """Row time_step * action_days (obs_days 1), else the obs_days rows from
    there flattened and reversed (env_resources.py:203-226)."""
    r0 = time_step * action_days
    if obs_days == 1:
        return market_extract[r0]
    return market_extract[r0:r0 + obs_days].reshape(-1)[::-1]
