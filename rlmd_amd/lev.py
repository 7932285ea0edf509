"""Fixed-leverage Monte-Carlo sweeps on the device.

Mirrors lev/lev_exp.py:29-53 (param_range) and :128-237 (coin_smart_lev) with
the reference's argument order and return values: `data` [n_lev, 13,
horizon - 1] (mean / mean_top / mean_adj, mad x3, std x3, median x3, lev after
each step) and `data_T` [n_lev, investors] (final values).  The sweep runs in
rlmd_lev_coin_sweep (rlmd_amd/csrc/lev.hip): up-count histograms instead of
one sort per (leverage, step).
"""
import numpy as np
import torch

from . import _abi


def param_range(low, high, increment):
    """lev/lev_exp.py:29-53: the leverage grid (0 dropped unless it is alone)."""
    lo = int(low / increment)
    hi = int(high / increment + 1)
    mod = low / increment - lo
    params = [(x + mod) * increment for x in range(lo, hi, 1)]
    if 0 in params and len(params) > 1:
        params.remove(0)
    return params


def pack_outcomes(outcomes, device="cuda:0"):
    """[investors, horizon] 0/1 (any dtype) -> device u8 rows padded to 64 steps."""
    o = torch.as_tensor(outcomes)
    inv, hor = o.shape
    ld = (hor + 63) // 64 * 64
    buf = torch.zeros((inv, ld), dtype=torch.uint8, device=device)
    buf[:, :hor] = (o == 1).to(device=device, dtype=torch.uint8)
    return buf, hor


def coin_smart_lev(device, outcomes, investors, horizon, top, value_0, up_r, down_r, lev_low, lev_high, lev_incr,
                   final_values=True):
    """lev_exp.py:128-237 on the device; outcomes may be a torch / NumPy 0/1
    matrix or a (u8 device buffer, horizon) pair from pack_outcomes."""
    dev = torch.device(device)
    buf, hor = outcomes if isinstance(outcomes, tuple) else pack_outcomes(outcomes, dev)
    inv = int(investors)
    if buf.shape[0] != inv or hor != int(horizon):
        raise ValueError("outcomes shape does not match investors x horizon")
    levs = np.array(param_range(lev_low, lev_high, lev_incr), dtype=np.float32)
    n_lev = len(levs)
    lib = _abi.lib()
    ws = torch.empty(int(lib.rlmd_lev_workspace_bytes(inv, hor)), dtype=torch.uint8, device=dev)
    data = torch.empty((n_lev, 13, hor - 1), dtype=torch.float32, device=dev)
    data_T = torch.empty((n_lev, inv), dtype=torch.float32, device=dev) if final_values else None
    P = _abi.ptr
    _abi.check(lib.rlmd_lev_coin_sweep(P(buf), inv, hor, buf.stride(0), int(top), float(value_0), float(up_r),
                                       float(down_r), levs.ctypes.data, n_lev, P(ws), ws.numel(), P(data),
                                       P(data_T) if data_T is not None else None, _abi.stream_ptr()))
    return data, data_T
