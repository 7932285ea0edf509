"""Fixed-leverage Monte-Carlo sweeps on the device.

Mirrors lev/lev_exp.py:29-53 (param_range), :128-237 (coin_smart_lev), :586-705
(dice_smart_lev), :1008-1119 (gbm_smart_lev) and :1209-1332 (dice_sh_smart_lev) with
the reference's argument order and return values: `data` [n_lev, 13,
horizon - 1] (mean / mean_top / mean_adj, mad x3, std x3, median x3, lev after
each step) and `data_T` [n_lev, investors] (final values).  The coin sweep runs
in rlmd_lev_coin_sweep (rlmd_amd/csrc/lev.hip: up-count histograms instead of
one sort per (leverage, step)); the die, safe-haven and GBM sweeps, whose values
are not monotone in one count, in rlmd_lev_sweep_sorted (lev_sort.hip: a device
radix sort per (step, leverage)).
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


def _lev_range(lev_low, lev_high, lev_incr, negate):
    """The reference's lev_range tensor (torch f32, negated for dice / dice_sh when
    -down_r > up_r, lev_exp.py:623-624, :1249-1250)."""
    r = torch.tensor([float(x) for x in param_range(float(lev_low), float(lev_high), float(lev_incr))],
                     dtype=torch.float32)
    return -r if negate else r


def _sorted_sweep(kind, dev, outc, inv, hor, top, value_0, table, levs, final_values):
    lib = _abi.lib()
    n_lev = int(levs.numel())
    ws = torch.empty(int(lib.rlmd_lev_sorted_workspace_bytes(int(inv), n_lev)), dtype=torch.uint8, device=dev)
    data = torch.empty((n_lev, 13, hor - 1), dtype=torch.float32, device=dev)
    data_T = torch.empty((n_lev, inv), dtype=torch.float32, device=dev) if final_values else None
    lv = np.ascontiguousarray(levs.numpy(), dtype=np.float32)
    assert table is None or table.dtype == np.float32, "factor table must be the reference's f32 arithmetic"
    tb = None if table is None else np.ascontiguousarray(table, dtype=np.float32)
    P = _abi.ptr
    _abi.check(lib.rlmd_lev_sweep_sorted(kind, P(outc), int(inv), int(hor), outc.stride(0), int(top), float(value_0),
                                         None if tb is None else tb.ctypes.data, lv.ctypes.data, n_lev, P(ws),
                                         ws.numel(), P(data), P(data_T) if data_T is not None else None,
                                         _abi.stream_ptr()))
    return data, data_T


def _categorical(outcomes, inv, hor, dev):
    o = torch.as_tensor(outcomes)
    if tuple(o.shape) != (int(inv), int(hor)):
        raise ValueError("outcomes shape does not match investors x horizon")
    return o.to(device=dev, dtype=torch.uint8).contiguous()


def dice_smart_lev(device, outcomes, investors, horizon, top, value_0, up_r, down_r, mid_r, lev_low, lev_high,
                   lev_incr, final_values=True):
    """lev/lev_exp.py:586-705 on the device (rlmd_lev_sweep_sorted, kind 0):
    outcomes [investors, horizon] in {0 up, 1 down, 2 mid}; the factor of each
    outcome is the reference's f32 torch arithmetic 1 + lev * r."""
    dev = torch.device(device)
    up_r, down_r, mid_r = float(up_r), float(down_r), float(mid_r)  # Python scalars: torch keeps f32
    levs = _lev_range(lev_low, lev_high, lev_incr, -down_r > up_r)
    table = torch.stack([torch.stack([1 + lev * up_r, 1 + lev * down_r, 1 + lev * mid_r]) for lev in levs])
    outc = _categorical(outcomes, investors, horizon, dev)
    return _sorted_sweep(0, dev, outc, int(investors), int(horizon), top, value_0, table.numpy(), levs, final_values)


def dice_sh_smart_lev(device, outcomes, investors, horizon, top, value_0, up_r, down_r, mid_r, sh_up_r, sh_down_r,
                      sh_mid_r, lev_low, lev_high, lev_incr, final_values=True):
    """lev/lev_exp.py:1209-1332 on the device: die + safe haven, factor
    1 + lev * r + (1 - lev) * r_sh per outcome (f32 torch arithmetic)."""
    dev = torch.device(device)
    up_r, down_r, mid_r = float(up_r), float(down_r), float(mid_r)  # Python scalars: torch keeps f32
    sh_up_r, sh_down_r, sh_mid_r = float(sh_up_r), float(sh_down_r), float(sh_mid_r)
    levs = _lev_range(lev_low, lev_high, lev_incr, -down_r > up_r)
    table = torch.stack([torch.stack([1 + lev * up_r + (1 - lev) * sh_up_r, 1 + lev * down_r + (1 - lev) * sh_down_r,
                                      1 + lev * mid_r + (1 - lev) * sh_mid_r]) for lev in levs])
    outc = _categorical(outcomes, investors, horizon, dev)
    return _sorted_sweep(0, dev, outc, int(investors), int(horizon), top, value_0, table.numpy(), levs, final_values)


def gbm_smart_lev(device, outcomes, investors, horizon, top, value_0, lev_low, lev_high, lev_incr,
                  final_values=True):
    """lev/lev_exp.py:1008-1119 on the device (kind 1): outcomes f32 log-returns
    [investors, horizon], factor expf(lev * outcome)."""
    dev = torch.device(device)
    levs = _lev_range(lev_low, lev_high, lev_incr, False)
    o = torch.as_tensor(outcomes, dtype=torch.float32)
    if tuple(o.shape) != (int(investors), int(horizon)):
        raise ValueError("outcomes shape does not match investors x horizon")
    outc = o.to(dev).contiguous()
    return _sorted_sweep(1, dev, outc, int(investors), int(horizon), top, value_0, None, levs, final_values)


# ---------------------------------------------------------------------------
# *_fixed_final_lev: statistics of the values at maturity (rlmd_lev_final_sorted)
# ---------------------------------------------------------------------------
STAT_NAMES = ["mean", "mean_top", "mean_adj", "mad", "mad_top", "mad_adj", "std", "std_top", "std_adj", "med",
              "med_top", "med_adj", "lev"]


def _final(kind, dev, outc, inv, hor, top, value_0, table, levs, verbose):
    lib = _abi.lib()
    n_lev = int(levs.numel())
    ws = torch.empty(int(lib.rlmd_lev_sorted_workspace_bytes(int(inv), n_lev)), dtype=torch.uint8, device=dev)
    stats = torch.empty((n_lev, 13), dtype=torch.float32, device=dev)
    values = torch.empty((n_lev, inv), dtype=torch.float32, device=dev)
    lv = np.ascontiguousarray(levs.numpy(), dtype=np.float32)
    tb = None if table is None else np.ascontiguousarray(table, dtype=np.float32)
    P = _abi.ptr
    _abi.check(lib.rlmd_lev_final_sorted(kind, P(outc), int(inv), int(hor), outc.stride(0), int(top), float(value_0),
                                         None if tb is None else tb.ctypes.data, lv.ctypes.data, n_lev, P(ws),
                                         ws.numel(), P(stats), P(values), _abi.stream_ptr()))
    if verbose:  # the reference's summary lines (lev_exp.py:103-125)
        for row in stats.cpu().numpy():
            m, mt, ma, d, dt, da, s, st, sa, md, mdt, mda, lev = row
            print(f"       lev {lev * 100:1.0f}%:\n"
                  f"                 avg mean/med/mad/std:  $ {m:1.2e} / {md:1.2e} / {d:1.1e} / {s:1.1e}\n"
                  f"                 top mean/med/mad/std:  $ {mt:1.2e} / {mdt:1.2e} / {dt:1.1e} / {st:1.1e}\n"
                  f"                 adj mean/med/mad/std:  $ {ma:1.2e} / {mda:1.2e} / {da:1.1e} / {sa:1.1e}")
    return stats, values


def coin_fixed_final_lev(device, outcomes, top, value_0, up_r, down_r, lev_low, lev_high, lev_incr, verbose=False):
    """lev/lev_exp.py:56-127: statistics of value_0 * prod(1 + lev * r) per leverage
    (outcome 1 up, else down).  Returns (stats [n_lev, 13] in STAT_NAMES order,
    final values [n_lev, investors]); the reference prints the statistics only."""
    dev = torch.device(device)
    up_r, down_r = float(up_r), float(down_r)
    levs = _lev_range(lev_low, lev_high, lev_incr, -down_r > up_r)
    table = torch.stack([torch.stack([1 + lev * down_r, 1 + lev * up_r, 1 + lev * up_r]) for lev in levs])
    o = torch.as_tensor(outcomes)
    inv, hor = o.shape
    outc = (o == 1).to(device=dev, dtype=torch.uint8).contiguous()
    return _final(0, dev, outc, inv, hor, top, value_0, table.numpy(), levs, verbose)


def dice_fixed_final_lev(device, outcomes, top, value_0, up_r, down_r, mid_r, lev_low, lev_high, lev_incr,
                         verbose=False):
    """lev/lev_exp.py:508-585 (outcomes {0 up, 1 down, 2 mid})."""
    dev = torch.device(device)
    up_r, down_r, mid_r = float(up_r), float(down_r), float(mid_r)
    levs = _lev_range(lev_low, lev_high, lev_incr, -down_r > up_r)
    table = torch.stack([torch.stack([1 + lev * up_r, 1 + lev * down_r, 1 + lev * mid_r]) for lev in levs])
    o = torch.as_tensor(outcomes)
    inv, hor = o.shape
    return _final(0, dev, _categorical(o, inv, hor, dev), inv, hor, top, value_0, table.numpy(), levs, verbose)


def dice_sh_fixed_final_lev(device, outcomes, top, value_0, up_r, down_r, mid_r, sh_up_r, sh_down_r, sh_mid_r,
                            lev_low, lev_high, lev_incr, verbose=False):
    """lev/lev_exp.py:1121-1208 (die + safe haven)."""
    dev = torch.device(device)
    up_r, down_r, mid_r = float(up_r), float(down_r), float(mid_r)
    sh_up_r, sh_down_r, sh_mid_r = float(sh_up_r), float(sh_down_r), float(sh_mid_r)
    levs = _lev_range(lev_low, lev_high, lev_incr, -down_r > up_r)
    table = torch.stack([torch.stack([1 + lev * up_r + (1 - lev) * sh_up_r, 1 + lev * down_r + (1 - lev) * sh_down_r,
                                      1 + lev * mid_r + (1 - lev) * sh_mid_r]) for lev in levs])
    o = torch.as_tensor(outcomes)
    inv, hor = o.shape
    return _final(0, dev, _categorical(o, inv, hor, dev), inv, hor, top, value_0, table.numpy(), levs, verbose)


def gbm_fixed_final_lev(device, outcomes, top, value_0, lev_low, lev_high, lev_incr, verbose=False):
    """lev/lev_exp.py:935-1007: factors exp(lev * outcome)."""
    dev = torch.device(device)
    levs = _lev_range(lev_low, lev_high, lev_incr, False)
    o = torch.as_tensor(outcomes, dtype=torch.float32)
    inv, hor = o.shape
    return _final(1, dev, o.to(dev).contiguous(), inv, hor, top, value_0, None, levs, verbose)


def coin_galaxy_brain_lev(device, ru_min, ru_max, ru_incr, rd_min, rd_max, rd_incr, pu_min, pu_max, pu_incr):
    """lev/lev_exp.py:455-505: the Kelly fraction pu / rd - (1 - pu) / ru over a
    (pu, ru, rd) grid, [n_pu, n_ru, n_ru, 4] = (pu, ru, rd, kelly) (the reference
    sizes the third axis by ru's grid and fills it from rd's).  A few hundred
    scalars: evaluated on the host in the reference's Python floats, stored f32."""
    ru_range = param_range(ru_min, ru_max, ru_incr)
    rd_range = param_range(rd_min, rd_max, rd_incr)
    pu_range = param_range(pu_min, pu_max, pu_incr)
    data = torch.zeros((len(pu_range), len(ru_range), len(ru_range), 4))
    for i, pu in enumerate(pu_range):
        for j, ru in enumerate(ru_range):
            for k, rd in enumerate(rd_range):
                data[i, j, k, :] = torch.tensor([pu, ru, rd, pu / rd - (1 - pu) / ru])
    return data.to(torch.device(device))


# ---------------------------------------------------------------------------
# *_big_brain_lev: investors that re-lever from their own value every step
# ---------------------------------------------------------------------------
def _brain(device, codes, inv, hor, top, value_0, rets3, lev_factor, stops, rolls, f64):
    dev = torch.device(device)
    lf = torch.as_tensor(lev_factor, dtype=torch.float32).reshape(())
    cfg = []
    for roll in rolls:  # roll-major, as the reference's data[j = roll, i = stop]
        for stop in stops:
            value_min = stop * value_0
            v0 = torch.tensor(value_0, dtype=torch.float32)
            # optimal leverage at value_0 (lev_exp.py:240-267, :704-738): the floor is
            # value_min either way (value_t <= value_0)
            lev0 = lf * (1 - value_min / v0)
            cfg.append([float(value_min), float(roll), float(lev0), 1.0 if float(roll) != 0 else 0.0, float(stop)])
    cfg = np.ascontiguousarray(cfg, dtype=np.float32)
    n_cfg = len(cfg)
    lib = _abi.lib()
    ws = torch.empty(int(lib.rlmd_lev_brain_workspace_bytes(int(inv), n_cfg)), dtype=torch.uint8, device=dev)
    data = torch.empty((len(rolls), len(stops), 26, hor - 1), dtype=torch.float32, device=dev)
    # coin: T.where(outcomes == 1, up_r, down_r) is f32; dice's outcomes are f64
    r3 = np.ascontiguousarray([float(r) if f64 else float(np.float32(r)) for r in rets3], dtype=np.float64)
    P = _abi.ptr
    _abi.check(lib.rlmd_lev_brain(1 if f64 else 0, P(codes), int(inv), int(hor), codes.stride(0), int(top), float(value_0),
                                  r3.ctypes.data, float(lf), cfg.ctypes.data, n_cfg, P(ws), ws.numel(), P(data),
                                  _abi.stream_ptr()))
    return data


def coin_big_brain_lev(device, outcomes, investors, horizon, top, value_0, up_r, down_r, lev_factor, stop_min,
                       stop_max, stop_incr, roll_min, roll_max, roll_incr):
    """lev/lev_exp.py:270-452 on the device (rlmd_lev_brain): data [n_roll,
    n_stop, 26, horizon - 1] = value statistics (rows 0-11), leverage statistics
    (12-23), stop, roll.  Outcome 1 up (return up_r), else down_r.  With a
    retention ratio > 0 the reference's coin_optimal_lev is handed the Python
    float value_0 for the first leverage and torch.where rejects its bool
    condition (TypeError); the build applies dice_optimal_lev's reading (the
    floor at value_0 is the stop-loss), which the reference uses for dice."""
    dev = torch.device(device)
    stops = torch.tensor(param_range(stop_min, stop_max, stop_incr), dtype=torch.float32)
    rolls = torch.tensor(param_range(roll_min, roll_max, roll_incr), dtype=torch.float32)
    o = torch.as_tensor(outcomes)
    codes = (o == 1).to(device=dev, dtype=torch.uint8).contiguous()  # code 0 down, 1 up
    return _brain(dev, codes, int(investors), int(horizon), top, value_0, [float(down_r), float(up_r), float(up_r)],
                  lev_factor, stops, rolls, False)


def dice_big_brain_lev(device, outcomes, investors, horizon, top, value_0, up_r, down_r, mid_r, lev_factor, stop_min,
                       stop_max, stop_incr, roll_min, roll_max, roll_incr):
    """lev/lev_exp.py:741-932 on the device: outcomes {0 up, 1 down, 2 mid}; the
    reference casts them to float64 (:751), so values are f64 (see rlmd_lev_brain)."""
    dev = torch.device(device)
    stops = torch.tensor(param_range(stop_min, stop_max, stop_incr), dtype=torch.float32)
    rolls = torch.tensor(param_range(roll_min, roll_max, roll_incr), dtype=torch.float32)
    codes = _categorical(outcomes, investors, horizon, dev)
    return _brain(dev, codes, int(investors), int(horizon), top, value_0, [float(up_r), float(down_r), float(mid_r)],
                  lev_factor, stops, rolls, True)
