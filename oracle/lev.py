"""CPU restatement of the fixed-leverage Monte-Carlo sweep.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of
rlmd_lev_coin_sweep; never called by the product path.

Follows lev/lev_exp.py:29-53 (param_range) and :128-237 (coin_smart_lev),
and (sorted_smart_lev below) :586-705 dice, :1008-1119 GBM, :1209-1332 dice_sh:
for each leverage l (negated when -down_r > up_r), every investor's value
is multiplied step by step by 1 + l*up_r (outcome 1) or 1 + l*down_r (0) in
float32; after each step t >= 1 the values are sorted descending, the first
`top` form the top group and the rest the adjusted group, and the table row
[mean, mean_top, mean_adj, mad, mad_top, mad_adj, std, std_top, std_adj,
 med, med_top, med_adj, lev] is stored (std unbiased=False, median = the
lower middle element, as torch.median).  data_T holds the values after all
`horizon` steps.  Pinned to the reference run on torch CPU
(tests/golden/lev.npz, make_golden.py:lev_fixtures).
"""
import numpy as np


def param_range(low, high, increment):
    """lev/lev_exp.py:29-53."""
    lo = int(low / increment)
    hi = int(high / increment + 1)
    mod = low / increment - lo
    params = [(x + mod) * increment for x in range(lo, hi, 1)]
    if 0 in params and len(params) > 1:
        params.remove(0)
    return params


def _group(v):
    """mean, mad, std, lower median of one group (float32 values, f64 sums)."""
    if v.size == 0:
        return np.nan, np.nan, np.nan, np.nan
    v = v.astype(np.float64)
    m = v.mean()
    return m, np.abs(v - m).mean(), np.sqrt(((v - m) ** 2).mean()), np.sort(v)[(v.size - 1) // 2]


def coin_smart_lev(outcomes, top, value_0, up_r, down_r, lev_low, lev_high, lev_incr):
    """lev/lev_exp.py:128-237 on a [investors, horizon] 0/1 matrix."""
    levs = np.array(param_range(lev_low, lev_high, lev_incr), dtype=np.float32)
    levs = -levs if -down_r > up_r else levs
    inv, hor = outcomes.shape
    data = np.zeros((len(levs), 13, hor - 1), dtype=np.float32)
    data_T = np.zeros((len(levs), inv), dtype=np.float32)
    up = outcomes == 1
    for i, lev in enumerate(levs):
        gu = np.float32(1) + lev * np.float32(up_r)
        gd = np.float32(1) + lev * np.float32(down_r)
        g = np.where(up, gu, gd).astype(np.float32)
        val = np.float32(value_0) * g[:, 0]
        for t in range(hor - 1):
            val = (val * g[:, t + 1]).astype(np.float32)
            s = np.sort(val)[::-1]
            a, tp, ad = _group(val), _group(s[:top]), _group(s[top:])
            data[i, :, t] = [a[0], tp[0], ad[0], a[1], tp[1], ad[1], a[2], tp[2], ad[2], a[3], tp[3], ad[3], lev]
        data_T[i] = val
    return data, data_T


def sorted_smart_lev(g_of_lev, levs, top, value_0, hor):
    """The shared loop of dice_smart_lev (lev/lev_exp.py:586-705), gbm_smart_lev
    (:1008-1119) and dice_sh_smart_lev (:1209-1332): g_of_lev(lev) -> the f32
    gamble factors [investors, horizon]; sequential f32 products, per-step sort."""
    data = np.zeros((len(levs), 13, hor - 1), dtype=np.float32)
    data_T = None
    for i, lev in enumerate(levs):
        g = g_of_lev(lev)
        if data_T is None:
            data_T = np.zeros((len(levs), g.shape[0]), dtype=np.float32)
        val = (np.float32(value_0) * g[:, 0]).astype(np.float32)
        for t in range(hor - 1):
            val = (val * g[:, t + 1]).astype(np.float32)
            s = np.sort(val)[::-1]
            a, tp, ad = _group(val), _group(s[:top]), _group(s[top:])
            data[i, :, t] = [a[0], tp[0], ad[0], a[1], tp[1], ad[1], a[2], tp[2], ad[2], a[3], tp[3], ad[3], lev]
        data_T[i] = val
    return data, data_T


def _levs(lev_low, lev_high, lev_incr, negate):
    levs = np.array(param_range(lev_low, lev_high, lev_incr), dtype=np.float32)
    return -levs if negate else levs


def dice_smart_lev(outcomes, top, value_0, up_r, down_r, mid_r, lev_low, lev_high, lev_incr):
    """lev/lev_exp.py:586-705 on a [investors, horizon] {0 up, 1 down, 2 mid}
    matrix; factors 1 + lev * r in float32."""
    levs = _levs(lev_low, lev_high, lev_incr, -down_r > up_r)
    f = lambda lev, r: np.float32(1) + lev * np.float32(r)  # noqa: E731
    g = lambda lev: np.where(outcomes == 0, f(lev, up_r), np.where(outcomes == 1, f(lev, down_r),  # noqa: E731
                                                                    f(lev, mid_r))).astype(np.float32)
    return sorted_smart_lev(g, levs, top, value_0, outcomes.shape[1])


def dice_sh_smart_lev(outcomes, top, value_0, up_r, down_r, mid_r, sh_up_r, sh_down_r, sh_mid_r, lev_low, lev_high,
                      lev_incr):
    """lev/lev_exp.py:1209-1332: factors 1 + lev * r + (1 - lev) * r_sh (float32)."""
    levs = _levs(lev_low, lev_high, lev_incr, -down_r > up_r)
    f = lambda lev, r, rs: (np.float32(1) + lev * np.float32(r)) + (np.float32(1) - lev) * np.float32(rs)  # noqa
    g = lambda lev: np.where(outcomes == 0, f(lev, up_r, sh_up_r),  # noqa: E731
                             np.where(outcomes == 1, f(lev, down_r, sh_down_r),
                                      f(lev, mid_r, sh_mid_r))).astype(np.float32)
    return sorted_smart_lev(g, levs, top, value_0, outcomes.shape[1])


def gbm_smart_lev(outcomes, top, value_0, lev_low, lev_high, lev_incr):
    """lev/lev_exp.py:1008-1119: factors exp(lev * outcome) in float32."""
    levs = _levs(lev_low, lev_high, lev_incr, False)
    o = outcomes.astype(np.float32)
    g = lambda lev: np.exp(lev * o).astype(np.float32)  # noqa: E731
    return sorted_smart_lev(g, levs, top, value_0, outcomes.shape[1])


def brain_lev(codes, rets3, top, value_0, lev_factor, stops, rolls, f64=False):
    """coin_big_brain_lev / dice_big_brain_lev (lev/lev_exp.py:270-452, :741-932)
    on outcome codes [investors, horizon] with rets3[code] the step return: per
    (roll, stop) the leverage re-set from each investor's value every step
    (coin_optimal_lev :240-267 / dice_optimal_lev :704-738).  Coin: float32
    throughout.  Dice (f64): the reference casts the outcomes to float64 (:751),
    so values are f64; with roll 0 the leverage is f64 (f32 lev_factor and floor
    against the f64 value), with roll > 0 dice_optimal_lev casts the values to
    float32 first and the leverage is f32."""
    inv, hor = codes.shape
    f = np.float32
    vt = np.float64 if f64 else np.float32
    r = np.asarray(rets3, dtype=vt)[codes]
    lf = f(lev_factor)
    data = np.zeros((len(rolls), len(stops), 26, hor - 1), dtype=np.float32)

    def opt(v, vmin, roll):
        if roll == 0:
            return (vt(lf) * (vt(1) - vt(vmin) / v)).astype(vt)
        vf = v.astype(np.float32)
        loss = np.where(vf <= f(value_0), vmin, f(value_0) + roll * (vf - f(value_0))).astype(np.float32)
        return (lf * (f(1) - loss / vf)).astype(np.float32).astype(vt)

    for j, roll in enumerate(np.asarray(rolls, dtype=np.float32)):
        for i, stop in enumerate(np.asarray(stops, dtype=np.float32)):
            vmin = stop * f(value_0)
            lev0 = lf * (f(1) - vmin / f(value_0))
            val = (vt(value_0) * (vt(1) + vt(lev0) * r[:, 0])).astype(vt)
            lev = opt(val, vmin, roll)
            for t in range(hor - 1):
                sl = np.sort(lev)[::-1]
                a, tp, ad = _group(lev), _group(sl[:top]), _group(sl[top:])
                data[j, i, 12:26, t] = [a[0], tp[0], ad[0], a[1], tp[1], ad[1], a[2], tp[2], ad[2], a[3], tp[3],
                                        ad[3], stop, roll]
                val = (val * (vt(1) + lev * r[:, t + 1])).astype(vt)
                lev = opt(val, vmin, roll)
                s = np.sort(val)[::-1]
                a, tp, ad = _group(val), _group(s[:top]), _group(s[top:])
                data[j, i, 0:12, t] = [a[0], tp[0], ad[0], a[1], tp[1], ad[1], a[2], tp[2], ad[2], a[3], tp[3], ad[3]]
    return data
