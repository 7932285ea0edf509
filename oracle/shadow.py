"""Power-law shadow means of the critic losses — TEST INFRASTRUCTURE (see oracle/__init__.py).

Restates tools/utils.py:374-400 (shadow_means) and :441-471 (agent_shadow_mean)
with the dtype flow the reference has on learn()'s float32 loss entries
(algo_sac.py:502-514): every product, exp and pow is float32; SciPy's gamma and
gammaincc (float32 loops: double evaluation, one rounding) come from SciPy
itself here.  Pinned by tests/golden/shadow.npz (the reference's outputs).
"""
import numpy as np
import scipy.special as sp

F32 = np.float32


def shadow_means(alpha, mn, mx, low_mul, high_mul, dtype=F32):
    """shadow_means on scalars of `dtype` (float32: learn()'s loss entries;
    float64: Python-float inputs); low_mul / high_mul are Python floats (weak)."""
    T = dtype
    alpha, mn, mx = T(alpha), T(mn), T(mx)
    low, high = mn * T(low_mul), mx * T(high_mul)
    x = alpha / high
    a1 = np.float64(T(1) - alpha)
    up = T(sp.gamma(a1)) * T(sp.gammaincc(a1, np.float64(x)))
    with np.errstate(all="ignore"):
        return low + (high - low) * np.exp(x) * x**alpha * up


def agent_shadow_mean(loss, low_mul=1.0, high_mul=10.0):
    """[shadow1, shadow2] from one loss[11] row: the empirical mean when alpha >= 1."""
    out = []
    for c in (0, 1):
        a = F32(loss[8 + c])
        out.append(shadow_means(a, loss[2 + c], loss[4 + c], low_mul, high_mul) if a < 1 else F32(loss[c]))
    return np.array(out, dtype=np.float32)


def shadow_equiv(mean, alpha, mn, mx, min_mul=1):
    """tools/utils.py:406-438 on float64 scalars: SciPy's MINPACK hybrd root of
    shadow_means(alpha, min, max, min_mul, m) - mean from m = 1 (the published
    algorithm the reference calls); 1 when alpha >= 1."""
    import scipy.optimize as op

    if alpha < 1:
        f = lambda m: np.atleast_1d(  # noqa: E731  (hybrd hands over m as a 1-element array)
            shadow_means(alpha, mn, mx, min_mul, float(np.ravel(m)[0]), dtype=np.float64) - mean)
        return float(np.atleast_1d(op.root(f, 1, method="hybr").x)[0])
    return 1.0
