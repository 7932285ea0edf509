"""Philox4x32-10 and the draw transforms of rlmd_amd/csrc/rlmd_common.h, in NumPy.

TEST INFRASTRUCTURE (see oracle/__init__.py).  The generator core is the
standard Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123), pinned
by its published known-answer vectors in tests/test_oracle_golden.py.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)

TAG_ENV_DRAW = 1
TAG_WARMUP_ACTION = 2
TAG_ACT_NOISE = 3
TAG_REPLAY_IDX = 4
TAG_EPS_NEXT = 5
TAG_EPS_CUR = 6
TAG_TD3_TARGET = 7
TAG_MKT_START = 8
TAG_MKT_PERM = 9


def philox(seed, c0, c1, c2, c3):
    """Vectorised Philox4x32-10; counters broadcast; returns 4 uint32 arrays."""
    seed = int(seed)
    k0 = np.uint32(seed & 0xFFFFFFFF)
    k1 = np.uint32((seed >> 32) & 0xFFFFFFFF)
    x0, x1, x2, x3 = np.broadcast_arrays(*(np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3)))
    x0, x1, x2, x3 = (a.astype(np.uint64) for a in (x0, x1, x2, x3))
    with np.errstate(over="ignore"):
        for r in range(10):
            if r:
                k0 = np.uint32(k0 + W0)
                k1 = np.uint32(k1 + W1)
            p0 = M0 * x0
            p1 = M1 * x2
            hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
            hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
            n0 = hi1 ^ x1 ^ np.uint64(k0)
            n2 = hi0 ^ x3 ^ np.uint64(k1)
            x0, x1, x2, x3 = n0, lo1, n2, lo0
    return tuple(a.astype(np.uint32) for a in (x0, x1, x2, x3))


def u01(a, b):
    """53-bit uniform in [0, 1) from two words (NumPy random_sample construction)."""
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    return ((a >> np.uint64(5)).astype(np.float64) * 67108864.0
            + (b >> np.uint64(6)).astype(np.float64)) * (1.0 / 9007199254740992.0)


def normal2(v):
    """Box–Muller pair of one Philox block: (r cos 2πu2, r sin 2πu2), r = sqrt(-2 ln(1-u1))."""
    u1 = u01(v[0], v[1])
    u2 = u01(v[2], v[3])
    r = np.sqrt(-2.0 * np.log(1.0 - u1))
    return r * np.cos(2.0 * np.pi * u2), r * np.sin(2.0 * np.pi * u2)


def below(a, b, n):
    """Uniform integer in [0, n): high 64 bits of (a<<32|b) * n."""
    x = (np.asarray(a, dtype=np.uint64) << np.uint64(32)) | np.asarray(b, dtype=np.uint64)
    n = int(n)
    # 64x64 -> high 64 via Python ints (exact), vectorised through object arrays
    xo = x.astype(object)
    return np.array([(int(v) * n) >> 64 for v in np.atleast_1d(xo)], dtype=np.int64).reshape(np.shape(x))


def uniform_draws(seed, lanes, step, tag, count):
    """count uniforms per lane: j-th from block j//2 (x,y for even j, z,w for odd)."""
    lanes = np.asarray(lanes)
    out = np.empty((lanes.size, count))
    for blk in range((count + 1) // 2):
        v = philox(seed, lanes, step, tag, blk)
        out[:, 2 * blk] = u01(v[0], v[1])
        if 2 * blk + 1 < count:
            out[:, 2 * blk + 1] = u01(v[2], v[3])
    return out


def normal_draws(seed, lanes, step, tag, count):
    lanes = np.asarray(lanes)
    out = np.empty((lanes.size, count))
    for blk in range((count + 1) // 2):
        z0, z1 = normal2(philox(seed, lanes, step, tag, blk))
        out[:, 2 * blk] = z0
        if 2 * blk + 1 < count:
            out[:, 2 * blk + 1] = z1
    return out
