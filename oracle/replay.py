"""Replay sampling restatement — TEST INFRASTRUCTURE (see oracle/__init__.py).

Reference: tools/replay.py:334-376 / tools/replay_torch.py:360-412 draw B
DISTINCT uniform indices over the filled ring (np.random.choice(max_mem, B,
replace=False) / randperm(max_mem)[:B]).  rlmd_amd draws them from Philox with
rounds of redraws for duplicates (rlmd_amd/csrc/replay.hip); this module
restates those rounds so a device sample can be checked index for index.
"""
import numpy as np

from . import philox as px


SORT_POPULATION = 8192


def sample_indices(seed, ctr, M, B, max_rounds=64):
    ctr = int(ctr)
    c1 = ctr & 0xFFFFFFFF
    c2 = px.TAG_REPLAY_IDX | ((ctr >> 32) << 8)
    if M <= SORT_POPULATION:
        # B smallest of (random32 << 32 | index) over the population
        e = np.arange(M)
        v = px.philox(seed, e, c1, c2, 0xFFFFFFFF)
        keys = (v[0].astype(np.uint64) << np.uint64(32)) | e.astype(np.uint64)
        return np.sort(keys)[:B].astype(np.uint64) & np.uint64(0xFFFFFFFF)
    slots = np.arange(B)
    v = px.philox(seed, slots, c1, c2, 0)
    cand = px.below(v[0], v[1], M)
    for rnd in range(1, max_rounds + 1):
        order = np.lexsort((slots, cand))  # sort by (index, slot)
        sc = cand[order]
        dup = np.zeros(B, bool)
        dup[1:] = sc[1:] == sc[:-1]
        redraw = order[dup]
        if redraw.size == 0:
            break
        v = px.philox(seed, redraw, c1, c2, rnd)
        cand = cand.copy()
        cand[redraw] = px.below(v[0], v[1], M)
    return cand


def ring_rows(mem_idx_before, n, capacity):
    """Rows a batch of n transitions occupies (store_exp at mem_idx % mem_size)."""
    return (mem_idx_before + np.arange(n)) % capacity
