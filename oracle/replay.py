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


class MultiStepRing:
    """Multi-step replay (tools/replay.py:93-332, ReplayBuffer with multi_steps > 1)
    restated for `lanes` independent transition streams sharing one ring.

    Transition p of lane l lives at row (p * lanes + l) % capacity (the rows the
    fused env step writes).  Each row is tagged with its lane-local position p,
    the ordinal j of its episode and that episode's start position; each lane
    keeps its finished-episode count m, the start of its in-progress episode and
    the end d0 of its first episode.  Episode ends are the stored done flags
    (learn_done, as the reference stores).  For a sampled row (s, j, a_j) the
    reference's history (_episode_history + _construct_history) is the lane-local
    position range [lo, b]:
      j == 0          episode 0:                lo = 0,   b = s
      0 < j < m       a finished episode:       lo = a_j, b = s if done[s] else s + 1
                      (the history slice is one step ahead, capped at the episode end)
      j == m > 0      the in-progress episode:  lo = 0,   b = min(s - a_j + 1, d0)
                      (its history is missing, episode 0's is used instead)
    eff = min(b - lo + 1, n); with f = b - eff + 1 the sample is
      reward  sum (dynamics "A") or product (otherwise) of gamma^t r[f + t], t < eff - 1
              (empty sum 0, empty product 1)
      state   next_state[f], action action[f]      (histories hold next states)
      next_state, done of the sampled row itself; the target bootstraps with gamma^eff.
    Valid while no needed row has been overwritten (the reference requires
    buffer >= cumulative steps, tools/replay.py:163)."""

    def __init__(self, capacity, S, A, lanes, n_steps, dynamics="A", gamma=0.99):
        assert capacity % lanes == 0
        self.C, self.S, self.A, self.L, self.n = capacity, S, A, lanes, n_steps
        self.additive, self.gamma = dynamics == "A", float(gamma)
        self.state = np.zeros((capacity, S))
        self.next_state = np.zeros((capacity, S))
        self.action = np.zeros((capacity, A))
        self.reward = np.zeros(capacity)
        self.done = np.zeros(capacity, bool)
        self.tag = np.zeros((capacity, 3), np.int64)  # pos, episode ordinal, episode start
        self.lane_pos = np.zeros(lanes, np.int64)
        self.lane_m = np.zeros(lanes, np.int64)
        self.lane_start = np.zeros(lanes, np.int64)
        self.lane_d0 = np.full(lanes, -1, np.int64)
        self.mem_idx = 0

    def row(self, lane, pos):
        return (pos * self.L + lane) % self.C

    def insert(self, s, a, r, s2, done):
        """One transition for each of the first k lanes (k <= lanes, in lane order
        of the global stream: transition i goes to lane (mem_idx + i) % lanes)."""
        s, a, s2 = (np.atleast_2d(np.asarray(x, float)) for x in (s, a, s2))
        r, done = np.atleast_1d(np.asarray(r, float)), np.atleast_1d(np.asarray(done, bool))
        for i in range(len(r)):
            g = self.mem_idx + i
            lane, row = g % self.L, g % self.C
            p = self.lane_pos[lane]
            self.state[row], self.action[row], self.reward[row] = s[i], a[i], r[i]
            self.next_state[row], self.done[row] = s2[i], done[i]
            self.tag[row] = (p, self.lane_m[lane], self.lane_start[lane])
            if done[i]:
                if self.lane_m[lane] == 0:
                    self.lane_d0[lane] = p
                self.lane_m[lane] += 1
                self.lane_start[lane] = p + 1
            self.lane_pos[lane] = p + 1
        self.mem_idx += len(r)

    def history_range(self, row):
        lane = row % self.L
        s, j, a_j = self.tag[row]
        m, d0 = self.lane_m[lane], self.lane_d0[lane]
        if j == 0:
            return lane, 0, s
        if j < m:
            return lane, a_j, (s if self.done[row] else s + 1)
        return lane, 0, min(s - a_j + 1, d0)

    def gather(self, rows):
        rows = np.asarray(rows, np.int64)
        B = len(rows)
        rew, eff = np.zeros(B), np.zeros(B, np.int64)
        st, ac = np.zeros((B, self.S)), np.zeros((B, self.A))
        for i, row in enumerate(rows):
            lane, lo, b = self.history_range(row)
            e = min(b - lo + 1, self.n)
            f = b - e + 1
            terms = [self.gamma ** t * self.reward[self.row(lane, f + t)] for t in range(e - 1)]
            if self.additive:
                acc = 0.0
                for x in terms:
                    acc += x
            else:
                acc = 1.0
                for x in terms:
                    acc *= x
            rew[i], eff[i] = acc, e
            st[i] = self.next_state[self.row(lane, f)]
            ac[i] = self.action[self.row(lane, f)]
        return rew, st, ac, self.next_state[rows], self.done[rows], eff
