"""CPU restatement of the experience-replay wrapper, one env.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the GPU replay kernel (csrc/qs_replay.h).

Follows gym_art/quadrotor_multi/quad_experience_replay.py (ReplayBuffer :16-63, ExperienceReplayWrapper
:66-216) plus the env-side bookkeeping it relies on (quadrotor_multi.py:182-185 state, :382-388
can_drones_fly, :461-465 reset accounting, :722-725 crash accumulation, :836 in-env reset on done).
Pinned to the reference by tests/golden/replay_*.npz (tools/gen_golden_replay.py runs the reference's own
wrapper class over a scripted stand-in env).

Storage is expressed the way the GPU holds it, so the kernel's integer state can be compared field by
field: the checkpoint deque is a ring of `keep` slots (ck_head = next write, ck_n = length); the
replay buffer's deque is `perm` (buffer position -> physical slot, a permutation of range(bufsz):
positions < buf_n are the deque in order, the rest are free slots) with `nrep` per physical slot.
ReplayBuffer.cleanup's rebuild is a stable partition of perm.  `tok_ck` / `tok_buf` hold whatever the
caller uses as the env state token (reference state ids, or GPU snapshot step indices).
"""
from collections import deque

import numpy as np

LAST_ADD_NONE = -1000000000   # last_tick_added_to_buffer = -1e9 (quad_experience_replay.py:91, :195)


class TapeDraws:
    """The reference's draws in call order: self.rng.uniform(0, 1) (:197), random.randint(0, len - 1) (:43)."""

    def __init__(self, tape):
        self.tape, self.pos = np.asarray(tape, dtype=np.float64), 0

    def _next(self):
        v = float(self.tape[self.pos])
        self.pos += 1
        return v

    def u(self):
        return self._next()

    def index(self, n):
        return int(np.floor(self._next() * n))


class FixedDraws:
    """Two uniforms of the GPU's Philox stream (S_REPLAY words 0, 1) for one new_episode."""

    def __init__(self, u, v):
        self._u, self._v = float(u), float(v)

    def u(self):
        return self._u

    def index(self, n):
        return int(np.floor(self._v * n))


class ReplayOracle:
    def __init__(self, prob, cp_every, grace, gap, bufsz=20, keep=6, steps_ago=3, max_rep=10, hist_len=100,
                 hist_min=10):
        self.prob, self.cp_every, self.grace, self.gap = prob, cp_every, grace, gap
        self.bufsz, self.keep, self.steps_ago, self.max_rep = bufsz, keep, steps_ago, max_rep
        self.hist_min = hist_min
        # env attributes (quadrotor_multi.py:178-185)
        self.active, self.saved = 0, 0
        self.hist, self.crash = deque([], maxlen=hist_len), 0.0
        # wrapper attributes (quad_experience_replay.py:86-95)
        self.ck_n, self.ck_head = 0, 0
        self.buf_n, self.buf_idx = 0, 0
        self.perm = list(range(bufsz))
        self.nrep = [0] * bufsz
        self.last_add = LAST_ADD_NONE
        self.episodes, self.replayed, self.index_err = 0, 0, 0
        self.last_slot = -1
        self.tok_ck = [None] * keep
        self.tok_buf = [None] * bufsz

    # ---- QuadrotorEnvMulti side ----
    def _can_fly(self):   # quadrotor_multi.py:382-388
        return int(len(self.hist) >= self.hist_min and abs(float(np.mean(self.hist))) < 1)

    def _env_reset(self):   # quadrotor_multi.py:461-465
        if not self.active:
            self.hist.append(self.crash)
            self.active = self._can_fly()
            self.crash = 0.0

    def explicit_reset(self):
        """ExperienceReplayWrapper.reset -> env.reset (quad_experience_replay.py:109-122)."""
        self._env_reset()

    # ---- one wrapper step (quad_experience_replay.py:124-180) ----
    def step(self, tick, done, col, floor0, crash_unit, draws, live_token):
        """tick: env tick after the step (pre-reset); crash_unit: dt * crash coefficient.
        Returns (token, restored): the token whose observation the wrapper returns instead of the live one
        (None: the live obs), and whether the env state itself was replaced by it (a replayed episode).
        A step that writes a collision event returns the event checkpoint's obs with restored=False: the
        reference rebinds `obs` to the checkpoint's (quad_experience_replay.py:175) and returns it (:180)
        while the env keeps its live state."""
        self.last_slot = -1
        self.pushed_slot = -1
        if not self.active:   # :724-725 crashes_last_episode += rew_crash of agent 0
            self.crash += -crash_unit * float(bool(floor0))
        if done:
            self._env_reset()           # the in-env reset (quadrotor_multi.py:836)
            return self._new_episode(draws)
        if self.active and not self.saved and tick % self.cp_every == 0:   # :157-159
            s = self.ck_head
            self.tok_ck[s] = live_token
            self.ck_head = (s + 1) % self.keep
            self.ck_n = min(self.ck_n + 1, self.keep)
        if col and self.active and tick > self.grace and not self.saved:   # :161-164
            if tick - self.last_add > self.gap:                          # :166
                if self.steps_ago > self.ck_n:                           # :171-173 (IndexError)
                    self.index_err += 1
                else:
                    src = (self.ck_head - self.steps_ago) % self.keep    # episode_checkpoints[-steps_ago]
                    if self.buf_n < self.bufsz:                          # write_cp_to_buffer :24-36
                        pos = self.buf_n
                        self.buf_n += 1
                    else:
                        pos = self.buf_idx
                    phys = self.perm[pos]
                    self.tok_buf[phys] = self.tok_ck[src]
                    self.nrep[phys] = 0
                    self.buf_idx = (self.buf_idx + 1) % self.bufsz
                    self.last_add = tick
                    self.pushed_slot = phys
                    return self.tok_ck[src], False
        return None, False

    def _new_episode(self, draws):   # :182-216
        self.episodes += 1
        self.last_add = LAST_ADD_NONE
        self.ck_n, self.ck_head = 0, 0
        u = draws.u()
        if u < self.prob and self.buf_n > 0 and self.active:
            self.replayed += 1
            pos = draws.index(self.buf_n)                                # sample_event :38-45
            phys = self.perm[pos]
            self.nrep[phys] += 1
            tok = self.tok_buf[phys]
            self.saved = 1   # the stored copy had saved_in_replay_buffer = True (:26)
            keep = [p for p in self.perm[:self.buf_n] if self.nrep[p] < self.max_rep]    # cleanup :47-54
            drop = [p for p in self.perm[:self.buf_n] if self.nrep[p] >= self.max_rep]
            self.perm = keep + drop + self.perm[self.buf_n:]
            self.buf_n = len(keep)
            self.last_slot = phys
            return tok, True
        self._env_reset()   # env.reset() (:209)
        self.saved = 0
        return None, False

    # views used by the tests
    def ck_tokens(self):
        """episode_checkpoints in deque order (oldest first)."""
        return [self.tok_ck[(self.ck_head - self.ck_n + i) % self.keep] for i in range(self.ck_n)]

    def buf_tokens(self):
        return [self.tok_buf[p] for p in self.perm[:self.buf_n]]

    def buf_nrep(self):
        return [self.nrep[p] for p in self.perm[:self.buf_n]]
