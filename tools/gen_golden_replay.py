#!/usr/bin/env python
"""Golden fixtures for the experience-replay wrapper.  TEST INFRASTRUCTURE, dev container only.

    python tools/gen_golden_replay.py        # writes tests/golden/replay_*.npz

Runs the reference's own ExperienceReplayWrapper / ReplayBuffer (gym_art/quadrotor_multi/quad_experience_replay.py)
and QuadrotorEnvMulti.can_drones_fly (quadrotor_multi.py:382-388) over a stand-in multi-env that carries
exactly the attributes the wrapper reads, driven by a scripted per-step sequence of (new drone collision,
drone 0 on the floor).  The stand-in restates the env's own replay bookkeeping:
  * quadrotor_multi.py:461-465  reset(): crash history append / activation while not yet active;
  * quadrotor_multi.py:722-725  step(): crashes_last_episode += infos[0]["rewards"]["rew_crash"];
  * quadrotor_multi.py:739, 836 step(): the in-env reset when the episode ends (tick > ep_len).
Every env state gets a unique id (a fresh one per step and per reset) and the observation is
[state id, tick], so deep copies made by the wrapper and restored later are visible in the recorded obs.
The wrapper's draws (self.rng.uniform, random.randint) come from a recorded uniform tape; randint(a, b)
is a + floor(u * (b - a + 1)) of the next tape value, which the oracle replays the same way.
Recorded per step: returned obs, activation / saved flags, checkpoint ids, buffer ids + replay counts,
buffer_idx, last_tick_added_to_buffer, replayed_events, episode_counter.
"""
import contextlib
import io
import os
import sys
from collections import deque

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the shims)

import gym_art.quadrotor_multi.quad_experience_replay as XR  # noqa: E402
from gym_art.quadrotor_multi.quadrotor_multi import QuadrotorEnvMulti  # noqa: E402

OUT = G.OUT


class Tape:
    def __init__(self, seed):
        self.g = np.random.default_rng(seed)
        self.vals = []

    def next(self):
        u = float(self.g.uniform())
        self.vals.append(u)
        return u

    def uniform(self, lo, hi):
        return lo + (hi - lo) * self.next()

    def randint(self, a, b):
        return a + int(np.floor(self.next() * (b - a + 1)))


class Sub:
    def __init__(self, control_freq):
        self.tick = 0
        self.control_freq = control_freq


class Script:
    def __init__(self, col, floor0):
        self.col, self.floor0, self.t = col, floor0, 0


class MockMultiEnv:
    """What ExperienceReplayWrapper reads of QuadrotorEnvMulti (attributes of quadrotor_multi.py:156-185)."""
    can_drones_fly = QuadrotorEnvMulti.can_drones_fly
    _uid = [0]

    def __init__(self, script, ep_len, control_freq, crash_unit, tape):
        self.envs = [Sub(control_freq)]
        self.script, self.ep_len, self.crash_unit = script, ep_len, crash_unit
        self.use_replay_buffer, self.activate_replay_buffer, self.saved_in_replay_buffer = True, False, False
        self.crashes_in_recent_episodes, self.crashes_last_episode = deque([], maxlen=100), 0
        self.last_step_unique_collisions = np.array([], dtype=np.int64)
        self.use_obstacles, self.curr_quad_col = False, []
        self.collisions_grace_period_seconds, self.collision_occurred = 1.5, False
        self.scenes, self.obst_density = None, 0.0
        self.collisions_per_episode = self.collisions_after_settle = 0
        self.obst_quad_collisions_per_episode = self.obst_quad_collisions_after_settle = 0
        self.rng = tape
        self.state_id = self._new_id()

    def __deepcopy__(self, memo):   # the env's state, sharing the script / tape like the real globals
        c = MockMultiEnv.__new__(MockMultiEnv)
        c.__dict__.update(self.__dict__)
        c.envs = [Sub(self.envs[0].control_freq)]
        c.envs[0].tick = self.envs[0].tick
        c.crashes_in_recent_episodes = deque(self.crashes_in_recent_episodes, maxlen=100)
        c.last_step_unique_collisions = self.last_step_unique_collisions.copy()
        return c

    def _new_id(self):
        MockMultiEnv._uid[0] += 1
        return MockMultiEnv._uid[0]

    def obs(self):
        return np.array([self.state_id, self.envs[0].tick], dtype=np.int64)

    def reset(self, obst_density=None, obst_size=None):
        if self.use_replay_buffer and not self.activate_replay_buffer:   # quadrotor_multi.py:462-465
            self.crashes_in_recent_episodes.append(self.crashes_last_episode)
            self.activate_replay_buffer = self.can_drones_fly()
            self.crashes_last_episode = 0
        self.envs[0].tick = 0
        self.state_id = self._new_id()
        return self.obs()

    def step(self, action):
        s = self.script
        col, fl = bool(s.col[s.t]), bool(s.floor0[s.t])
        s.t += 1
        self.envs[0].tick += 1
        self.state_id = self._new_id()
        self.last_step_unique_collisions = np.array([0, 1] if col else [], dtype=np.int64)
        if self.use_replay_buffer and not self.activate_replay_buffer:   # :724-725
            self.crashes_last_episode += -self.crash_unit * float(fl)
        done = self.envs[0].tick > self.ep_len
        obs = self.obs()
        if done:
            obs = self.reset()                                            # :836
        return obs, [0.0], [done], [{"episode_extra_stats": {}}]


def run(name, steps, ep_len, control_freq, crash_unit, col_p, floor_steps, floor_p, seed, col_steps=None):
    rng = np.random.default_rng(seed)
    col = (rng.uniform(size=steps) < col_p) & (np.arange(steps) < (col_steps or steps))
    col = col.astype(np.uint8)
    floor0 = np.where(np.arange(steps) < floor_steps, rng.uniform(size=steps) < floor_p, False).astype(np.uint8)
    tape = Tape(seed + 100)
    XR.random.randint = tape.randint
    env = MockMultiEnv(Script(col, floor0), ep_len, control_freq, crash_unit, tape)
    w = XR.ExperienceReplayWrapper(env, 0.75, 0.0, 0.0)
    rec = {k: [] for k in ["obs", "active", "saved", "ck", "buf", "nrep", "buf_idx", "last_add", "replayed",
                           "episodes", "tape_pos", "live"]}
    with contextlib.redirect_stdout(io.StringIO()):
        obs0 = w.reset()
        for _ in range(steps):
            obs, _, _, _ = w.step(None)
            rec["obs"].append(obs)
            rec["live"].append(w.env.obs())   # the env's own state (differs from obs on an event-write step)
            rec["active"].append(int(w.env.activate_replay_buffer))
            rec["saved"].append(int(w.env.saved_in_replay_buffer))
            ck = [c[0].state_id for c in w.episode_checkpoints]
            rec["ck"].append(ck + [0] * (6 - len(ck)))
            b = [ev.env.state_id for ev in w.replay_buffer.buffer]
            n = [ev.num_replayed for ev in w.replay_buffer.buffer]
            rec["buf"].append(b + [0] * (20 - len(b)))
            rec["nrep"].append(n + [-1] * (20 - len(n)))
            rec["buf_idx"].append(w.replay_buffer.buffer_idx)
            rec["last_add"].append(int(max(w.last_tick_added_to_buffer, -1e9)))
            rec["replayed"].append(w.replayed_events)
            rec["episodes"].append(w.episode_counter)
            rec["tape_pos"].append(len(tape.vals))
    out = {k: np.asarray(v, dtype=np.int64) for k, v in rec.items()}
    out.update(col=col, floor0=floor0, obs0=np.asarray(obs0, dtype=np.int64), tape=np.asarray(tape.vals),
               ep_len=ep_len, control_freq=control_freq, crash_unit=crash_unit, prob=0.75)
    path = os.path.join(OUT, f"replay_{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{path}: {steps} steps, episodes {out['episodes'][-1]}, replayed {out['replayed'][-1]}, "
          f"max buffer {int((out['nrep'] >= 0).sum(1).max())}, tape {len(tape.vals)}")


def main():
    # control_freq 10: checkpoints every 5 ticks, grace 15, gap 50 ticks (the reference's 100 Hz values / 10)
    run("a", steps=12000, ep_len=120, control_freq=10.0, crash_unit=0.02, col_p=0.05, floor_steps=3000,
        floor_p=0.9, seed=7)
    # denser collisions, early activation: the buffer fills, wraps (buffer_idx) and cleanup drops events
    run("b", steps=20000, ep_len=90, control_freq=10.0, crash_unit=0.02, col_p=0.2, floor_steps=0,
        floor_p=0.0, seed=8)
    # collisions only early on, then replays alone: events reach 10 replays and cleanup drops them
    run("c", steps=30000, ep_len=60, control_freq=10.0, crash_unit=0.02, col_p=0.3, floor_steps=0,
        floor_p=0.0, seed=9, col_steps=6000)


if __name__ == "__main__":
    main()
