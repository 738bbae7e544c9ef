#!/usr/bin/env python
"""Golden fixtures for the flavor-B goal scenarios.  TEST INFRASTRUCTURE, dev container only.

    python tools/gen_golden_scen.py        # writes tests/golden/scen_*.npz

Runs the reference's own scenario classes (gym_art/quadrotor_multi/scenarios/*.py, created through
scenarios/mix.py:create_scenario like QuadrotorEnvMulti does) on stand-in sub-envs that carry exactly the
attributes the scenarios read (tick, box, control_freq, use_obstacles, goal), and records:
  * every draw in call order ("tape"): the env Generator's integers / uniform (any size, flattened) and
    shuffle (recorded as the permutation it applied), and np.random.uniform / randint;
  * the goals after reset() and after every step() (ticks 1..T), plus the scenario attributes.
The oracle (oracle/quadswarm_oracle_scen.c) replays the tape and must reproduce the goals.

Harness-side stand-ins (third-party code absent from the image):
  * bezier.Curve(nodes, degree=2).evaluate_multi -- the `bezier` package's Bernstein evaluation
    (evaluate_multi_barycentric), restated here;
  * Generator.shuffle is replaced by a permutation draw applied to the rows (same distribution; the
    permutation is what the tape records, so the oracle needs no numpy shuffle internals).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the shims; its np.random tape stays off here)

OUT = G.OUT
TAPE = []
ON = [False]


def _rec(v):
    if ON[0]:
        TAPE.extend(np.ravel(np.asarray(v, dtype=np.float64)).tolist())
    return v


_np_uniform, _np_randint = np.random.uniform, np.random.randint
np.random.uniform = lambda *a, **k: _rec(_np_uniform(*a, **k))
np.random.randint = lambda *a, **k: _rec(_np_randint(*a, **k))


class Curve:
    """bezier.Curve stand-in: degree-2 Bernstein form as bezier's evaluate_multi_barycentric computes it."""

    def __init__(self, nodes, degree):
        self.nodes = np.asarray(nodes, dtype=np.float64)
        self.degree = degree

    def evaluate_multi(self, s):
        l1, l2 = (1.0 - s)[None, :], np.asarray(s)[None, :]
        n = self.nodes
        r = l1 * n[:, [0]]
        r = r + 2.0 * l2 * n[:, [1]]
        r = r * l1
        return r + l2 * l2 * n[:, [2]]


import bezier  # noqa: E402  (the empty stand-in module from tools/refshim.py)

bezier.Curve = Curve


class RecGen:
    """Records the env Generator's draws in call order."""

    def __init__(self, g):
        self.g = g

    def integers(self, *a, **k):
        return _rec(self.g.integers(*a, **k))

    def uniform(self, *a, **k):
        return _rec(self.g.uniform(*a, **k))

    def shuffle(self, x):
        perm = self.g.permutation(len(x))
        x[:] = np.asarray(x)[perm]
        _rec(perm)


class SubEnv:
    """The attributes of QuadrotorSingle the scenarios read (box 2.0 quadrotor_single.py:218, control_freq
    sim_freq / sim_steps = 100)."""

    def __init__(self):
        self.tick, self.box, self.control_freq, self.use_obstacles, self.goal = 0, 2.0, 100.0, False, None


import gym_art.quadrotor_multi.scenarios.mix as MIX  # noqa: E402

ATTRS = ["formation_size", "lowest_formation_size", "highest_formation_size", "layer_dist", "control_step_for_sec",
         "control_speed", "increase_formation_size", "num_agents_per_layer"]


def run(mode, n, T, seed, resets=1, record_every_step=True):
    """One scenario object per reset (like Scenario_mix.reset); goals recorded after reset and steps."""
    rng = RecGen(np.random.default_rng(seed))
    np.random.seed(seed + 1)
    envs = [SubEnv() for _ in range(n)]
    tapes, tape_len, goals, ticks, mode_ids = [], [], [], [], []
    del TAPE[:]
    ON[0] = True
    for rr in range(resets):
        start = len(TAPE)
        if mode == "mix":
            sc = MIX.Scenario_mix("mix", envs, n, [10, 10, 10], rng)
            sc.reset()
            actual = type(sc.scenario).__name__[len("Scenario_"):]
        else:
            sc = MIX.create_scenario(mode, envs, n, [10, 10, 10], rng)
            sc.reset()
            actual = mode
        mode_ids.append(MODES.index(actual))
        for i, e in enumerate(envs):
            e.goal = np.array(sc.goals[i], dtype=np.float64)
            e.tick = 0
        goals.append(np.array([e.goal for e in envs]))
        ticks.append(0)
        prev = goals[-1]
        for t in range(1, T + 1):
            for e in envs:
                e.tick = t
            sc.step()
            cur = np.array([np.asarray(e.goal, dtype=np.float64) for e in envs])
            if record_every_step or not np.array_equal(cur, prev):
                goals.append(cur)
                ticks.append(t)
            prev = cur
        tapes.append(start)
        tape_len.append(len(TAPE) - start)
    ON[0] = False
    return dict(tape=np.array(TAPE), reset_tape_start=np.array(tapes), reset_tape_len=np.array(tape_len),
                goals=np.stack(goals), ticks=np.array(ticks), modes=np.array(mode_ids), n=n, T=T)


MODES = ["static_same_goal", "static_diff_goal", "ep_lissajous3D", "ep_rand_bezier", "dynamic_same_goal",
         "dynamic_diff_goal", "dynamic_formations", "swap_goals", "swarm_vs_swarm", "run_away"]


def main():
    os.makedirs(OUT, exist_ok=True)
    out = {}
    # event-driven modes: goals change every 4-6 s (400-600 ticks); record only the changes
    for m, n, seed in [("static_diff_goal", 8, 1), ("dynamic_same_goal", 8, 2), ("dynamic_diff_goal", 8, 3),
                       ("swap_goals", 8, 4), ("swarm_vs_swarm", 8, 5), ("run_away", 8, 6), ("dynamic_diff_goal", 32, 7),
                       ("swarm_vs_swarm", 4, 8), ("swap_goals", 32, 9), ("static_same_goal", 8, 10)]:
        out[f"{m}_n{n}"] = run(m, n, 1300, seed, resets=3, record_every_step=False)
    # per-step modes
    for m, n, seed, T in [("ep_lissajous3D", 4, 11, 300), ("ep_rand_bezier", 4, 12, 1100),
                          ("dynamic_formations", 8, 13, 700), ("dynamic_formations", 5, 14, 400)]:
        out[f"{m}_n{n}"] = run(m, n, T, seed, resets=2, record_every_step=m != "ep_rand_bezier")
    # mix: mode draws over many resets (short episodes), N = 8 and the single-drone list
    out["mix_n8"] = run("mix", 8, 5, 15, resets=60, record_every_step=False)
    out["mix_n1"] = run("mix", 1, 5, 16, resets=30, record_every_step=False)
    for name, d in out.items():
        np.savez_compressed(os.path.join(OUT, f"scen_{name}.npz"), **d)
        print(name, d["goals"].shape, len(d["tape"]), os.path.getsize(os.path.join(OUT, f"scen_{name}.npz")))


if __name__ == "__main__":
    main()
