#!/usr/bin/env python
"""Golden fixtures for the obstacle maps' dynamic scenarios (VERDICT r05 missing #1).  TEST
INFRASTRUCTURE, dev container only.

    python tools/gen_golden_oscen.py        # writes tests/golden/oscen_*.npz

Runs the reference's own Scenario_o_swap_goals / Scenario_o_ep_rand_bezier / Scenario_o_dynamic_same_goal
(gym_art/quadrotor_multi/scenarios/obstacles/*.py, QUADS_MODE_LIST_OBSTACLES_TEST) on stand-in sub-envs that carry
the attributes the scenarios read (tick, control_freq, goal) and random obstacle maps shaped like
QuadrotorEnvMulti.obst_generation_given_density builds them (quadrotor_multi.py:405-426: an 8 x 8 map, 20 % pillars,
get_cell_centers), and records:
  * every draw in call order ("tape"): np.random.uniform / randint, np.random.choice (the chosen values),
    np.random.shuffle (the permutation it applied), and the scenario Generator's integers / uniform;
  * the spawn points and goals after reset(), then the goals after every step() whose goals changed (ticks 1..T),
    the scenario attributes (control_step_for_sec, end_point / formation).
The oracle (oracle/quadswarm_oracle_scen.c or_oscen_reset / or_oscen_step) replays the tape and must reproduce them.

Harness-side fixes (documented in DESIGN.md, like tools/gen_golden_obst.py's):
  * the o_* classes take no rng argument (o_base.py:7), so their QuadrotorScenario builds an unseeded
    np.random.default_rng(); the harness hands them a recorded, seeded Generator after construction (the
    "rng factory patch");
  * the reference reaches these classes only through create_scenario / QUADS_MODE_LIST_OBSTACLES_TEST (its env's
    Scenario_mix passes a mode_index their reset() does not take), so they are driven directly here;
  * np.random.shuffle(goals) is recorded as the permutation: the harness shuffles an index array with the same
    global state (shuffle's draws depend only on the length) and applies it;
  * bezier.Curve: the Bernstein restatement of tools/gen_golden_scen.py.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden_scen as GS  # noqa: E402  (shims, the bezier stand-in, the np.random uniform / randint tape)

OUT = GS.OUT
TAPE, ON = GS.TAPE, GS.ON
_rec = GS._rec

_np_choice, _np_shuffle = np.random.choice, np.random.shuffle


def _choice(*a, **k):
    return _rec(_np_choice(*a, **k))


def _shuffle(x):
    perm = np.arange(len(x))
    _np_shuffle(perm)
    x[:] = np.asarray(x)[perm]
    _rec(perm)


np.random.choice = _choice
np.random.shuffle = _shuffle

from gym_art.quadrotor_multi.obstacles.utils import get_cell_centers  # noqa: E402
import gym_art.quadrotor_multi.scenarios.mix as MIX  # noqa: E402
from gym_art.quadrotor_multi.scenarios.utils import QUADS_FORMATION_LIST  # noqa: E402

MODES = ["o_swap_goals", "o_ep_rand_bezier", "o_dynamic_same_goal"]


def random_map(rng, n=8, density=0.2):
    """obst_generation_given_density's map (quadrotor_multi.py:405-426) from a harness generator."""
    m = np.zeros((n, n))
    for o in rng.choice(n * n, int(n * n * density), replace=False):
        m[o // n, o % n] = 1
    return m


def run(mode, n, T, seed, resets):
    rng = GS.RecGen(np.random.default_rng(seed))
    np.random.seed(seed + 1)
    mrng = np.random.default_rng(seed + 2)
    cc = get_cell_centers(obst_area_length=8, obst_area_width=8, grid_size=1.0)
    envs = [GS.SubEnv() for _ in range(n)]
    del TAPE[:]
    out = dict(maps=[], tape_start=[], tape_len=[], spawns=[], goals=[], ticks=[], reset_id=[], period=[], end=[],
               formation=[], size=[], layer=[])
    for rr in range(resets):
        omap = random_map(mrng)
        ON[0] = True
        start = len(TAPE)
        sc = getattr(MIX, "Scenario_" + mode)(mode, envs, n, [10, 10, 10])
        sc.rng = rng                     # the rng factory patch (see the module docstring)
        sc.reset(obst_map=omap, cell_centers=cc)
        out["maps"].append(omap)
        out["spawns"].append(np.array(sc.spawn_points, dtype=np.float64))
        out["period"].append(int(sc.control_step_for_sec))
        # the scenario's centre: o_swap_goals' formation_center, the other two's end_point
        out["end"].append(np.asarray(sc.formation_center if mode == "o_swap_goals" else sc.end_point, dtype=np.float64))
        out["formation"].append(QUADS_FORMATION_LIST.index(sc.formation))
        out["size"].append(float(sc.formation_size))
        out["layer"].append(float(sc.layer_dist))
        for i, e in enumerate(envs):
            e.goal = np.array(sc.goals[i], dtype=np.float64)
            e.tick = 0
        out["goals"].append(np.array([e.goal for e in envs]))
        out["ticks"].append(0)
        out["reset_id"].append(rr)
        prev = out["goals"][-1]
        for t in range(1, T + 1):
            for e in envs:
                e.tick = t
            sc.step()
            cur = np.array([np.asarray(e.goal, dtype=np.float64) for e in envs])
            if not np.array_equal(cur, prev):
                out["goals"].append(cur)
                out["ticks"].append(t)
                out["reset_id"].append(rr)
            prev = cur
        ON[0] = False
        out["tape_start"].append(start)
        out["tape_len"].append(len(TAPE) - start)
    d = {k: np.array(v) for k, v in out.items()}
    d.update(tape=np.array(TAPE, dtype=np.float64), n=n, T=T, mode=MODES.index(mode), cell_centers=cc)
    return d


def main():
    os.makedirs(OUT, exist_ok=True)
    cases = [("o_swap_goals", 8, 1300, 31, 4), ("o_swap_goals", 5, 700, 32, 3), ("o_swap_goals", 2, 700, 33, 3),
             ("o_dynamic_same_goal", 8, 1300, 34, 4), ("o_dynamic_same_goal", 4, 700, 35, 3),
             ("o_ep_rand_bezier", 4, 1300, 36, 3), ("o_ep_rand_bezier", 8, 700, 37, 2)]
    for mode, n, T, seed, resets in cases:
        d = run(mode, n, T, seed, resets)
        name = f"oscen_{mode}_n{n}.npz"
        np.savez_compressed(os.path.join(OUT, name), **d)
        print(name, d["goals"].shape, len(d["tape"]), os.path.getsize(os.path.join(OUT, name)))


if __name__ == "__main__":
    main()
