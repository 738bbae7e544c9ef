"""The oracle's obstacle-map dynamic scenarios (oracle/quadswarm_oracle_scen.c or_oscen_reset / or_oscen_step)
replayed against the reference.

tests/golden/oscen_*.npz were recorded from the reference's own Scenario_o_swap_goals, Scenario_o_ep_rand_bezier and
Scenario_o_dynamic_same_goal (scenarios/obstacles/*.py) by tools/gen_golden_oscen.py on random 8 x 8 obstacle maps:
every np.random / Generator draw in call order (np.random.choice as the chosen values, np.random.shuffle as its
permutation), the spawn points and goals after reset(), the goals after every step() that moved them.  Replaying the
tape, the oracle must reproduce every spawn point, goal and scenario attribute and consume exactly the reference's
draws -- this pins the restatement the GPU kernels are compared with draw for draw (tests/test_gpu_parity_obst.py).
"""
import ctypes
import glob
import os

import numpy as np
import pytest

import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(glob.glob(os.path.join(GOLD, "oscen_*.npz")))


def _params(n):
    p = O.default_params(num_agents=n, num_envs=1)
    p.control_dt = 0.01        # control_freq 100 (the stand-in sub-envs')
    p.use_obstacles = 1
    p.obst_area = 8
    for k in range(3):         # room_dims [10, 10, 10] as the harness passes it
        p.room_lo[k], p.room_hi[k] = (-5.0, -5.0, 0.0)[k], (5.0, 5.0, 10.0)[k]
    return p


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[6:-4] for f in FILES])
def test_obstacle_scenario_replays_reference(path):
    g = np.load(path)
    n, T = int(g["n"]), int(g["T"])
    omode = 2 + int(g["mode"])
    p = _params(n)
    L = O.lib()
    cc = g["cell_centers"]
    goals_rec, ticks, rid = g["goals"], g["ticks"], g["reset_id"]
    k = 0
    for r in range(len(g["maps"])):
        omap = np.ascontiguousarray(g["maps"][r].astype(np.uint8).ravel())
        tape = g["tape"][g["tape_start"][r]:g["tape_start"][r] + g["tape_len"][r]]
        draws = O.ScenDraws(tape=tape)
        sc = O.OrScen()
        cells = np.zeros(n, dtype=np.int32)
        sz = np.zeros(n)
        goals = np.zeros((n, 3))
        L.or_oscen_reset(ctypes.byref(p), omode, ctypes.byref(sc), draws.ref,
                         omap.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), 8,
                         cells.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), O.dptr(sz), O.dptr(goals))
        # spawn points: free cell c (row-major) -> cell_centers[row + 8 col], z ~ U(1, 3)
        spawn = np.array([[*cc[c // 8 + 8 * (c % 8)], z] for c, z in zip(cells, sz)])
        np.testing.assert_allclose(spawn, g["spawns"][r], rtol=0, atol=1e-12, err_msg=f"reset {r}: spawn points")
        assert sc.period == g["period"][r]
        np.testing.assert_allclose(np.ctypeslib.as_array(sc.center), g["end"][r], rtol=0, atol=1e-12)
        assert sc.formation == g["formation"][r]
        np.testing.assert_allclose([sc.size, sc.layer], [g["size"][r], g["layer"][r]], rtol=0, atol=1e-12)
        assert rid[k] == r and ticks[k] == 0
        np.testing.assert_allclose(goals, goals_rec[k], rtol=0, atol=1e-10, err_msg=f"reset {r}")
        k += 1
        for t in range(1, T + 1):
            prev = goals.copy()
            L.or_oscen_step(ctypes.byref(p), ctypes.byref(sc), t, draws.ref,
                            omap.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), 8, O.dptr(goals))
            if k < len(ticks) and rid[k] == r and ticks[k] == t:
                np.testing.assert_allclose(goals, goals_rec[k], rtol=0, atol=1e-10, err_msg=f"reset {r} tick {t}")
                k += 1
            else:
                np.testing.assert_array_equal(goals, prev, err_msg=f"reset {r} tick {t}: goals moved, reference kept them")
        assert draws.s.tape_pos == len(tape) and not draws.s.overrun, f"reset {r}: draw count differs from the reference"
    assert k == len(ticks)


def test_fixtures_cover_the_events():
    """Every mode's fixture crosses its events: swaps / resamples after reset, several curves for the bezier mode."""
    seen = {}
    for f in FILES:
        g = np.load(f)
        seen.setdefault(int(g["mode"]), 0)
        seen[int(g["mode"])] += int((g["ticks"] > 0).sum())
    assert sorted(seen) == [0, 1, 2] and min(seen.values()) >= 5
