"""Pin the obstacle rows of the CPU oracle against the reference.

Fixtures: tests/golden/obst_*.npz from tools/gen_golden_obst.py (obstacles/utils.py,
collisions/obstacles.py, scenarios/obstacles/*, QuadrotorEnvMulti with use_obstacles=True) with the
np.random tape (incl. np.random.choice) and the Generator tape (spawn jitter, mix mode index).
CPU-only.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN

RTOL_TRAJ, ATOL_TRAJ = 1e-7, 1e-8


def close(a, b, rtol, atol, msg=""):
    np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64), rtol=rtol,
                               atol=atol, err_msg=msg)


def obst_params(golden, **over):
    p = O.params_from_golden(golden("params"), use_obstacles=1, num_obstacles=12, obst_area=8, obst_size=0.6,
                             obst_z=5.0, sdf_resolution=0.1, rew_quadcol_bin_obst=5.0, spawn_box=0.1)
    for k, v in over.items():
        setattr(p, k, v)
    return p


def env_with_obstacles(obst):
    ev = O.OrEnv()
    ev.n_obst = len(obst)
    for o in range(len(obst)):
        ev.obst[o][0], ev.obst[o][1] = obst[o][0], obst[o][1]
    return ev


def test_cell_centers(golden):
    g = golden("obst_sdf")
    cc = g["cell_centers"]
    out = np.zeros(2)
    for idx in range(64):
        # get_cell_centers order: index = row + 8 * col for the env's (row, col) cells
        row, col = idx % 8, idx // 8
        O.lib().or_cell_xy(row, col, 8, O.dptr(out))
        np.testing.assert_array_equal(out, cc[idx])


def test_reference_unit_test_values():
    """obstacles/test/unit_test.py:6-22 (quad at 0, obstacle at (0.2, 0), radius 0.3) and
    collisions/test/unit_test/obstacles.py:6-18 (collision normal (-1,-1,0)/sqrt 2)."""
    p = O.default_params(use_obstacles=1, obst_size=0.6, sdf_resolution=0.1)
    ev = env_with_obstacles([[0.2, 0.0]])
    out = np.zeros(9)
    O.lib().or_obst_sdf(ctypes.byref(p), ctypes.byref(ev), O.dptr(np.zeros(2)), O.dptr(out))
    want = [np.hypot(x - 0.2, y) - 0.3 for x in (-0.1, 0, 0.1) for y in (-0.1, 0, 0.1)]
    close(out, want, 1e-15, 1e-15)
    assert O.lib().or_obst_detect(ctypes.byref(p), ctypes.byref(ev), O.dptr(np.zeros(2))) == 0


def test_sdf_and_detection(golden):
    g = golden("obst_sdf")
    p = O.params_from_golden(golden("params"), use_obstacles=1, obst_size=0.6, sdf_resolution=0.1)
    hits = 0
    for c in range(len(g["quad"])):
        ev = env_with_obstacles(g["obst"][c])
        for i in range(8):
            out = np.zeros(9)
            q = np.ascontiguousarray(g["quad"][c][i])
            O.lib().or_obst_sdf(ctypes.byref(p), ctypes.byref(ev), O.dptr(q), O.dptr(out))
            close(out, g["sdf"][c][i], 1e-13, 1e-13)
            got = O.lib().or_obst_detect(ctypes.byref(p), ctypes.byref(ev), O.dptr(q))
            assert got == int(g["col"][c][i])
            hits += got >= 0
    assert hits > 20


def test_max_square_area_center(golden):
    g = golden("obst_maps")
    out = np.zeros(2)
    for c in range(len(g["maps"])):
        m = np.ascontiguousarray(g["maps"][c].astype(np.uint8).ravel())
        O.lib().or_max_square_center(m.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), 8, O.dptr(out))
        np.testing.assert_array_equal(out, g["center"][c][:2])
        assert g["center"][c][2] == g["tape"][c][0]


def test_obstacle_impulse(golden):
    g = golden("obst_impulse")
    p = O.params_from_golden(golden("params"), obst_size=0.6)
    inside = 0
    for c in range(len(g["inp"])):
        x = g["inp"][c]
        d = O.OrDrone()
        O.set_drone(d, pos=x[0:3], vel=x[3:6], omega=x[6:9])
        tape = O.TapeRng(g["tape"][c][:int(g["tape_len"][c])])
        O.lib().or_collide_obstacle(ctypes.byref(p), ctypes.byref(d), O.dptr(np.ascontiguousarray(x[9:12])), tape.ref, 0)
        assert not tape.r.overrun and tape.r.tape_pos == int(g["tape_len"][c])
        close(np.concatenate([O.get_arr(d.vel), O.get_arr(d.omega)]), g["out"][c], 1e-10, 1e-11)
        inside += np.linalg.norm(x[0:3] - x[9:12]) < 0.3
    assert inside > 5


def apply_dr(p, envs, g):
    """A fixture reset with env.reset(obst_density, obst_size) (the domain-randomisation wrapper's choice):
    the pair becomes table entry 1 and the env's current indices point at it.  Tape mode replays the bare
    env, so the oracle does not draw the choice; the env's in-env resets keep it."""
    if "dr_density" not in g or float(g["dr_density"]) == 0.0:
        return
    p.dr_n_counts, p.dr_n_sizes = 1, 1
    p.dr_counts[1] = int(p.obst_area * p.obst_area * float(g["dr_density"]))   # quadrotor_multi.py:414
    p.dr_sizes[1] = float(g["dr_size"])
    envs[0].obst_mi, envs[0].obst_si = 1, 1


def load_traj_obst(golden, name, which="init"):
    g = golden("obst_traj_" + name)
    n, k = int(g["n"]), int(g["k"])
    p = obst_params(golden, num_agents=n, num_envs=1, k_neighbors=k, obs_repr=1, ep_len=int(g["ep_len"]),
                    use_downwash=int(g["downwash"]), rew_quadcol_smooth_max=10.0)
    drones, envs = O.drones_array(n), O.envs_array(1)
    w = which + "_"
    for i in range(n):
        d = drones[i]
        O.set_drone(d, pos=g[w + "pos"][i], vel=g[w + "vel"][i], rot=g[w + "rot"][i], omega=g[w + "omega"][i],
                    acc=g[w + "acc"][i], thrust_rot_damp=g[w + "rd"][i], thrust_cmds_damp=g[w + "cd"][i],
                    ou=g[w + "ou"][i], goal=g[w + "goal"][i])
        d.since_last_svd = float(g[w + "since"][i])
        d.on_floor = int(g[w + "on_floor"][i])
        d.prev_obst = int(g[w + "prev_obst"][i])
        d.prev_wall = int(g[w + "wall_prev"][i])
        d.prev_ceiling = int(g[w + "ceil_prev"][i])
        for a in range(3):
            envs[0].obs_vel[i][a] = g[w + "env_vel"][i][a]
    ob = g[w + "obst"]
    envs[0].n_obst = len(ob)
    for o in range(len(ob)):
        envs[0].obst[o][0], envs[0].obst[o][1] = ob[o][0], ob[o][1]
    envs[0].obst_mode = int(g[w + "mode"])
    envs[0].tick = int(g[w + "tick"])
    apply_dr(p, envs, g)
    return g, p, drones, envs


@pytest.mark.parametrize("name", ["c4", "n4none", "dr3", "dr9"])
def test_first_reset_with_obstacles(golden, name):
    g, p, _, _ = load_traj_obst(golden, name)
    n = p.num_agents
    od = O.lib().or_obs_dim(ctypes.byref(p))
    drones, envs = O.drones_array(n), O.envs_array(1)
    apply_dr(p, envs, g)
    tape = O.TapeRng(g["tape0"], g["spawn0"])
    obs = np.zeros((n, od))
    O.lib().or_env_reset(ctypes.byref(p), drones, envs, 0, tape.ref, O.dptr(obs))
    assert not tape.r.overrun
    assert tape.r.tape_pos == len(g["tape0"]) and tape.r.spawn_pos == len(g["spawn0"])
    close(obs, g["obs0"], 1e-11, 1e-12)
    ob = np.array([[envs[0].obst[o][0], envs[0].obst[o][1]] for o in range(envs[0].n_obst)])
    close(ob, g["init_obst"][:, :2], 0, 0)
    assert envs[0].obst_mode == int(g["init_mode"])


@pytest.mark.parametrize("name", ["c4", "n4none", "dr3", "dr9"])
def test_trajectory_with_obstacles(golden, name):
    g, p, drones, envs = load_traj_obst(golden, name)
    n = p.num_agents
    od = O.lib().or_obs_dim(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["spawn"])
    n_obst_hits = 0
    for t in range(len(g["actions"])):
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        O.lib().or_env_step(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                            done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), O.dptr(term))
        assert not tape.r.overrun, f"tape ran dry at step {t}"
        np.testing.assert_array_equal(done.astype(bool), g["done"][t].astype(bool))
        close(rew, g["rew"][t], RTOL_TRAJ, ATOL_TRAJ, f"rew step {t}")
        close(obs, g["obs"][t], RTOL_TRAJ, ATOL_TRAJ, f"obs step {t}")
        n_obst_hits += int((g["rew"][t] < -4.0).sum())
    assert tape.r.tape_pos == len(g["tape"])
    assert tape.r.spawn_pos == len(g["spawn"])
    assert n_obst_hits >= 1


def test_domain_random_tables(golden):
    """The wrapper's choice lists (np.arange, quad_experience_replay.py:82, 86) and the pillar counts the env
    makes of them (int(area^2 * density), quadrotor_multi.py:414), as the host config computes them; a 0.0
    choice is falsy at quadrotor_multi.py:443-446 and keeps the env's value (-1 / 0 in the tables)."""
    from quadswarm_amd import QuadSwarmConfig
    t = golden("obst_dr_tables")
    for i in range(int(t["n_ranges"])):
        dlo, dhi, slo, shi = t["range_%d" % i]
        cfg = QuadSwarmConfig.c4(num_envs=4, replay_buffer_sample_prob=0.75, domain_random=True,
                                 obst_density_random=True, obst_size_random=True, obst_density_min=dlo,
                                 obst_density_max=dhi, obst_size_min=slo, obst_size_max=shi)
        dens, counts, sizes = cfg.domain_random_tables()
        np.testing.assert_array_equal(dens, t["densities_%d" % i])
        np.testing.assert_array_equal(sizes, t["sizes_%d" % i])
        want = [c if d != 0.0 else -1 for c, d in zip(t["counts_%d" % i], t["densities_%d" % i])]
        assert counts == want


def test_step_infos_with_obstacles(golden):
    """infos[i]["rewards"] with the obstacle terms rew_quadcol_obstacle / rewraw_quadcol_obstacle
    (quadrotor_multi.py:642-651): oracle components through quadswarm_amd.infos vs the reference's dicts."""
    import json
    from quadswarm_amd.infos import REWARD_KEYS_B, REWARD_KEYS_OBST, reward_columns_b

    keys = json.load(open(os.path.join(GOLDEN, "obst_traj_c4info_infokeys.json")))["rewards_keys"]
    assert sorted(keys) == sorted(REWARD_KEYS_B + REWARD_KEYS_OBST)
    g, p, drones, envs = load_traj_obst(golden, "c4info")
    n = p.num_agents
    od = O.lib().or_obs_dim(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["spawn"])
    coeff = {"pos": p.rew_pos, "effort": p.rew_effort, "crash": p.rew_crash, "orient": p.rew_orient,
             "spin": p.rew_spin, "quadcol_bin": p.rew_quadcol_bin, "quadcol_bin_obst": p.rew_quadcol_bin_obst}
    hits = 0
    for t in range(len(g["actions"])):
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        O.lib().or_env_step(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                            done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), O.dptr(term))
        comp = np.array([list(drones[i].rinfo) for i in range(n)]).T
        cols = reward_columns_b(comp, coeff, p.dt, use_obstacles=True)
        for c, k in enumerate(keys):
            close(cols[k], g["info_rewards"][t, :, c], 1e-9, 1e-12, f"step {t} {k}")
        hits += int((g["info_rewards"][t, :, keys.index("rewraw_quadcol_obstacle")] != 0).sum())
    assert tape.r.tape_pos == len(g["tape"])
    assert hits >= 1
