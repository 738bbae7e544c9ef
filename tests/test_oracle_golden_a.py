"""Pin the flavor-A CPU oracle (oracle/quadswarm_oracle_a.c) against the reference's golden vectors.

Fixtures: tests/golden/a_*.npz from tools/gen_golden_a.py (the reference's quadrotor_multi_rewards
env, Controller/ cascade, get_state and camera model, run through tools/refshim.py), with tapes of
every value the reference drew from np.random and from its np.random.Generator.  CPU-only.
"""
import ctypes

import numpy as np
import pytest

import oracle as O

RTOL_FN, ATOL_FN = 1e-11, 1e-12
RTOL_TRAJ, ATOL_TRAJ = 1e-7, 1e-8
NTYPES = ["dist_angle", "dist_sangle", "ndist_nsangle", "dist_angle_heading", "dist_sangle_sheading",
          "pos", "npos", "pos_vel"]


def close(a, b, rtol, atol, msg=""):
    np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64), rtol=rtol,
                               atol=atol, err_msg=msg)


def golden_params_a(golden, **kw):
    g = golden("params")
    p = O.params_a(**kw)
    p.mass = float(g["mass"])
    for i in range(3):
        p.inertia[i] = float(g["inertia"][i])
    for k in range(4):
        p.thrust_max[k] = float(g["thrust_max"][k])
        p.torque_max[k] = float(g["torque_max"][k])
    p.arm = float(g["arm"])
    p.motor_tau_up = float(g["motor_tau_up"])
    p.motor_tau_down = float(g["motor_tau_down"])
    return p


def test_controller_constants(golden):
    g = golden("a_pid")
    p = O.params_a()
    np.testing.assert_array_equal(np.array(p.mixer).reshape(4, 4), g["mixer"])
    close([p.pid_kp[7] / 3.1222, p.pid_kp[8] / 3.1222, p.pid_kp[9] / 3.1222], g["J"], 1e-15, 0)


def test_pid_cascade(golden):
    """Controller.update_vel_height_dir (Controller.py:76-101) incl. every PID, the acceleration
    controller's oblique projection, attitude error, rate PIDs x J x 800 and the mixer desaturation."""
    g = golden("a_pid")
    p = O.params_a()
    L = O.lib()
    n = len(g["pos"])
    sat = 0
    for c in range(n):
        d = O.OrDrone()
        O.set_drone(d, pos=g["pos"][c], vel=g["vel"][c], rot=g["rot"][c], omega=g["omega"][c], pid=g["pid_in"][c])
        d.angle = float(g["angle"][c])
        m = np.zeros(4)
        L.or_ctrl_a(ctypes.byref(p), ctypes.byref(d), float(g["cmd"][c][0]), float(g["height"][c]), O.dptr(m))
        close(m, g["motors"][c], 1e-9, 1e-11, f"case {c} motors")
        close(O.get_arr(d.pid), g["pid_out"][c], 1e-9, 1e-11, f"case {c} pid")
        close(d.angle, g["angle_out"][c], 1e-13, 1e-13)
        sat += int(np.max(g["motors"][c]) > 1.0 - 1e-12 or np.min(g["motors"][c]) < 1e-12)
    assert sat > 10   # the desaturation branches were exercised


def test_camera(golden):
    g = golden("a_camera")
    p = O.params_a()
    L = O.lib()
    n = g["rel"].shape[1]
    for sig in (0, 3):
        tape = g[f"s{sig}_tape"]
        for c in range(n):
            l, a = ctypes.c_double(), ctypes.c_double()
            L.or_camera(ctypes.byref(p), float(g["rel"][0, c]), float(g["rel"][1, c]), float(g["ga"][c]),
                        float(tape[c]), float(tape[n + c]), ctypes.byref(l), ctypes.byref(a))
            close([l.value, a.value], [g[f"s{sig}_l"][c], g[f"s{sig}_a"][c]], 1e-9, 1e-10, f"sigma {sig} case {c}")
    assert np.sum(g["s0_l"] == 0.0) >= 10   # NaN -> 0 path (target inside the marker radius)


@pytest.mark.parametrize("ri", range(4))
def test_self_obs(golden, ri):
    g = golden("a_obs")
    r = O.A_REPRS[ri]
    p = O.params_a(obs_repr=r)
    p.cam_size, p.cam_focal, p.cam_px_noise, p.n_cameras = float(g["cam"][0]), float(g["cam"][1]), \
        float(g["cam"][2]), int(g["cam"][3])
    dim = 7 if "sangle" in r else 6
    for c in range(len(g[r + "_pos"])):
        d = O.OrDrone()
        O.set_drone(d, pos=g[r + "_pos"][c], vel=g[r + "_vel"][c], rot=g[r + "_rot"][c], omega=g[r + "_omega"][c],
                    goal=g[r + "_goal"][c])
        d.angle, d.ang_vel = float(g[r + "_angle"][c]), float(g[r + "_angvel"][c])
        tape = O.TapeRng(g[r + "_tape"][c])
        out = np.zeros(dim)
        O.lib().or_self_obs_a(ctypes.byref(p), ctypes.byref(d), tape.ref, 0, O.S_SENSOR, 15, O.dptr(out))
        assert not tape.r.overrun
        close(out, g[r + "_obs"][c], 1e-9, 1e-10, f"{r} case {c}")


@pytest.mark.parametrize("ntype", NTYPES)
@pytest.mark.parametrize("n,k", [(8, 7), (8, 3), (4, 3)])
def test_neighbor_obs_a(golden, ntype, n, k):
    g = golden("a_neighbors")
    key = f"{ntype}_n{n}k{k}"
    p = O.params_a(num_agents=n, k=k, ntype=ntype, cam_px_noise=3.0 if ntype == "ndist_nsangle" else 0.0)
    so = 7
    od = so + k * p.nfeat_dim
    for c in range(len(g[key + "_pos"])):
        ev = O.OrEnv()
        drones = O.drones_array(n)
        for i in range(n):
            for a in range(3):
                ev.obs_pos[i][a] = g[key + "_pos"][c][i][a]
                ev.obs_vel[i][a] = g[key + "_vel"][c][i][a]
            ev.heading[i] = g[key + "_heading"][c][i]
            drones[i].angle = g[key + "_angle"][c][i]
        tl = int(g[key + "_tapelen"][c])
        tape = O.TapeRng(g[key + "_tape"][c][:tl] if tl else np.zeros(0))
        obs = np.zeros((n, od))
        O.lib().or_neighbor_obs_a(ctypes.byref(p), ctypes.byref(ev), drones, tape.ref, 0, 0, O.dptr(obs), od)
        assert not tape.r.overrun
        assert tape.r.tape_pos == tl
        close(obs[:, so:], g[key + "_obs"][c], 1e-9, 1e-10, f"{key} case {c}")


def load_traj_a(golden, name, which="init"):
    g = golden("a_traj_" + name)
    n, k = int(g["n"]), int(g["k"])
    room = tuple(float(x) for x in g["room"])
    p = golden_params_a(golden, num_agents=n, num_envs=1, k=k, obs_repr=O.A_REPRS[int(g["obs_repr"])],
                        ntype=NTYPES[int(g["ntype"])], room=room)
    p.ep_len = int(g["ep_len"])
    p.sense_noise = int(g["sense"])
    p.ou_sigma = 0.2 * float(g["thrust_noise"])
    p.cam_px_noise = float(g["px_noise"])
    p.use_downwash = int(name.endswith("dw"))     # use_downwash (quadrotor_multi_rewards.py:810-815)
    drones = O.drones_array(n)
    envs = O.envs_array(1)
    w = which + "_"
    for i in range(n):
        d = drones[i]
        O.set_drone(d, pos=g[w + "pos"][i], vel=g[w + "vel"][i], rot=g[w + "rot"][i], omega=g[w + "omega"][i],
                    thrust_rot_damp=g[w + "rd"][i], thrust_cmds_damp=g[w + "cd"][i], ou=g[w + "ou"][i],
                    goal=g[w + "goal"][i], pid=g[w + "pid"][i])
        d.since_last_svd = float(g[w + "since"][i])
        d.on_floor = int(g[w + "on_floor"][i])
        d.angle, d.ang_vel = float(g[w + "angle"][i]), float(g[w + "angvel"][i])
        for a in range(3):
            envs[0].obs_vel[i][a] = g[w + "env_vel"][i][a]
            envs[0].obs_pos[i][a] = g[w + "env_pos"][i][a]
        envs[0].heading[i] = g[w + "heading"][i]
    envs[0].tick = int(g[w + "tick"])
    envs[0].target[0], envs[0].target[1] = g[w + "target"]
    envs[0].success = int(g[w + "success"])
    envs[0].capture_radius = float(g[w + "capture"])
    envs[0].has_pos = 1
    return g, p, drones, envs


TRAJ = ["n4", "n8", "n8k3cam", "n1", "n4quiet", "n8dw", "n8stats", "n128k7"]


@pytest.mark.parametrize("name", [t for t in TRAJ if t not in ("n8dw", "n8stats")])   # edited after the reset
def test_first_reset_tape_replay(golden, name):
    """QuadrotorEnvMulti.reset from construction (no dynamics.pos yet: no chaser force, :38)."""
    g, p, _, _ = load_traj_a(golden, name)
    n = p.num_agents
    od = O.lib().or_obs_dim_a(ctypes.byref(p))
    drones, envs = O.drones_array(n), O.envs_array(1)
    envs[0].target[0] = envs[0].target[1] = 0.0
    tape = O.TapeRng(g["tape0"], g["gtape0"])
    obs = np.zeros((n, od))
    ri = np.zeros(1, dtype=np.uint8)
    O.lib().or_env_reset_a(ctypes.byref(p), drones, envs, 0, tape.ref, O.dptr(obs),
                           ri.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)))
    assert not tape.r.overrun
    assert tape.r.tape_pos == len(g["tape0"]) and tape.r.spawn_pos == len(g["gtape0"])
    close(obs, g["obs0"], RTOL_FN, ATOL_FN)
    close(np.stack([O.get_arr(drones[i].pos) for i in range(n)]), g["init_pos"], RTOL_FN, ATOL_FN)
    close(np.stack([O.get_arr(drones[i].rot) for i in range(n)]).reshape(n, 3, 3), g["init_rot"], RTOL_FN, ATOL_FN)
    close(list(envs[0].target), g["init_target"], RTOL_FN, ATOL_FN)
    close([drones[i].angle for i in range(n)], g["init_angle"], RTOL_FN, ATOL_FN)


@pytest.mark.parametrize("name", TRAJ)
def test_trajectory_tape_replay_a(golden, name):
    g, p, drones, envs = load_traj_a(golden, name)
    n = p.num_agents
    od = O.lib().or_obs_dim_a(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["gtape"])
    resets = 0
    U8 = ctypes.POINTER(ctypes.c_ubyte)
    for t in range(len(g["actions"])):
        envs[0].capture_radius = float(g["capture"][t])
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        ri = np.zeros(1, dtype=np.uint8)
        O.lib().or_env_step_a(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                              done.ctypes.data_as(U8), O.dptr(term), ri.ctypes.data_as(U8))
        assert not tape.r.overrun, f"tape ran dry at step {t}"
        np.testing.assert_array_equal(done.astype(bool), g["done"][t].astype(bool), err_msg=f"step {t}")
        close(rew, g["rew"][t], RTOL_TRAJ, ATOL_TRAJ, f"rew step {t}")
        if done[0]:
            close(term, g["term"][t], RTOL_TRAJ, ATOL_TRAJ, f"term step {t}")
            assert ri[0] - 1 == int(g["reset_info"][t])
            resets += 1
        else:
            assert ri[0] == 0
        close(obs, g["obs"][t], RTOL_TRAJ, ATOL_TRAJ, f"obs step {t}")
    assert tape.r.tape_pos == len(g["tape"])
    assert tape.r.spawn_pos == len(g["gtape"])
    close(np.stack([O.get_arr(drones[i].pos) for i in range(n)]), g["final_pos"], RTOL_TRAJ, ATOL_TRAJ)
    close(np.stack([O.get_arr(drones[i].pid) for i in range(n)]), g["final_pid"], 1e-6, 1e-8)
    if name in ("n4", "n8", "n1"):
        assert resets >= 1


@pytest.mark.parametrize("mode", ["mix", "static_diff_goal", "ep_lissajous3D", "dynamic_formations", "swap_goals",
                                  "swarm_vs_swarm", "run_away"])
def test_goal_scenarios_run_in_flavor_a(mode):
    """create_scenario goal scenarios in the flavor-A env (quadrotor_multi_rewards.py:123, :560, :848): the
    scenario functions are the ones pinned by the scenario tapes (test_oracle_scen.py); here their wiring --
    goals from scenario.reset(), drones spawned at their goal, goals moved by scenario.step() every tick."""
    from quadswarm_amd import QuadSwarmConfig
    from parity_utils import oracle_params_a
    cfg = QuadSwarmConfig.sb_train(num_envs=6, num_agents=8, neighbor_obs_type="dist_angle", quads_mode=mode,
                                   episode_duration=1.0, seed=2)
    oenv = O.OracleEnvA(oracle_params_a(cfg), seed=2)
    oenv.set_capture_radius(0.0)
    obs, _ = oenv.reset()
    goals = np.array([oenv.drones[g].goal[:] for g in range(48)])
    pos = np.array([oenv.drones[g].pos[:] for g in range(48)])
    np.testing.assert_allclose(pos[:, :2], goals[:, :2])          # spawn at the goal (spawn_points None)
    if mode in ("static_diff_goal", "swap_goals", "swarm_vs_swarm", "dynamic_formations"):   # a goal per drone
        assert len({tuple(np.round(g, 6)) for g in goals[:8]}) > 1
    rng = np.random.default_rng(0)
    moved = False
    for t in range(12):
        obs, rew, done, _, _ = oenv.step(rng.uniform(-1, 1, (48, 2)))
        assert np.isfinite(obs).all() and np.isfinite(rew).all()
        g2 = np.array([oenv.drones[g].goal[:] for g in range(48)])
        moved |= bool(np.abs(g2 - goals).max() > 1e-9)
    if mode in ("ep_lissajous3D", "dynamic_formations"):
        assert moved


def test_episode_extra_stats_a_tape_replay(golden):
    """Flavor A's infos[i]["episode_extra_stats"] (quadrotor_multi_rewards.py:886-969): the oracle's per-tick
    collision / room bookkeeping, replayed on the reference's draws, gives the reference's dicts -- keys built
    by the product's quadswarm_amd.stats, distance_to_goal_* = nan (the env never appends distances)."""
    import json
    import os
    from conftest import GOLDEN
    from quadswarm_amd.stats import ES_D1, ES_D3, ES_D5, episode_extra_stats

    ref = json.load(open(os.path.join(GOLDEN, "a_traj_n8stats_stats.json")))["events"]
    g, p, drones, envs = load_traj_a(golden, "n8stats")
    n = p.num_agents
    od = O.lib().or_obs_dim_a(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["gtape"])
    U8 = ctypes.POINTER(ctypes.c_ubyte)
    got = []
    for t in range(len(g["actions"])):
        envs[0].capture_radius = float(g["capture"][t])
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        ri = np.zeros(1, dtype=np.uint8)
        O.lib().or_env_step_a(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                              done.ctypes.data_as(U8), O.dptr(term), ri.ctypes.data_as(U8))
        if done.any():
            rows = []
            for i in range(n):
                row = np.array(envs[0].ep_stats[:], dtype=np.float64)
                row[ES_D1], row[ES_D3], row[ES_D5] = drones[i].ep_dist[0], drones[i].ep_dist[1], drones[i].ep_dist[2]
                rows.append(episode_extra_stats(row))
            got.append({"step": t, "agents": rows})
    assert [e["step"] for e in got] == [e["step"] for e in ref] and len(ref) >= 1
    for eg, er in zip(got, ref):
        for i in range(n):
            a, b = eg["agents"][i], er["agents"][i]
            assert sorted(a) == sorted(b)
            for key in b:
                if np.isnan(b[key]):
                    assert np.isnan(a[key]), key
                else:
                    assert a[key] == pytest.approx(b[key], rel=1e-9, abs=1e-12), (eg["step"], i, key)
    # the run exercised collisions after settle, the final-5 s window and the room lists
    r0 = ref[0]["agents"][0]
    assert r0["num_collisions_after_settle"] > 0 and r0["num_collisions_with_room"] > 0


def test_step_infos_goal_dist_a(golden):
    """Flavor A's per-step infos[i] = {"rewards": {}, "goal_dist": |pos - goal|} of the last executed tick
    (quadrotor_single_rewards.py:457), through captures and timeouts: the oracle's OR_RI_GOAL_DIST vs the
    reference's values."""
    g, p, drones, envs = load_traj_a(golden, "n4info")
    n = p.num_agents
    od = O.lib().or_obs_dim_a(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["gtape"])
    U8 = ctypes.POINTER(ctypes.c_ubyte)
    dones = 0
    for t in range(len(g["actions"])):
        envs[0].capture_radius = float(g["capture"][t])
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        ri = np.zeros(1, dtype=np.uint8)
        O.lib().or_env_step_a(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                              done.ctypes.data_as(U8), O.dptr(term), ri.ctypes.data_as(U8))
        gd = np.array([drones[i].rinfo[O.RI_GOAL_DIST] for i in range(n)])
        close(gd, g["info_goal_dist"][t], 1e-9, 1e-12, f"goal_dist step {t}")
        dones += int(done[0])
    assert tape.r.tape_pos == len(g["tape"])
    assert dones >= 2   # goal_dist of a finished step is the pre-reset one
