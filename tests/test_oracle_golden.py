"""Pin the CPU oracle (oracle/quadswarm_oracle.c) against the reference's golden vectors.

The fixtures in tests/golden were produced by tools/gen_golden.py from the reference itself
(priban42/quad-swarm-rl-stable-baselines3 imported through tools/refshim.py), including a
"tape" of every np.random value the reference drew, so the oracle replays the same draws.
CPU-only; no GPU needed.
"""
import ctypes
import os

import numpy as np
import pytest

from conftest import GOLDEN

import oracle as O

RTOL_FN = 1e-11      # per-function (one call, fp64 vs fp64, libm ulp differences only)
ATOL_FN = 1e-12
RTOL_TRAJ = 1e-7     # whole trajectories: ulp differences amplified by the closed loop
ATOL_TRAJ = 1e-8


def close(a, b, rtol, atol):
    np.testing.assert_allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64), rtol=rtol, atol=atol)


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors (kat_vectors)."""
    L = O.lib()
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in cases:
        c = (ctypes.c_uint32 * 4)(*ctr)
        k = (ctypes.c_uint32 * 2)(*key)
        o = (ctypes.c_uint32 * 4)()
        L.or_philox4x32_10(c, k, o)
        assert tuple(o) == want


def test_params_match_reference(golden):
    g = golden("params")
    p = O.default_params()
    assert p.mass == float(g["mass"])
    assert list(p.inertia) == list(g["inertia"])
    assert list(p.thrust_max) == list(g["thrust_max"])
    assert list(p.torque_max) == list(g["torque_max"])
    assert p.arm == float(g["arm"])
    assert p.motor_tau_up == float(g["motor_tau_up"])
    for k in range(4):
        assert list(p.prop_cross[k]) == list(g["prop_cross"][k])


def test_dyn_substep(golden):
    g = golden("dyn_substep")
    p = O.params_from_golden(golden("params"))
    L = O.lib()
    n = len(g["pos"])
    n_svd = n_floor = n_flip = 0
    for c in range(n):
        d = O.OrDrone()
        O.set_drone(d, pos=g["pos"][c], vel=g["vel"][c], rot=g["rot"][c], omega=g["omega"][c],
                    thrust_rot_damp=g["rd"][c], thrust_cmds_damp=g["cd"][c])
        d.since_last_svd = float(g["since"][c])
        d.on_floor = int(g["on_floor"][c])
        s, ln = int(g["tape_start"][c]), int(g["tape_len"][c])
        tape = O.TapeRng(g["tape"][s:s + ln])
        cmds = np.ascontiguousarray(g["cmds"][c])
        noise = np.ascontiguousarray(g["noise"][c])
        L.or_dyn_substep(ctypes.byref(p), ctypes.byref(d), O.dptr(cmds), O.dptr(noise), tape.ref, 0, 0)
        assert tape.r.tape_pos == ln and not tape.r.overrun
        close(O.get_arr(d.pos), g["o_pos"][c], RTOL_FN, ATOL_FN)
        close(O.get_arr(d.vel), g["o_vel"][c], RTOL_FN, ATOL_FN)
        close(O.get_arr(d.rot, (3, 3)), g["o_rot"][c], RTOL_FN, ATOL_FN)
        close(O.get_arr(d.omega), g["o_omega"][c], RTOL_FN, ATOL_FN)
        close(O.get_arr(d.acc), g["o_acc"][c], RTOL_FN, ATOL_FN)
        close(O.get_arr(d.thrust_rot_damp), g["o_rd"][c], RTOL_FN, ATOL_FN)
        close(O.get_arr(d.thrust_cmds_damp), g["o_cd"][c], RTOL_FN, ATOL_FN)
        assert d.since_last_svd == pytest.approx(float(g["o_since"][c]), abs=1e-15)
        assert d.on_floor == int(g["o_on_floor"][c])
        assert d.crashed_floor == int(g["o_crashed_floor"][c])
        assert d.crashed_wall == int(g["o_crashed_wall"][c])
        assert d.crashed_ceiling == int(g["o_crashed_ceiling"][c])
        n_svd += float(g["o_since"][c]) == 0.0
        n_floor += int(g["o_on_floor"][c])
        n_flip += ln
    # the fixture must actually exercise the edge branches
    assert n_svd > 10 and n_floor > 50 and n_flip > 3


def test_polar_is_svd_polar_factor():
    rng = np.random.default_rng(0)
    for _ in range(50):
        a = np.linalg.qr(rng.normal(size=(3, 3)))[0]
        if np.linalg.det(a) < 0:
            a[:, 0] *= -1
        a = a + rng.normal(scale=1e-3, size=(3, 3))
        u, s, vh = np.linalg.svd(a)
        want = u @ vh
        x = np.ascontiguousarray(a.ravel())
        O.lib().or_polar(O.dptr(x))
        close(x.reshape(3, 3), want, 1e-12, 1e-13)


def test_ou(golden):
    g = golden("ou")
    p = O.default_params(ou_theta=float(g["theta"]), ou_sigma=float(g["sigma"]))
    tape = O.TapeRng(g["tape"])
    ou = np.zeros(4)
    for t in range(len(g["seq"])):
        O.lib().or_ou_noise(ctypes.byref(p), O.dptr(ou), tape.ref, 0)
        close(ou, g["seq"][t], RTOL_FN, ATOL_FN)


def test_sensor_noise(golden):
    g = golden("sensor")
    p = O.default_params()
    L = O.lib()
    for c in range(len(g["pos"])):
        tape = O.TapeRng(g["tape"][c])
        outs = [np.zeros(3), np.zeros(3), np.zeros(9), np.zeros(3)]
        ins = [np.ascontiguousarray(g[k][c].ravel()) for k in ("pos", "vel", "rot", "omega")]
        L.or_sensor_noise(ctypes.byref(p), *[O.dptr(a) for a in ins], tape.ref, 0, 3, *[O.dptr(a) for a in outs])
        assert tape.r.tape_pos == 27
        close(outs[0], g["n_pos"][c], RTOL_FN, ATOL_FN)
        close(outs[1], g["n_vel"][c], RTOL_FN, ATOL_FN)
        close(outs[2].reshape(3, 3), g["n_rot"][c], 1e-10, 1e-11)
        close(outs[3], g["n_omega"][c], RTOL_FN, ATOL_FN)


def test_collide_drones(golden):
    g = golden("collisions")
    L = O.lib()
    for c in range(len(g["dd_in"])):
        x = g["dd_in"][c]
        arrs = [np.ascontiguousarray(x[3 * i:3 * i + 3]) for i in range(6)]
        tape = O.TapeRng(g["dd_tape"][c][:int(g["dd_tape_len"][c])])
        L.or_collide_drones(*[O.dptr(a) for a in arrs], tape.ref, 0, 1)
        assert tape.r.tape_pos == int(g["dd_tape_len"][c])
        got = np.concatenate([arrs[1], arrs[2], arrs[4], arrs[5]])
        close(got, g["dd_out"][c], 1e-10, 1e-11)


def test_collide_wall_ceiling(golden):
    g = golden("collisions")
    p = O.default_params()
    L = O.lib()
    for c in range(len(g["wall_in"])):
        for kind in ("wall", "ceil"):
            x = g[f"{kind}_in"][c]
            d = O.OrDrone()
            O.set_drone(d, pos=x[0:3], vel=x[3:6], omega=x[6:9])
            tape = O.TapeRng(g[f"{kind}_tape"][c])
            if kind == "wall":
                L.or_collide_wall(ctypes.byref(p), ctypes.byref(d), tape.ref, 0)
            else:
                L.or_collide_ceiling(ctypes.byref(d), tape.ref, 0)
            assert not tape.r.overrun
            close(np.concatenate([O.get_arr(d.vel), O.get_arr(d.omega)]), g[f"{kind}_out"][c], 1e-10, 1e-11)


@pytest.mark.parametrize("n,k", [(8, 6), (8, 2), (8, 7), (32, 6), (64, 6), (64, 63), (128, 6), (128, 16)])
def test_neighbor_obs(golden, n, k):
    g = golden({64: "neighbors64", 128: "neighbors128"}.get(n, "neighbors"))
    p = O.default_params(num_agents=n, k_neighbors=k)
    od = 18 + 6 * k
    for c in range(len(g[f"n{n}k{k}_pos"])):
        ev = O.OrEnv()
        for i in range(n):
            for a in range(3):
                ev.obs_pos[i][a] = g[f"n{n}k{k}_pos"][c][i][a]
                ev.obs_vel[i][a] = g[f"n{n}k{k}_vel"][c][i][a]
        obs = np.zeros((n, od))
        O.lib().or_neighbor_obs(ctypes.byref(p), ctypes.byref(ev), O.dptr(obs), od)
        close(obs[:, 18:], g[f"n{n}k{k}_obs"][c], RTOL_FN, ATOL_FN)


def load_traj_env(golden, name):
    g = golden("traj_" + name)
    n, k = int(g["n"]), int(g["k"])
    k = n - 1 if k == -1 else k
    self_dim = g["obs"].shape[-1] - 6 * k          # 18 / 19 / 24: xyz_vxyz_R_omega[_floor|_wall]
    p = O.params_from_golden(golden("params"), num_agents=n, num_envs=1, k_neighbors=k,
                             ep_len=int(g["ep_len"]), use_downwash=int(g["downwash"]),
                             sense_noise=int(g["sense"]), ou_sigma=0.2 * float(g["thrust_noise"]),
                             obs_repr={18: 0, 19: 1, 24: 2}[self_dim])
    drones = O.drones_array(n)
    envs = O.envs_array(1)
    for i in range(n):
        d = drones[i]
        O.set_drone(d, pos=g["init_pos"][i], vel=g["init_vel"][i], rot=g["init_rot"][i], omega=g["init_omega"][i],
                    acc=g["init_acc"][i], thrust_rot_damp=g["init_rd"][i], thrust_cmds_damp=g["init_cd"][i],
                    ou=g["init_ou"][i], goal=g["init_goal"][i])
        d.since_last_svd = float(g["init_since"][i])
        d.on_floor = int(g["init_on_floor"][i])
        for a in range(3):
            envs[0].obs_vel[i][a] = g["init_env_vel"][i][a]
    envs[0].tick = int(g["init_tick"])
    return g, p, drones, envs


@pytest.mark.parametrize("name", ["n8k6", "n8k7", "n1", "n8dw", "n32k6", "n8quiet", "n8wall", "n4wallquiet", "n8stats",
                                  "n64k6", "n128k6"])
def test_trajectory_tape_replay(golden, name):
    g, p, drones, envs = load_traj_env(golden, name)
    n = p.num_agents
    od = O.lib().or_obs_dim(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["spawn"])
    n_done = 0
    for t in range(len(g["actions"])):
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs = np.zeros((n, od))
        term = np.zeros((n, od))
        rew = np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        O.lib().or_env_step(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                            done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), O.dptr(term))
        assert not tape.r.overrun, f"tape ran dry at step {t}"
        np.testing.assert_array_equal(done.astype(bool), g["done"][t].astype(bool))
        close(rew, g["rew"][t], RTOL_TRAJ, ATOL_TRAJ)
        close(obs, g["obs"][t], RTOL_TRAJ, ATOL_TRAJ)
        n_done += int(done[0])
    # every recorded draw consumed, in order
    assert tape.r.tape_pos == len(g["tape"])
    assert tape.r.spawn_pos == len(g["spawn"])
    close(np.stack([O.get_arr(drones[i].pos) for i in range(n)]), g["final_pos"], RTOL_TRAJ, ATOL_TRAJ)
    if name in ("n8k6", "n8k7", "n1", "n32k6", "n8wall", "n8stats", "n64k6", "n128k6"):
        assert n_done >= 1   # the auto-reset path was exercised
    if name == "n8wall":     # the wall features saw contacts: clipped at 0 and at 5
        w = g["obs"][:, :, 18:24]
        assert (w == 0).any() and (w == 5).any()


def test_episode_extra_stats_tape_replay(golden):
    """episode_extra_stats of every finished episode (quadrotor_multi.py:739-831): the oracle's accumulators,
    replayed on the reference's own draws, give the reference's dicts -- the same keys (built by the product's
    quadswarm_amd.stats from the oracle's row) and the same values."""
    import json
    from quadswarm_amd.stats import ES_D1, ES_D3, ES_D5, NES, episode_extra_stats

    ref = json.load(open(os.path.join(GOLDEN, "traj_n8stats_stats.json")))["events"]
    g, p, drones, envs = load_traj_env(golden, "n8stats")
    n = p.num_agents
    od = O.lib().or_obs_dim(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["spawn"])
    got = []
    for t in range(len(g["actions"])):
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        O.lib().or_env_step(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                            done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), O.dptr(term))
        if done.any():
            rows = []
            for i in range(n):
                row = np.array(envs[0].ep_stats[:], dtype=np.float64)
                assert len(row) == NES
                row[ES_D1], row[ES_D3], row[ES_D5] = drones[i].ep_dist[0], drones[i].ep_dist[1], drones[i].ep_dist[2]
                rows.append(episode_extra_stats(row))
            got.append({"step": t, "agents": rows})
    assert [e["step"] for e in got] == [e["step"] for e in ref] and len(ref) == 2
    for eg, er in zip(got, ref):
        for i in range(n):
            a, b = eg["agents"][i], er["agents"][i]
            assert sorted(a) == sorted(b)
            for key in b:
                assert a[key] == pytest.approx(b[key], rel=1e-9, abs=1e-12), (eg["step"], i, key)


def oracle_coeff(p):
    return {"pos": p.rew_pos, "effort": p.rew_effort, "crash": p.rew_crash, "orient": p.rew_orient,
            "spin": p.rew_spin, "quadcol_bin": p.rew_quadcol_bin, "quadcol_bin_obst": p.rew_quadcol_bin_obst}


def test_step_infos_tape_replay(golden):
    """Per-step infos[i]["rewards"] (quadrotor_single.py:79-105, 371; quadrotor_multi.py:642-651): the oracle's
    reward components, replayed on the reference's draws through a crowded run with collisions, proximity,
    floor / wall contacts and an auto-reset, turned into dicts by the product's quadswarm_amd.infos, are the
    reference's own dicts -- the same keys and values."""
    import json
    from quadswarm_amd.infos import REWARD_KEYS_B, reward_columns_b

    keys = json.load(open(os.path.join(GOLDEN, "traj_n8info_infokeys.json")))["rewards_keys"]
    assert sorted(keys) == sorted(REWARD_KEYS_B)
    g, p, drones, envs = load_traj_env(golden, "n8info")
    n = p.num_agents
    od = O.lib().or_obs_dim(ctypes.byref(p))
    tape = O.TapeRng(g["tape"], g["spawn"])
    ref = g["info_rewards"]
    nonzero = {k: 0 for k in keys}
    for t in range(len(g["actions"])):
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64)
        obs, term, rew = np.zeros((n, od)), np.zeros((n, od)), np.zeros(n)
        done = np.zeros(n, dtype=np.uint8)
        O.lib().or_env_step(ctypes.byref(p), drones, envs, 0, O.dptr(a), tape.ref, O.dptr(obs), O.dptr(rew),
                            done.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), O.dptr(term))
        comp = np.array([list(drones[i].rinfo) for i in range(n)]).T
        cols = reward_columns_b(comp, oracle_coeff(p), p.dt)
        for c, k in enumerate(keys):
            np.testing.assert_allclose(cols[k], ref[t, :, c], rtol=1e-9, atol=1e-12, err_msg=f"step {t} {k}")
            nonzero[k] += int((ref[t, :, c] != 0).sum())
    assert tape.r.tape_pos == len(g["tape"])
    # the run exercises every term (collisions, proximity, floor contact)
    assert all(v > 0 for v in nonzero.values()), nonzero
