#!/usr/bin/env python
"""Golden fixtures for the obstacle rows of flavor B.  TEST INFRASTRUCTURE,
dev container only.

    python tools/gen_golden_obst.py        # writes tests/golden/obst_*.npz

Reference code exercised: obstacles/utils.py (get_surround_sdfs, collision_detection, get_cell_centers),
collisions/obstacles.py (perform_collision_with_obstacle), scenarios/obstacles/o_base.py
(max_square_area_center, generate_pos_obst_map*), o_random.py, o_static_same_goal.py, scenarios/mix.py,
and QuadrotorEnvMulti with use_obstacles=True (quadrotor_multi.py:405-426, 440-517, 570-720).

Harness-side fix (documented in DESIGN.md): Scenario_mix builds its sub-scenario with
create_scenario(..., rng) (scenarios/mix.py:33-35), but the obstacle scenarios' constructors take no
rng argument (o_base.py:7), so the reference's obstacle path raises TypeError as committed.  The
generator wraps create_scenario to drop the rng for o_* classes, which is what SURVEY §8c verified.

Tapes: np.random.normal/uniform/randn (gen_golden) plus np.random.choice (recorded as the chosen
values, in call order) go to "tape"; the env Generator's uniform(size=3) spawn draws and its
integers() mode index go to "spawn".
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the shims and the np.random tape)

_choice = np.random.choice


def _rec_choice(*a, **k):
    v = _choice(*a, **k)
    if G.TAPE.on:
        G.TAPE.vals.extend(np.ravel(np.asarray(v, dtype=np.float64)).tolist())
    return v


np.random.choice = _rec_choice

import gym_art.quadrotor_multi.scenarios.mix as MIX  # noqa: E402
from gym_art.quadrotor_multi.obstacles.utils import get_surround_sdfs, collision_detection, get_cell_centers  # noqa: E402
from gym_art.quadrotor_multi.collisions.obstacles import perform_collision_with_obstacle  # noqa: E402
from gym_art.quadrotor_multi.scenarios.obstacles.o_base import Scenario_o_base  # noqa: E402


def _create_scenario(quads_mode, envs, num_agents, room_dims, rng):
    cls = getattr(MIX, "Scenario_" + quads_mode)
    if quads_mode.startswith("o_"):
        return cls(quads_mode, envs, num_agents, room_dims)
    return cls(quads_mode, envs, num_agents, room_dims, rng)


MIX.create_scenario = _create_scenario
OUT = G.OUT


class GenProxyObst(G.GenProxy):
    def integers(self, *a, **k):
        v = self._g.integers(*a, **k)
        if G.TAPE.on:
            G.TAPE.spawn.extend(np.ravel(np.asarray(v, dtype=np.float64)).tolist())
        return v


def random_map(rng, L=8, W=8, density=0.2):
    m = np.zeros((L, W))
    idx = rng.choice(L * W, int(L * W * density), replace=False)
    for o in idx:
        m[o // W, o % W] = 1
    return m, idx


def gen_sdf(n=300, seed=41):
    rng = np.random.default_rng(seed)
    cc = get_cell_centers(obst_area_length=8, obst_area_width=8, grid_size=1.0)
    Q, Ob, S, C = [], [], [], []
    for c in range(n):
        _, idx = random_map(rng)
        obst = cc[idx]
        q = rng.uniform(-4.5, 4.5, (8, 2))
        if c % 3 == 0:   # put drones right next to / inside obstacles
            q[:3] = obst[:3] + rng.normal(scale=0.2, size=(3, 2))
        sdf = get_surround_sdfs(q, obst, 100 * np.ones((8, 9)), obst_radius=0.3, resolution=0.1)
        col = collision_detection(q, obst, obst_radius=0.3, quad_radius=0.04596194077712559)
        Q.append(q); Ob.append(obst); S.append(sdf.copy()); C.append(col)
    np.savez_compressed(os.path.join(OUT, "obst_sdf.npz"), quad=np.array(Q), obst=np.array(Ob), sdf=np.array(S),
                        col=np.array(C), cell_centers=cc)


def gen_maps(n=200, seed=42):
    rng = np.random.default_rng(seed)
    cc = get_cell_centers(obst_area_length=8, obst_area_width=8, grid_size=1.0)
    sc = Scenario_o_base("o_random", [], 8, [10, 10, 10])
    M, OUTP, T = [], [], []
    for c in range(n):
        m, _ = random_map(rng, density=[0.2, 0.05, 0.4, 0.0][c % 4])
        sc.obstacle_map = m
        sc.cell_centers = cc
        G.begin()
        p = sc.max_square_area_center()
        tv, _ = G.end()
        M.append(m); OUTP.append(p); T.append(tv)
    np.savez_compressed(os.path.join(OUT, "obst_maps.npz"), maps=np.array(M), center=np.array(OUTP),
                        tape=np.array(T).reshape(n, -1))


def gen_impulse(n=200, seed=43):
    rng = np.random.default_rng(seed)
    d = G.make_dyn()
    ins, outs, tapes = [], [], []
    for c in range(n):
        o = np.array([rng.integers(-4, 4) + 0.5, rng.integers(-4, 4) + 0.5, 5.0])
        ang = rng.uniform(-np.pi, np.pi)
        r = rng.uniform(0.2, 0.35)
        pos = o + np.array([r * np.cos(ang), r * np.sin(ang), 0.0])
        pos[2] = rng.uniform(0.5, 3.0) if c % 5 else rng.uniform(4.9, 5.1)   # 3-D "inside" branch
        vel = rng.uniform(-2, 2, 3)
        om = rng.uniform(-3, 3, 3)
        d.pos, d.vel, d.omega = pos.copy(), vel.copy(), om.copy()
        G.begin()
        perform_collision_with_obstacle(drone_dyn=d, obstacle_pos=o, obstacle_size=0.6)
        tv, _ = G.end()
        ins.append(np.concatenate([pos, vel, om, o]))
        outs.append(np.concatenate([d.vel, d.omega]))
        tapes.append(tv)
    L = max(len(t) for t in tapes)
    np.savez_compressed(os.path.join(OUT, "obst_impulse.npz"), inp=np.array(ins), out=np.array(outs),
                        tape=np.stack([np.pad(t, (0, L - len(t))) for t in tapes]),
                        tape_len=np.array([len(t) for t in tapes]))


def make_env_obst(n=8, k=2, seed=0, ep_time=15.0, obs_type="pos_vel", downwash=True, sense="default",
                  thrust_noise=0.05):
    from gym_art.quadrotor_multi.quadrotor_multi import QuadrotorEnvMulti

    class Cfg:
        pass
    cfg = Cfg()
    cfg.seed = seed
    env = QuadrotorEnvMulti(
        num_agents=n, ep_time=ep_time, rew_coeff=dict(G.REW, quadcol_bin_obst=5.0), obs_repr="xyz_vxyz_R_omega_floor",
        cfg=cfg, neighbor_visible_num=k, neighbor_obs_type=obs_type, collision_hitbox_radius=2.0,
        collision_falloff_radius=4.0, use_obstacles=True, obst_density=0.2, obst_size=0.6,
        obst_spawn_area=[8, 8], use_downwash=downwash, use_numba=True, quads_mode="mix",
        room_dims=[10, 10, 10], use_replay_buffer=False, quads_view_mode=[], quads_render=False,
        dynamics_params="Crazyflie", raw_control=True, raw_control_zero_middle=True,
        dynamics_randomize_every=None,
        dynamics_change=dict(noise=dict(thrust_noise_ratio=thrust_noise), damp=dict(vel=0, omega_quadratic=0)),
        dyn_sampler_1=None, sense_noise=sense, init_random_state=False)
    px = GenProxyObst(env.rng)
    env.rng = px
    env.scenario.rng = px
    for e in env.envs:
        e.rng = px
    return env


def snapshot(env):
    s = G.snapshot(env)
    s["obst"] = np.array(env.obstacles.pos_arr, dtype=np.float64)
    s["prev_obst"] = np.zeros(len(env.envs))
    prev = getattr(env, "prev_obst_quad_collisions", [])
    for q in np.asarray(prev, dtype=int):
        s["prev_obst"][q] = 1.0
    s["mode"] = np.array(float(type(env.scenario.scenario).__name__ == "Scenario_o_static_same_goal"))
    s["wall_prev"] = np.array([float(i in set(np.asarray(env.prev_crashed_walls, dtype=int).tolist()))
                               for i in range(len(env.envs))])
    s["ceil_prev"] = np.array([float(i in set(np.asarray(env.prev_crashed_ceiling, dtype=int).tolist()))
                               for i in range(len(env.envs))])
    return s


def setup_obst(env, rng):
    """Aim drones at obstacles (obstacle collisions + impulses) and pair two drones (drone collision)."""
    ds = [e.dynamics for e in env.envs]
    ob = np.array(env.obstacles.pos_arr)
    for i in range(min(3, len(ds))):
        ang = rng.uniform(-np.pi, np.pi)
        ds[i].pos = np.array([ob[i, 0] + 0.45 * np.cos(ang), ob[i, 1] + 0.45 * np.sin(ang), 2.0])
        ds[i].vel = np.array([-2.0 * np.cos(ang), -2.0 * np.sin(ang), 0.0])
        env.pos[i] = ds[i].pos
    if len(ds) >= 6:
        ds[5].pos = ds[4].pos + np.array([0.05, 0.03, 0.0])


def gen_traj(name, n, k, steps, seed, ep_time, setup=None, hover=False, reset_kw=None, infos=False, **kw):
    np.random.seed(seed)
    env = make_env_obst(n, k, seed=seed, ep_time=ep_time, **kw)
    G.begin()
    obs0, _ = env.reset(**(reset_kw or {}))
    tv0, sp0 = G.end()
    if setup is not None:
        setup(env, np.random.default_rng(seed + 100))
    init = snapshot(env)
    act_rng = np.random.default_rng(seed + 200)
    actions = np.clip(act_rng.uniform(-1.0, 1.0, (steps, n, 4)) * 0.6 + 0.3, -1, 1)
    if hover:   # ~hover thrust with small perturbations: no contacts, no random impulses
        actions = 0.0526 + 0.1 * act_rng.uniform(-1.0, 1.0, (steps, n, 4))
    obs, rew, done = [], [], []
    rinfo, rkeys = [], None
    G.begin()
    for t in range(steps):
        o, r, dn, info = env.step(actions[t])
        if infos:   # infos[i]["rewards"] incl. the obstacle terms (quadrotor_multi.py:642-651)
            rkeys = rkeys or sorted(info[0]["rewards"])
            rinfo.append([[float(info[i]["rewards"][key]) for key in rkeys] for i in range(n)])
        obs.append(np.array(o, dtype=np.float64))
        rew.append(np.array(r, dtype=np.float64))
        done.append(np.array(dn, dtype=np.float64))
    tv, sp = G.end()
    extra = {}
    if infos:
        import json
        with open(os.path.join(OUT, f"obst_traj_{name}_infokeys.json"), "w") as f:
            json.dump({"name": name, "rewards_keys": rkeys}, f, indent=0, sort_keys=True)
        extra["info_rewards"] = np.array(rinfo, dtype=np.float64)
    final = snapshot(env)
    np.savez_compressed(os.path.join(OUT, f"obst_traj_{name}.npz"), actions=actions, obs=np.stack(obs), **extra,
                        rew=np.stack(rew), done=np.stack(done), tape=tv, spawn=sp, tape0=tv0, spawn0=sp0,
                        obs0=np.array(obs0, dtype=np.float64), n=n, k=k, ep_len=env.envs[0].ep_len,
                        downwash=int(kw.get("downwash", True)), sense=int(kw.get("sense", "default") == "default"),
                        thrust_noise=kw.get("thrust_noise", 0.05),
                        dr_density=float((reset_kw or {}).get("obst_density") or 0.0),
                        dr_size=float((reset_kw or {}).get("obst_size") or 0.0),
                        **{"init_" + a: b for a, b in init.items()}, **{"final_" + a: b for a, b in final.items()})


DR_RANGES = [(0.05, 0.2, 0.3, 0.6),    # runs/obstacles/obst_domain_random.py (= the quadrotor_params defaults)
             (0.0, 0.2, 0.0, 0.6),     # a zero choice: falsy at quadrotor_multi.py:443-446, keeps the env's value
             (0.1, 0.35, 0.2, 0.9)]


def gen_dr():
    """Obstacle domain randomisation (quad_experience_replay.py:76-87, 106-118): the choice lists the reference's
    wrapper builds (np.arange) for DR_RANGES, then env.reset(obst_density, obst_size) with a chosen pair followed by
    a trajectory whose in-env resets keep the pair (quadrotor_multi.py:440-450, 836)."""
    import gym_art.quadrotor_multi.quad_experience_replay as XR
    env = make_env_obst(8, 2, seed=60)
    tabs = {}
    for i, (dlo, dhi, slo, shi) in enumerate(DR_RANGES):
        w = XR.ExperienceReplayWrapper(env, 0.75, 0.2, 0.6, True, True, True, dlo, dhi, slo, shi)
        tabs[f"range_{i}"] = np.array([dlo, dhi, slo, shi])
        tabs[f"densities_{i}"] = np.asarray(w.obst_densities, dtype=np.float64)
        tabs[f"sizes_{i}"] = np.asarray(w.obst_sizes, dtype=np.float64)
        # int(num_room_grids * density) of obst_generation_given_density (quadrotor_multi.py:414)
        counts = []
        for d in w.obst_densities:
            env.obst_density = d
            counts.append(len(env.obst_generation_given_density()[1]))
        tabs[f"counts_{i}"] = np.array(counts, dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "obst_dr_tables.npz"), n_ranges=len(DR_RANGES), **tabs)
    d0, s0 = tabs["densities_0"], tabs["sizes_0"]
    gen_traj("dr3", 8, 2, 90, seed=61, ep_time=0.3, setup=setup_obst,
             reset_kw=dict(obst_density=d0[0], obst_size=s0[1]))
    gen_traj("dr9", 8, 2, 90, seed=62, ep_time=0.3, setup=setup_obst,
             reset_kw=dict(obst_density=d0[2], obst_size=s0[2]))


def main():
    os.makedirs(OUT, exist_ok=True)
    if len(sys.argv) > 1 and sys.argv[1] == "dr":
        gen_dr()
        return
    if len(sys.argv) > 1 and sys.argv[1] == "info":   # per-step infos["rewards"] with the obstacle terms
        gen_traj("c4info", 8, 2, 40, seed=54, ep_time=0.3, setup=setup_obst, infos=True)
        return
    gen_sdf()
    gen_maps()
    gen_impulse()
    # C4: 8 drones, pos_vel k=2, floor repr, downwash, mix of o_random / o_static_same_goal; short
    # episodes so the run crosses several in-env resets (new maps and scenario modes)
    gen_traj("c4", 8, 2, 90, seed=51, ep_time=0.3, setup=setup_obst)
    gen_traj("n4none", 4, 0, 60, seed=52, ep_time=0.25, obs_type="none", downwash=False, setup=setup_obst)
    # noise-free, contact-free: the GPU replays it directly (SDF obs over a 150-step flight)
    gen_traj("quiet", 8, 2, 150, seed=53, ep_time=15.0, hover=True, sense=None, thrust_noise=0.0, downwash=False)
    for f in sorted(os.listdir(OUT)):
        if f.startswith("obst_"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
