#!/usr/bin/env python
"""Golden fixtures for flavor A (quadrotor_multi_rewards / quadrotor_single_rewards + Controller/),
the env swarm_rl.sb_train actually trains on.  TEST INFRASTRUCTURE, dev container only.

    python tools/gen_golden_a.py          # writes tests/golden/a_*.npz

Uses the same import harness and np.random tape recorder as tools/gen_golden.py.  The env's
np.random.Generator (QuadrotorEnvMulti.rng: scenario resets, headings) is wrapped so its outputs
are recorded as a second tape ("gtape", call order).

Harness-side deviation (documented in DESIGN.md): Scenario_dynamic_repulsive initialises its target
position as an int array (scenarios/dynamic_repulsive.py:34), which makes its first reset produce a
NaN->int target; the generator sets it to float zeros before the first reset ("float-fixed", the fix
SURVEY.md §8(f) names).  Every later reset of the reference is unaffected by this.

Fixtures (plain arrays, np.load(allow_pickle=False)):
  a_pid.npz        Controller.update_vel_height_dir on random states / PID states (one call each)
  a_camera.npz     simulate_camera_measurement_vect with recorded pixel noise
  a_obs.npz        state_* of every flavor-A obs repr with recorded sensor noise
  a_neighbors.npz  QuadrotorEnvMulti.add_neighborhood_obs for every flavor-A neighbour type
  a_traj_*.npz     whole-env trajectories (step + the SB3 worker's reset on done) with both tapes
                   (a_traj_n128k7: `python tools/gen_golden_a.py n128`, see main_extra)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the shims and the np.random tape)

from swarm_rl.global_cfg import QuadrotorEnvConfig  # noqa: E402
from gym_art.quadrotor_multi.quadrotor_multi_rewards import QuadrotorEnvMulti  # noqa: E402
from gym_art.quadrotor_multi.Controller.Controller import Controller  # noqa: E402
from gym_art.quadrotor_multi.Controller.MultirotorModel import State  # noqa: E402
from gym_art.quadrotor_multi import get_state  # noqa: E402

OUT = G.OUT
GTAPE = []
REPRS = ["aw_awdot_dist_distdot_angle_angledot", "cdist_cdistdot_dist_distdot_angle_angledot",
         "cdist_cdistdot_dist_distdot_sangle_angledot", "cdist_cdistdot_ndist_distdot_nsangle_angledot"]
# QUADS_NEIGHBOR_OBS_TYPE keys the flavor-A env can build an observation space for
# (quadrotor_single_rewards.py:321-344; plain "dist"/"angle" have no branch there and fail to clip)
NTYPES = ["dist_angle", "dist_sangle", "ndist_nsangle", "dist_angle_heading", "dist_sangle_sheading",
          "pos", "npos", "pos_vel"]


class GenTape:
    """Records every value the env's Generator returns (random/uniform/integers), in call order."""

    def __init__(self, g):
        self._g = g

    def _rec(self, v):
        if G.TAPE.on:
            GTAPE.extend(np.ravel(np.asarray(v, dtype=np.float64)).tolist())
        return v

    def random(self, *a, **k):
        return self._rec(self._g.random(*a, **k))

    def uniform(self, *a, **k):
        return self._rec(self._g.uniform(*a, **k))

    def integers(self, *a, **k):
        return self._rec(self._g.integers(*a, **k))

    def __getattr__(self, n):
        return getattr(self._g, n)


def begin():
    GTAPE.clear()
    G.begin()


def end():
    tv, _ = G.end()
    return tv, np.array(GTAPE, dtype=np.float64)


def make_env_A(n, k=-1, repr_="cdist_cdistdot_dist_distdot_sangle_angledot", ntype="ndist_nsangle",
               px_noise=0.0, ep_time=30.0, sense="default", thrust_noise=None, seed=0, capture=3.0, downwash=False):
    cfg = QuadrotorEnvConfig()
    cfg.use_downwash = downwash
    cfg.num_agents = n
    cfg.neighbor_visible_num = k
    cfg.obs_repr = repr_
    cfg.neighbor_obs_type = ntype
    cfg.pixel_noise_cam = px_noise
    cfg.episode_duration = ep_time
    cfg.sense_noise = sense
    cfg.seed = seed
    cfg.initial_capture_radius = capture
    if thrust_noise is not None:
        cfg.dynamics_change = dict(noise=dict(thrust_noise_ratio=thrust_noise))
    env = QuadrotorEnvMulti(cfg)
    px = GenTape(env.rng)
    env.rng = px
    env.scenario.rng = px
    for e in env.envs:
        e.rng = px
    if hasattr(env.scenario, "pos"):
        env.scenario.pos = np.zeros(2)     # float-fixed dynamic_repulsive (module docstring)
    return env


PID_NAMES = [("position_controller", "pid_z")] + [("velocity_controller", a) for a in ("pid_x", "pid_y", "pid_z")] + \
    [("attitude_controller", a) for a in ("pid_x", "pid_y", "pid_z")] + \
    [("rate_controller", a) for a in ("pid_x", "pid_y", "pid_z")]


def get_pids(c):
    out = []
    for ctl, pid in PID_NAMES:
        p = getattr(getattr(c, ctl), pid)
        out += [p.last_error, p.integral]
    return np.array(out)


def set_pids(c, v):
    for n, (ctl, pid) in enumerate(PID_NAMES):
        p = getattr(getattr(c, ctl), pid)
        p.last_error, p.integral = float(v[2 * n]), float(v[2 * n + 1])


def gen_pid(n=400, seed=21):
    rng = np.random.default_rng(seed)
    rows = {k: [] for k in ["pos", "vel", "rot", "omega", "cmd", "height", "angle", "pid_in", "pid_out",
                            "angle_out", "motors"]}
    for c in range(n):
        ctl = Controller()
        pos = rng.uniform(-3, 3, 3); pos[2] = rng.uniform(0.2, 3.0)
        vel = rng.uniform(-1.5, 1.5, 3) * (0.1 if c % 4 == 0 else 1.0)
        rot = G.rand_rot(rng) if c % 3 == 0 else _small_tilt(rng)
        om = rng.uniform(-4, 4, 3) * (0.05 if c % 4 == 0 else 1.0)
        pid = rng.normal(size=20) * (np.array([0.5, 2] + [0.3, 1] * 3 + [0.1, 0.5] * 3 + [0.5, 0.5] * 3))
        if c % 5 == 0:
            pid[:] = 0.0
        set_pids(ctl, pid)
        ctl.angle = rng.uniform(-np.pi, np.pi)
        cmd = np.array([rng.uniform(-1.5, 1.5), rng.uniform(-1, 1)])
        height = 2.0 if c % 2 else rng.uniform(0.5, 3.0)
        st = State(pos.copy(), vel.copy(), np.zeros(3), rot.copy(), om.copy(), np.zeros(4))
        rows["angle"].append(ctl.angle)
        m = ctl.update_vel_height_dir(st, cmd, height, 0.005)
        for k_, v in dict(pos=pos, vel=vel, rot=rot.reshape(-1), omega=om, cmd=cmd, height=height, pid_in=pid,
                          pid_out=get_pids(ctl), angle_out=ctl.angle, motors=np.asarray(m, dtype=np.float64)).items():
            rows[k_].append(v)
    np.savez_compressed(os.path.join(OUT, "a_pid.npz"), **{k: np.array(v) for k, v in rows.items()},
                        mixer=ctl.mixer.allocation_matrix_inv, J=np.diag(ctl.params.J))


def _small_tilt(rng):
    ax = rng.normal(size=3); ax /= np.linalg.norm(ax)
    ang = rng.uniform(0, 0.6)
    K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
    yaw = rng.uniform(-np.pi, np.pi)
    c, s = np.cos(yaw), np.sin(yaw)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]]) @ R


def gen_camera(n=400, seed=22):
    rng = np.random.default_rng(seed)
    rel = rng.uniform(-6, 6, (2, n))
    rel[:, :20] *= 0.01                     # inside the target radius: NaN -> 0 path
    rel[:, 20:40] = np.array([[1.0], [0.0]]) * rng.uniform(0.2, 3, 20)   # on a camera axis
    ga = rng.uniform(-np.pi, np.pi, n)
    ga[40:60] = np.round(ga[40:60] / (2 * np.pi / 3)) * (2 * np.pi / 3)
    out = {}
    for sig in (0.0, 3.0):
        begin()
        l, a = get_state.simulate_camera_measurement_vect(rel, 0.2, 0.035, sig, ga, cameras_num=np.ones(n) * 3)
        tv, _ = end()
        out[f"s{int(sig)}_l"], out[f"s{int(sig)}_a"], out[f"s{int(sig)}_tape"] = l, a, tv
    np.savez_compressed(os.path.join(OUT, "a_camera.npz"), rel=rel, ga=ga, **out)


def gen_obs(n=200, seed=23):
    rng = np.random.default_rng(seed)
    env = make_env_A(1)
    e = env.envs[0]
    out = {}
    for r in REPRS:
        fn = getattr(get_state, "state_" + r)
        P, V, R, W, Gl, A, AV, O, T = [], [], [], [], [], [], [], [], []
        for c in range(n):
            d = e.dynamics
            d.pos = rng.uniform(-5, 5, 3); d.vel = rng.uniform(-2, 2, 3)
            d.rot = G.rand_rot(rng); d.omega = rng.uniform(-3, 3, 3)
            d.accelerometer = np.array([0.0, 0.0, 9.81])
            if c % 7 == 0:
                d.pos[:2] = 0.0
            e.goal = np.array([rng.uniform(-4, 4), rng.uniform(-4, 4), 2.0])
            if c % 11 == 0:
                e.goal[:2] = d.pos[:2] + rng.normal(scale=0.03, size=2)
            e.pre_controller.angle = rng.uniform(-np.pi, np.pi)
            e.pre_controller.angular_velocity = rng.uniform(-1.5, 1.5) if c % 5 else 0.0
            begin()
            o = fn(e)
            tv, _ = end()
            P.append(d.pos.copy()); V.append(d.vel.copy()); R.append(d.rot.reshape(-1).copy())
            W.append(np.array(d.omega, dtype=np.float64)); Gl.append(e.goal.copy())
            A.append(e.pre_controller.angle); AV.append(e.pre_controller.angular_velocity)
            O.append(np.array(o, dtype=np.float64)); T.append(tv)
        L = max(len(t) for t in T)
        out.update({f"{r}_pos": np.array(P), f"{r}_vel": np.array(V), f"{r}_rot": np.array(R),
                    f"{r}_omega": np.array(W), f"{r}_goal": np.array(Gl), f"{r}_angle": np.array(A),
                    f"{r}_angvel": np.array(AV), f"{r}_obs": np.array(O),
                    f"{r}_tape": np.stack([np.pad(t, (0, L - len(t))) for t in T])})
    out["cam"] = np.array([e.cfg.neighbour_size_cam, e.cfg.focal_length_cam, e.cfg.pixel_noise_cam, e.cfg.n_cameras])
    np.savez_compressed(os.path.join(OUT, "a_obs.npz"), **out)


def gen_neighbors(seed=24):
    rng = np.random.default_rng(seed)
    out = {}
    for ntype in NTYPES:
        for n, k in [(8, -1), (8, 3), (4, -1)]:
            env = make_env_A(n, k=k, ntype=ntype, px_noise=3.0 if ntype == "ndist_nsangle" else 0.0)
            K = n - 1 if k == -1 else k
            P, V, H, A, O, T = [], [], [], [], [], []
            for c in range(30):
                env.pos = rng.uniform(-6, 6, (n, 3)); env.pos[:, 2] = rng.uniform(0.5, 2.5, n)
                env.vel = rng.uniform(-2, 2, (n, 3))
                env.heading = rng.uniform(-np.pi, np.pi, n)
                ang = env.heading.copy() if c % 2 else rng.uniform(-np.pi, np.pi, n)
                for i, e in enumerate(env.envs):
                    e.pre_controller.angle = ang[i]
                if c % 6 == 0:
                    env.pos[1] = env.pos[0] + np.array([0.03, 0.02, 0.0])   # inside the camera target radius
                begin()
                o = env.add_neighborhood_obs([np.zeros(7) for _ in range(n)])
                tv, _ = end()
                P.append(env.pos.copy()); V.append(env.vel.copy()); H.append(env.heading.copy()); A.append(ang)
                O.append(np.array(o)[:, 7:]); T.append(tv)
            L = max(len(t) for t in T)
            key = f"{ntype}_n{n}k{K}"
            out.update({key + "_pos": np.array(P), key + "_vel": np.array(V), key + "_heading": np.array(H),
                        key + "_angle": np.array(A), key + "_obs": np.array(O),
                        key + "_tape": np.stack([np.pad(t, (0, L - len(t))) for t in T]),
                        key + "_tapelen": np.array([len(t) for t in T])})
    np.savez_compressed(os.path.join(OUT, "a_neighbors.npz"), **out)


def snapshot(env):
    ds = [e.dynamics for e in env.envs]
    cs = [e.pre_controller for e in env.envs]
    return dict(
        pos=np.stack([d.pos for d in ds]), vel=np.stack([d.vel for d in ds]), rot=np.stack([d.rot for d in ds]),
        omega=np.stack([np.asarray(d.omega, dtype=np.float64) for d in ds]),
        rd=np.stack([d.thrust_rot_damp for d in ds]), cd=np.stack([d.thrust_cmds_damp for d in ds]),
        ou=np.stack([np.array(d.thrust_noise.state) for d in ds]),
        since=np.array([d.since_last_svd for d in ds]), on_floor=np.array([d.on_floor for d in ds], dtype=np.float64),
        goal=np.stack([e.goal for e in env.envs]), tick=np.array(env.envs[0].tick),
        pid=np.stack([get_pids(c) for c in cs]), angle=np.array([c.angle for c in cs]),
        angvel=np.array([c.angular_velocity for c in cs], dtype=np.float64),
        target=np.array(env.scenario.pos, dtype=np.float64), heading=env.heading.copy(), env_vel=env.vel.copy(),
        env_pos=env.pos.copy(), success=np.array(float(env.episode_success)),
        capture=np.array(float(env.capture_radius)))


def gen_traj(name, n, steps, seed, capture_schedule=None, act_scale=1.0, setup=None, stats=False, infos=False, **kw):
    np.random.seed(seed)
    env = make_env_A(n, seed=seed, **kw)
    begin()
    obs0, info0 = env.reset()
    tv0, gt0 = end()
    if setup is not None:   # state edits after the reset (the replayed steps start from the snapshot below)
        setup(env)
    init = snapshot(env)
    act_rng = np.random.default_rng(seed + 200)
    actions = act_rng.uniform(-1.0, 1.0, (steps, n, 2)) * act_scale
    caps = np.array([capture_schedule(t) for t in range(steps)]) if capture_schedule else \
        np.full(steps, env.capture_radius)
    obs, rew, done, term, rinfo = [], [], [], [], []
    events, gdist = [], []
    begin()
    for t in range(steps):
        env.set_capture_radius(float(caps[t]))
        o, r, dn, info = env.step(actions[t])
        if infos:   # infos[i] = {"rewards": {}, "goal_dist": ...} of the last tick (quadrotor_single_rewards.py:457)
            assert all(info[i]["rewards"] == {} for i in range(n))
            gdist.append([float(info[i]["goal_dist"]) for i in range(n)])
        if stats and any(dn):   # infos[i]["episode_extra_stats"] (quadrotor_multi_rewards.py:886-969)
            events.append({"step": t, "agents": [{k_: float(v) for k_, v in info[i]["episode_extra_stats"].items()}
                                                 for i in range(n)]})
        o = np.array(o, dtype=np.float64)
        term.append(o.copy())
        ri = -1.0
        if any(dn):
            o, info = env.reset()       # SubprocVecEnvCustom worker (subproc_vec_env_custom.py:42-46)
            o = np.array(o, dtype=np.float64)
            ri = float(info["success"])
        obs.append(o); rew.append(np.array(r, dtype=np.float64)); done.append(np.array(dn, dtype=np.float64))
        rinfo.append(ri)
    tv, gt = end()
    if stats:
        import json
        with open(os.path.join(OUT, f"a_traj_{name}_stats.json"), "w") as f:
            json.dump({"name": name, "events": events}, f, indent=0, sort_keys=True)
    final = snapshot(env)
    c = env.cfg
    extra = {"info_goal_dist": np.array(gdist, dtype=np.float64)} if infos else {}
    np.savez_compressed(
        os.path.join(OUT, f"a_traj_{name}.npz"), actions=actions, capture=caps, obs0=np.array(obs0, dtype=np.float64),
        obs=np.stack(obs), term=np.stack(term), rew=np.stack(rew), done=np.stack(done), reset_info=np.array(rinfo),
        tape0=tv0, gtape0=gt0, tape=tv, gtape=gt, n=n, k=env.num_use_neighbor_obs, ep_len=env.envs[0].ep_len,
        obs_repr=REPRS.index(c.obs_repr), ntype=NTYPES.index(c.neighbor_obs_type), px_noise=c.pixel_noise_cam,
        sense=int(c.sense_noise == "default"), thrust_noise=env.envs[0].dynamics.thrust_noise_ratio,
        room=np.array(c.room_dims, dtype=np.float64), **extra,
        **{"init_" + a: b for a, b in init.items()}, **{"final_" + a: b for a, b in final.items()})


def main():
    os.makedirs(OUT, exist_ok=True)
    gen_pid()
    gen_camera()
    gen_obs()
    gen_neighbors()
    # sb_train's sweep config (sb_train.py:123-133): N=4, sangle repr, ndist_nsangle with pixel noise 0
    gen_traj("n4", 4, 120, seed=31, capture_schedule=lambda t: 3.0 if t >= 100 else 0.3, ep_time=0.8)
    # N=8 swarm (BASELINE metric), all neighbours, headings; curriculum radius that captures sometimes
    gen_traj("n8", 8, 80, seed=32, ntype="dist_sangle_sheading", capture_schedule=lambda t: 1.0 + 0.05 * t,
             ep_time=30.0)
    # sorted neighbours (k < N-1) with camera noise in both the selection and the obs pass
    gen_traj("n8k3cam", 8, 40, seed=33, k=3, ntype="ndist_nsangle", px_noise=3.0,
             repr_="cdist_cdistdot_ndist_distdot_nsangle_angledot", capture_schedule=lambda t: 0.2, ep_time=30.0)
    gen_traj("n1", 1, 60, seed=34, ntype="dist_angle", repr_="aw_awdot_dist_distdot_angle_angledot",
             capture_schedule=lambda t: 0.1, ep_time=0.4)
    # noise off (no sensor, no thrust noise): deterministic long run for fp32-vs-fp64 GPU checks
    gen_traj("n4quiet", 4, 150, seed=35, ntype="dist_angle_heading", sense=None, thrust_noise=0.0,
             repr_="cdist_cdistdot_dist_distdot_angle_angledot", capture_schedule=lambda t: 0.05, ep_time=30.0)
    for f in sorted(os.listdir(OUT)):
        if f.startswith("a_"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


def setup_stacks_a(env):
    """Drones in vertical pairs (0.3 m apart, same xy): perform_downwash's cone (downwash.py:23-49)."""
    for i, e in enumerate(env.envs):
        d = e.dynamics
        col = i // 2
        d.pos = np.array([-1.5 + col * 1.0, 0.5, 1.2 + 0.3 * (i % 2)])
        d.vel = np.zeros(3)
        d.rot = np.eye(3)
        d.omega = np.zeros(3)
        env.pos[i] = d.pos


def setup_stats_a(env):
    """Past the 1.5 s grace (tick 140 of a 3 s episode); drone pairs 4-6 cm apart (collisions after settle),
    one drone rising into the 3 m ceiling and one dropping to the floor (room lists)."""
    for e in env.envs:
        e.tick = 140
    ds = [e.dynamics for e in env.envs]
    ds[1].pos = ds[0].pos + np.array([0.05, 0.0, 0.0])
    ds[3].pos = ds[2].pos + np.array([0.0, 0.06, 0.0])
    ds[4].pos = np.array([0.5, 0.5, 2.96]); ds[4].vel = np.array([0.0, 0.0, 3.0])
    ds[5].pos = np.array([-0.5, 0.5, 0.08]); ds[5].vel = np.array([0.0, 0.0, -3.0])
    for i, d in enumerate(ds):
        env.pos[i] = d.pos


def main_extra(which):
    """Fixtures added later, generated on their own (the ones above stay byte-identical):
      dw     use_downwash (quadrotor_multi_rewards.py:810-815) with stacked drone pairs, 8 drones
      stats  episode_extra_stats of the episodes that end (quadrotor_multi_rewards.py:886-969)
      info   every agent's per-step infos["goal_dist"] (quadrotor_single_rewards.py:457), captures and timeouts
      n128   the paper's largest swarm (paper/fps_compare.py:7): 128 drones, the 7 nearest by the camera key (k < N - 1:
             the selection pass over every pair, then the obs pass), five steps"""
    os.makedirs(OUT, exist_ok=True)
    if "dw" in which:
        gen_traj("n8dw", 8, 40, seed=36, ntype="dist_angle", repr_="cdist_cdistdot_dist_distdot_angle_angledot",
                 capture_schedule=lambda t: 0.05, ep_time=30.0, downwash=True, setup=setup_stacks_a)
    if "info" in which:
        gen_traj("n4info", 4, 120, seed=38, capture_schedule=lambda t: 3.0 if t >= 100 else 0.3, ep_time=0.8,
                 infos=True)
    if "n128" in which:
        gen_traj("n128k7", 128, 5, seed=39, k=7, capture_schedule=lambda t: 0.5, ep_time=30.0)
    if "stats" in which:
        gen_traj("n8stats", 8, 40, seed=37, ntype="dist_angle", repr_="cdist_cdistdot_dist_distdot_angle_angledot",
                 capture_schedule=lambda t: 0.01, ep_time=3.0, setup=setup_stats_a, stats=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        main_extra(sys.argv[1:])
    else:
        main()
