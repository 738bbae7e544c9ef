#!/usr/bin/env python
"""Generate golden fixtures from the reference (TEST INFRASTRUCTURE, run in the dev container only).

    python tools/gen_golden.py            # writes tests/golden/*.npz

Imports the read-only reference (/root/reference) through tools/refshim.py and records
inputs/outputs of the hot-path functions, plus every value the reference draws from
np.random (its "tape"), so the CPU oracle can replay the exact same random numbers and be
pinned bit-for-bit.  The GPU box never runs this; it only sees the committed .npz files.

Fixtures (all plain numeric arrays, np.load(allow_pickle=False)):
  params.npz        derived Crazyflie constants (QuadrotorDynamics.update_model)
  dyn_substep.npz   QuadrotorDynamics.step1_numba on edge-case states (floor, flips, walls, SVD)
  ou.npz            OUNoiseNumba.noise sequences
  sensor.npz        SensorNoise.add_noise_numba with recorded draws (+ bypass obs)
  collisions.npz    collision matrix / proximity / drone, wall, ceiling impulses (recorded draws)
  neighbors.npz     QuadrotorEnvMulti.add_neighborhood_obs (pos_vel), N=8 k=6/2/7 and N=32 k=6
  traj_*.npz        whole QuadrotorEnvMulti.step trajectories with the recorded tape
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

refshim.install()
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")

# ---------------------------------------------------------------------------------------------
# draw recording
# ---------------------------------------------------------------------------------------------
_orig = {"normal": np.random.normal, "uniform": np.random.uniform, "randn": np.random.randn}


class Tape:
    def __init__(self):
        self.vals = []
        self.spawn = []
        self.on = False


TAPE = Tape()


def _wrap(name):
    f = _orig[name]

    def g(*a, **k):
        v = f(*a, **k)
        if TAPE.on:
            TAPE.vals.extend(np.ravel(np.asarray(v, dtype=np.float64)).tolist())
        return v
    return g


np.random.normal = _wrap("normal")
np.random.uniform = _wrap("uniform")
np.random.randn = _wrap("randn")
import gym_art.quadrotor_multi.sensor_noise as _sn  # noqa: E402

_sn.normal = np.random.normal
_sn.uniform = np.random.uniform


class GenProxy:
    """Wraps the env's np.random.Generator; records the spawn draws (uniform, size=(3,))."""

    def __init__(self, g):
        self._g = g

    def uniform(self, *a, **k):
        v = self._g.uniform(*a, **k)
        size = k.get("size", a[2] if len(a) > 2 else None)
        if TAPE.on and size == (3,):
            TAPE.spawn.extend(np.ravel(v).tolist())
        return v

    def __getattr__(self, n):
        return getattr(self._g, n)


def begin():
    TAPE.vals, TAPE.spawn, TAPE.on = [], [], True


def end():
    TAPE.on = False
    return np.array(TAPE.vals, dtype=np.float64), np.array(TAPE.spawn, dtype=np.float64)


# ---------------------------------------------------------------------------------------------
from gym_art.quadrotor_multi.quad_models import crazyflie_params  # noqa: E402
from gym_art.quadrotor_multi.quadrotor_dynamics import QuadrotorDynamics  # noqa: E402
from gym_art.quadrotor_multi.numba_utils import OUNoiseNumba  # noqa: E402
from gym_art.quadrotor_multi.sensor_noise import SensorNoise  # noqa: E402
from gym_art.quadrotor_multi.collisions.quadrotors import (  # noqa: E402
    calculate_collision_matrix, calculate_drone_proximity_penalties, perform_collision_between_drones)
from gym_art.quadrotor_multi.collisions.room import perform_collision_with_wall, perform_collision_with_ceiling  # noqa: E402
from gym_art.quadrotor_multi import get_state  # noqa: E402

REW = dict(pos=1.0, effort=0.05, spin=0.1, vel=0.0, crash=1.0, orient=1.0, yaw=0.0,
           quadcol_bin=5.0, quadcol_bin_smooth_max=10.0, quadcol_bin_obst=0.0)


def rand_rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def make_dyn():
    return QuadrotorDynamics(crazyflie_params(), room_box=np.array([[-5., -5., 0.], [5., 5., 10.]]),
                             dynamics_steps_num=2, use_numba=True, dt=0.005)


def gen_params():
    d = make_dyn()
    np.savez_compressed(os.path.join(OUT, "params.npz"), mass=d.mass, inertia=d.inertia,
                        thrust_max=d.thrust_max, torque_max=d.torque_max, prop_cross=d.prop_crossproducts,
                        prop_ccw=d.prop_ccw, arm=d.arm, motor_tau_up=d.motor_tau_up,
                        motor_tau_down=d.motor_tau_down, prop_pos=d.prop_pos)


def gen_dyn_substep(n=400, seed=1):
    rng = np.random.default_rng(seed)
    d = make_dyn()
    fields = {k: [] for k in ["pos", "vel", "rot", "omega", "rd", "cd", "since", "on_floor", "cmds", "noise",
                              "o_pos", "o_vel", "o_rot", "o_omega", "o_acc", "o_rd", "o_cd", "o_since",
                              "o_on_floor", "o_crashed_floor", "o_crashed_wall", "o_crashed_ceiling",
                              "tape_start", "tape_len"]}
    tape_all = []
    for c in range(n):
        kind = c % 8
        pos = rng.uniform([-4.5, -4.5, 0.5], [4.5, 4.5, 9.5])
        vel = rng.uniform(-3, 3, 3)
        rot = rand_rot(rng)
        omega = rng.uniform(-20, 20, 3)
        on_floor = False
        since = float(rng.uniform(0, 0.45))
        if kind == 1:   # floor first hit (sometimes upside down -> random yaw draw)
            pos[2] = rng.uniform(0.0, 0.05)
            vel[2] = -abs(vel[2])
        elif kind == 2:  # resting on floor, zero velocity (static friction branch)
            pos[2] = rng.uniform(0.0, 0.04)
            vel[:] = 0.0
            on_floor = True
            rot = np.array([[np.cos(0.3), -np.sin(0.3), 0], [np.sin(0.3), np.cos(0.3), 0], [0, 0, 1.]])
            rot = rot @ rand_rot(rng) if rng.uniform() < 0.5 else rot
        elif kind == 3:  # sliding on floor
            pos[2] = rng.uniform(0.0, 0.04)
            on_floor = True
        elif kind == 4:  # wall / ceiling crossing
            pos = np.array([rng.choice([-4.999, 4.999]), rng.uniform(-4, 4), rng.choice([5.0, 9.999])])
            vel = rng.uniform(-3, 3, 3) * 3
        elif kind == 5:  # SVD due within the step (0.5 s threshold)
            since = 0.5 - 0.005 * rng.uniform(0.2, 1.8)
            rot = rot + rng.normal(scale=1e-4, size=(3, 3))
        elif kind == 6:  # omega clip
            omega = rng.uniform(-45, 45, 3)
        rd = rng.uniform(0, 1, 4)
        cd = np.clip(rd ** 2 + rng.normal(scale=0.01, size=4), 0, 1)
        cmds = rng.uniform(-0.2, 1.2, 4)
        noise = rng.normal(scale=0.02, size=4)
        d.pos, d.vel, d.rot, d.omega = pos.copy(), vel.copy(), rot.copy(), omega.copy()
        d.thrust_rot_damp, d.thrust_cmds_damp = rd.copy(), cd.copy()
        d.since_last_svd, d.on_floor = since, on_floor
        for k, v in [("pos", pos), ("vel", vel), ("rot", rot), ("omega", omega), ("rd", rd), ("cd", cd),
                     ("since", since), ("on_floor", on_floor), ("cmds", cmds), ("noise", noise)]:
            fields[k].append(np.array(v, dtype=np.float64))
        begin()
        d.step1_numba(cmds, 0.005, noise)
        tv, _ = end()
        fields["tape_start"].append(len(tape_all))
        fields["tape_len"].append(len(tv))
        tape_all.extend(tv.tolist())
        for k, v in [("o_pos", d.pos), ("o_vel", d.vel), ("o_rot", d.rot), ("o_omega", d.omega),
                     ("o_acc", d.acc), ("o_rd", d.thrust_rot_damp), ("o_cd", d.thrust_cmds_damp),
                     ("o_since", d.since_last_svd), ("o_on_floor", d.on_floor),
                     ("o_crashed_floor", d.crashed_floor), ("o_crashed_wall", d.crashed_wall),
                     ("o_crashed_ceiling", d.crashed_ceiling)]:
            fields[k].append(np.array(v, dtype=np.float64))
    out = {k: np.stack(v) for k, v in fields.items()}
    out["tape"] = np.array(tape_all)
    np.savez_compressed(os.path.join(OUT, "dyn_substep.npz"), **out)


def gen_ou(n=200, seed=2):
    np.random.seed(seed)
    ou = OUNoiseNumba(4, sigma=0.2 * 0.05)
    begin()
    seq = np.stack([np.array(ou.noise()) for _ in range(n)])
    tv, _ = end()
    np.savez_compressed(os.path.join(OUT, "ou.npz"), seq=seq, tape=tv, theta=ou.theta, sigma=ou.sigma)


def gen_sensor(n=300, seed=3):
    rng = np.random.default_rng(seed)
    np.random.seed(seed)
    sn = SensorNoise(bypass=False, use_numba=True)
    ins = {k: [] for k in ["pos", "vel", "rot", "omega", "acc"]}
    outs = {k: [] for k in ["n_pos", "n_vel", "n_rot", "n_omega"]}
    tapes = []
    for c in range(n):
        pos, vel, omega, acc = rng.uniform(-5, 5, 3), rng.uniform(-3, 3, 3), rng.uniform(-30, 30, 3), rng.uniform(-20, 20, 3)
        rot = rand_rot(rng)
        if c % 4 == 1:  # non-orthonormal drift, exercises the quaternion round trip
            rot = rot + rng.normal(scale=1e-3, size=(3, 3))
        if c % 4 == 2:  # large rotations: trace <= 0 branches
            rot = np.diag([1., -1., -1.]) @ rand_rot(rng) if c % 8 == 2 else np.diag([-1., 1., -1.])
        begin()
        npos, nvel, nrot, nomega, _ = sn.add_noise_numba(pos, vel, rot, omega, acc, 0.005)
        tv, _ = end()
        tapes.append(tv)
        for k, v in zip(ins, [pos, vel, rot, omega, acc]):
            ins[k].append(v)
        for k, v in zip(outs, [npos, nvel, nrot, nomega]):
            outs[k].append(v)
    out = {k: np.stack(v) for k, v in {**ins, **outs}.items()}
    out["tape"] = np.stack(tapes)
    # bypass observation packing (get_state.py:226-292)

    class Fake:
        pass
    f = Fake()
    f.use_numba = True
    f.sense_noise = SensorNoise(bypass=True)
    f.dt = 0.005
    f.room_box = np.array([[-5., -5., 0.], [5., 5., 10.]])
    obs18, obs19, obs24, goals = [], [], [], []
    for c in range(50):
        f.dynamics = make_dyn()
        f.dynamics.accelerometer = np.array([0.0, 0.0, 9.81])
        f.dynamics.pos, f.dynamics.vel = rng.uniform(-5, 5, 3), rng.uniform(-3, 3, 3)
        f.dynamics.rot, f.dynamics.omega = rand_rot(rng), rng.uniform(-9, 9, 3)
        f.dynamics.pos[2] = abs(f.dynamics.pos[2]) * 2
        f.goal = rng.uniform(-2, 2, 3)
        obs18.append(np.concatenate([f.dynamics.pos, f.dynamics.vel, f.dynamics.rot.ravel(), f.dynamics.omega, f.goal]))
        obs19.append(get_state.state_xyz_vxyz_R_omega_floor(f))
        obs24.append(get_state.state_xyz_vxyz_R_omega_wall(f))
        goals.append(get_state.state_xyz_vxyz_R_omega(f))
    out["bp_in"] = np.stack(obs18)
    out["bp_obs18"] = np.stack(goals)
    out["bp_obs19"] = np.stack(obs19)
    out["bp_obs24"] = np.stack(obs24)
    np.savez_compressed(os.path.join(OUT, "sensor.npz"), **out)


def gen_collisions(seed=4):
    rng = np.random.default_rng(seed)
    np.random.seed(seed)
    out = {}
    # collision matrix + proximity: clustered positions
    P, M, D, PEN = [], [], [], []
    arm = make_dyn().arm
    for c in range(100):
        pos = rng.uniform(-0.3, 0.3, (8, 3)) + np.array([0, 0, 2.0])
        col, pairs, dm = calculate_collision_matrix(pos, 2 * arm)
        near = dm[np.where(dm[:, 2] <= 4 * arm)]
        pen = calculate_drone_proximity_penalties(near, 4 * arm, 0.01, 10.0, 8) if len(near) else np.zeros(8)
        P.append(pos); M.append(col); D.append(dm); PEN.append(pen)
    out.update(cm_pos=np.stack(P), cm_col=np.stack(M), cm_dist=np.stack(D), cm_pen=np.stack(PEN))
    # drone-drone impulses
    ins, outs, tapes = [], [], []
    for c in range(200):
        p1, p2 = rng.uniform(-1, 1, 3), rng.uniform(-1, 1, 3)
        if c % 10 == 0:
            p2 = p1.copy()       # coincident drones: EPS branch of the normal
        v1, v2 = rng.uniform(-3, 3, 3), rng.uniform(-3, 3, 3)
        if c % 10 == 1:
            v1[:] = 0.0; v2[:] = 0.0
        w1, w2 = rng.uniform(-5, 5, 3), rng.uniform(-5, 5, 3)
        ins.append(np.concatenate([p1, v1, w1, p2, v2, w2]))
        begin()
        a, b, cc, dd = perform_collision_between_drones(p1.copy(), v1.copy(), w1.copy(), p2.copy(), v2.copy(), w2.copy())
        tv, _ = end()
        tapes.append(tv)
        outs.append(np.concatenate([a, b, cc, dd]))
    L = max(len(t) for t in tapes)
    out.update(dd_in=np.stack(ins), dd_out=np.stack(outs), dd_tape=np.stack([np.pad(t, (0, L - len(t))) for t in tapes]),
               dd_tape_len=np.array([len(t) for t in tapes]))
    # wall / ceiling
    room = np.array([[-5., -5., 0.], [5., 5., 10.]])
    wi, wo, wt, ci, co, ct = [], [], [], [], [], []
    for c in range(100):
        d = make_dyn()
        pos = rng.uniform(-4, 4, 3)
        pos[2] = abs(pos[2]) + 1
        for ax in range(2):
            r = rng.uniform()
            if r < 0.3:
                pos[ax] = -5.0
            elif r < 0.6:
                pos[ax] = 5.0
        vel = rng.uniform(-4, 4, 3) * (0.0 if c % 10 == 0 else 1.0)
        d.pos, d.vel, d.omega = pos.copy(), vel.copy(), rng.uniform(-3, 3, 3)
        wi.append(np.concatenate([d.pos, d.vel, d.omega]))
        begin()
        perform_collision_with_wall(d, room)
        tv, _ = end()
        wt.append(tv)
        wo.append(np.concatenate([d.vel, d.omega]))
        d2 = make_dyn()
        d2.pos, d2.vel, d2.omega = pos.copy(), vel.copy(), rng.uniform(-3, 3, 3)
        ci.append(np.concatenate([d2.pos, d2.vel, d2.omega]))
        begin()
        perform_collision_with_ceiling(d2)
        tv, _ = end()
        ct.append(tv)
        co.append(np.concatenate([d2.vel, d2.omega]))
    Lw = max(len(t) for t in wt)
    out.update(wall_in=np.stack(wi), wall_out=np.stack(wo),
               wall_tape=np.stack([np.pad(t, (0, Lw - len(t))) for t in wt]),
               ceil_in=np.stack(ci), ceil_out=np.stack(co), ceil_tape=np.stack(ct))
    np.savez_compressed(os.path.join(OUT, "collisions.npz"), **out)


# ---------------------------------------------------------------------------------------------
# whole-env trajectories
# ---------------------------------------------------------------------------------------------
def make_env_B(n, k, obs_type="pos_vel", ep_time=15.0, downwash=False, sense="default", thrust_noise=0.05,
               obs_repr="xyz_vxyz_R_omega", seed=0):
    from gym_art.quadrotor_multi.quadrotor_multi import QuadrotorEnvMulti

    class Cfg:
        pass
    cfg = Cfg()
    cfg.seed = seed
    env = QuadrotorEnvMulti(
        num_agents=n, ep_time=ep_time, rew_coeff=dict(REW), obs_repr=obs_repr, cfg=cfg,
        neighbor_visible_num=k, neighbor_obs_type=obs_type, collision_hitbox_radius=2.0,
        collision_falloff_radius=4.0, use_obstacles=False, obst_density=0.2, obst_size=1.0,
        obst_spawn_area=[6, 6], use_downwash=downwash, use_numba=True, quads_mode="static_same_goal",
        room_dims=[10, 10, 10], use_replay_buffer=False, quads_view_mode=[], quads_render=False,
        dynamics_params="Crazyflie", raw_control=True, raw_control_zero_middle=True,
        dynamics_randomize_every=None,
        dynamics_change=dict(noise=dict(thrust_noise_ratio=thrust_noise), damp=dict(vel=0, omega_quadratic=0)),
        dyn_sampler_1=None, sense_noise=sense, init_random_state=False)
    px = GenProxy(env.rng)
    env.rng = px
    env.scenario.rng = px
    for e in env.envs:
        e.rng = px
    return env


def snapshot(env):
    ds = [e.dynamics for e in env.envs]
    return dict(
        pos=np.stack([d.pos for d in ds]), vel=np.stack([d.vel for d in ds]), rot=np.stack([d.rot for d in ds]),
        omega=np.stack([np.asarray(d.omega, dtype=np.float64) for d in ds]), acc=np.stack([d.acc for d in ds]),
        rd=np.stack([d.thrust_rot_damp for d in ds]), cd=np.stack([d.thrust_cmds_damp for d in ds]),
        ou=np.stack([np.array(d.thrust_noise.state) for d in ds]),
        since=np.array([d.since_last_svd for d in ds]), on_floor=np.array([d.on_floor for d in ds], dtype=np.float64),
        goal=np.stack([e.goal for e in env.envs]), tick=np.array(env.envs[0].tick),
        env_vel=env.vel.copy())


def gen_traj(name, n, k, steps, ep_time, seed, setup=None, hover=False, stats=False, infos=False, **kw):
    np.random.seed(seed)
    env = make_env_B(n, k, ep_time=ep_time, seed=seed, **kw)
    env.reset()
    if setup is not None:
        setup(env, np.random.default_rng(seed + 100))
    init = snapshot(env)
    act_rng = np.random.default_rng(seed + 200)
    actions = act_rng.uniform(-1.0, 1.0, (steps, n, 4))
    if hover:  # ~hover thrust (cmd 1/t2w) with small perturbations: no contacts, deterministic
        actions = 0.0526 + 0.1 * actions
    elif n > 1:  # climbing thrust so drones stay airborne and interact
        actions = np.clip(actions * 0.6 + 0.3, -1, 1)
    obs, rew, done = [], [], []
    events, rinfo, rkeys = [], [], None
    begin()
    for t in range(steps):
        o, r, dn, info = env.step(actions[t])
        if infos:   # every agent's infos[i]["rewards"] (quadrotor_single.py:79-105, quadrotor_multi.py:642-651)
            rkeys = rkeys or sorted(info[0]["rewards"])
            assert all(sorted(info[i]["rewards"]) == rkeys for i in range(n))
            rinfo.append([[float(info[i]["rewards"][key]) for key in rkeys] for i in range(n)])
        obs.append(np.array(o, dtype=np.float64))
        rew.append(np.array(r, dtype=np.float64))
        done.append(np.array(dn, dtype=np.float64))
        if stats and any(dn):   # infos[i]["episode_extra_stats"] of every agent (quadrotor_multi.py:739-831)
            events.append({"step": t, "agents": [{k_: float(v) for k_, v in info[i]["episode_extra_stats"].items()}
                                                 for i in range(n)]})
    tv, sp = end()
    if stats:
        import json
        with open(os.path.join(OUT, f"traj_{name}_stats.json"), "w") as f:
            json.dump({"name": name, "events": events}, f, indent=0, sort_keys=True)
    extra = {}
    if infos:
        import json
        with open(os.path.join(OUT, f"traj_{name}_infokeys.json"), "w") as f:
            json.dump({"name": name, "rewards_keys": rkeys, "rew_coeff": REW}, f, indent=0, sort_keys=True)
        extra["info_rewards"] = np.array(rinfo, dtype=np.float64)
    final = snapshot(env)
    np.savez_compressed(os.path.join(OUT, f"traj_{name}.npz"), actions=actions, obs=np.stack(obs), **extra,
                        rew=np.stack(rew), done=np.stack(done), tape=tv, spawn=sp, n=n, k=k,
                        ep_len=env.envs[0].ep_len, downwash=int(kw.get("downwash", False)),
                        sense=int(kw.get("sense", "default") == "default"),
                        thrust_noise=kw.get("thrust_noise", 0.05),
                        **{"init_" + a: b for a, b in init.items()}, **{"final_" + a: b for a, b in final.items()})


def setup_crowd(env, rng):
    """Pull pairs of drones together (collisions) and push one at the wall / ceiling."""
    ds = [e.dynamics for e in env.envs]
    n = len(ds)
    if n >= 4:
        ds[1].pos = ds[0].pos + np.array([0.05, 0.02, 0.0])
        ds[3].pos = ds[2].pos + np.array([0.0, 0.07, 0.03])
        ds[3].vel = np.array([0.0, -0.5, 0.0])
    if n >= 6:
        ds[4].pos = np.array([4.97, 0.5, 3.0]); ds[4].vel = np.array([3.0, 0.0, 0.0])
        ds[5].pos = np.array([0.5, 0.2, 9.97]); ds[5].vel = np.array([0.0, 0.0, 4.0])
    if n >= 8:
        ds[6].pos = np.array([1.0, 1.0, 0.3]); ds[6].vel = np.array([0.0, 0.0, -2.0])
        ds[6].rot = np.diag([1.0, -1.0, -1.0])   # upside down: floor flip draws a random yaw
        ds[7].pos = ds[6].pos + np.array([0.0, 0.0, 0.4])


def setup_stack(env, rng):
    """Vertical stacks for downwash."""
    ds = [e.dynamics for e in env.envs]
    for i, d in enumerate(ds):
        col = i // 2
        d.pos = np.array([-1.0 + col * 0.8, 0.5, 1.5 + 0.3 * (i % 2)])
        d.vel = np.zeros(3)


def main():
    os.makedirs(OUT, exist_ok=True)
    gen_params()
    gen_dyn_substep()
    gen_ou()
    gen_sensor()
    gen_collisions()
    gen_neighbors()
    gen_traj("n8k6", 8, 6, 120, ep_time=0.5, seed=11, setup=setup_crowd)
    gen_traj("n8k7", 8, -1, 60, ep_time=0.3, seed=12, setup=setup_crowd)
    gen_traj("n1", 1, 0, 80, ep_time=0.4, seed=13, obs_type="none")
    gen_traj("n8dw", 8, 2, 60, ep_time=15.0, seed=14, setup=setup_stack, downwash=True)
    gen_traj("n32k6", 32, 6, 25, ep_time=0.2, seed=15, setup=setup_crowd)
    gen_traj("n8quiet", 8, 6, 300, ep_time=15.0, seed=16, hover=True, sense=None, thrust_noise=0.0)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


def gen_neighbors(seed=5):
    gen_neighbors_sizes("neighbors.npz", [(8, 6), (8, 2), (8, 7), (32, 6)], seed)


def gen_neighbors_sizes(fname, sizes, seed, count=40):
    rng = np.random.default_rng(seed)
    out = {}
    for n, k in sizes:
        env = make_env_B(n, k)
        P, V, O = [], [], []
        for c in range(count):
            env.pos = rng.uniform(-6, 6, (n, 3))
            env.vel = rng.uniform(-4, 4, (n, 3))
            if c % 5 == 0:  # near-duplicates around the 0.01 key clamp
                env.pos[1] = env.pos[0] + 1e-3
                env.vel[1] = env.vel[0]
            o = env.add_neighborhood_obs([np.zeros(18) for _ in range(n)])
            P.append(env.pos.copy()); V.append(env.vel.copy()); O.append(np.array(o)[:, 18:])
        out[f"n{n}k{k}_pos"] = np.stack(P)
        out[f"n{n}k{k}_vel"] = np.stack(V)
        out[f"n{n}k{k}_obs"] = np.stack(O)
    np.savez_compressed(os.path.join(OUT, fname), **out)


def main_extra(which):
    """Fixtures added later, generated on their own (the ones above stay byte-identical):
      wall   the xyz_vxyz_R_omega_wall self obs (get_state.py:270-292): a noisy 8-drone run with wall / ceiling
             contacts and a noise-free 4-drone hover the GPU replays
      stats  episode_extra_stats of every finished episode (quadrotor_multi.py:739-831) over 2-s episodes
      n64    a 64-drone crowded trajectory and 64-drone neighbour selections (k = 6 and all 63 visible)
      n128   a 128-drone crowded trajectory with an in-env auto-reset and 128-drone neighbour selections (k = 6, 16;
             the paper's largest swarm, paper/fps_compare.py:7)
      info   every agent's per-step infos["rewards"] dict (quadrotor_single.py:79-105, quadrotor_multi.py:642-651)
             over a crowded 8-drone run with an in-env auto-reset"""
    os.makedirs(OUT, exist_ok=True)
    if "wall" in which:
        gen_traj("n8wall", 8, 6, 120, ep_time=0.5, seed=17, setup=setup_crowd, obs_repr="xyz_vxyz_R_omega_wall")
        gen_traj("n4wallquiet", 4, 3, 150, ep_time=15.0, seed=18, hover=True, sense=None, thrust_noise=0.0,
                 obs_repr="xyz_vxyz_R_omega_wall")
    if "stats" in which:
        gen_traj("n8stats", 8, 6, 420, ep_time=2.0, seed=19, setup=setup_crowd, stats=True)
    if "info" in which:
        gen_traj("n8info", 8, 6, 60, ep_time=0.3, seed=21, setup=setup_crowd, infos=True)
    if "n64" in which:   # 64-drone swarms: the first size past one drone per lane of a wave with Q > 1
        gen_traj("n64k6", 64, 6, 25, ep_time=0.2, seed=20, setup=setup_crowd)
        gen_neighbors_sizes("neighbors64.npz", [(64, 6), (64, 63)], seed=6, count=10)
    if "n128" in which:  # 128-drone swarms: an env spans two waves (a 128-lane workgroup)
        gen_traj("n128k6", 128, 6, 14, ep_time=0.1, seed=22, setup=setup_crowd)
        gen_neighbors_sizes("neighbors128.npz", [(128, 6), (128, 16)], seed=7, count=6)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        main_extra(sys.argv[1:])
    else:
        main()
