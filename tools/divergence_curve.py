#!/usr/bin/env python
"""Divergence-time curve (SURVEY §8c tolerance plan: "position error <= 1e-3 m after 100 control ticks for noise-off
B ... report the divergence-time curve"): the reference's own noise-free trajectories replayed on the GPU, the
largest position / self-obs error over the drones that are still airborne, per control tick.

    python tools/divergence_curve.py [traj_n8quiet traj_n4wallquiet a_traj_n4quiet ...]      (needs the GPU)

Flavor A (a_traj_*): the fixture holds the reference's observations per step but its positions only at the end, so
the per-step position error is taken against the C oracle stepped alongside (identical Philox draws, the oracle
itself pinned to this reference trajectory draw for draw by tests/test_oracle_golden_a.py), the obs error against
the reference's own observations.

Prints one line per tick and a summary (the first tick each error bound is crossed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))   # oracle/oracle.py (not the oracle/ directory as a package)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def curve(name):
    from quadswarm_amd import QuadSwarmConfig
    from quadswarm_amd.env import QuadSwarmEnv
    from test_gpu_parity import _load_initial_state
    g = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"), allow_pickle=False)
    n, k = int(g["n"]), int(g["k"])
    so = g["obs"].shape[-1] - 6 * k
    rep = {18: "xyz_vxyz_R_omega", 19: "xyz_vxyz_R_omega_floor", 24: "xyz_vxyz_R_omega_wall"}[so]
    cfg = QuadSwarmConfig(num_envs=1, num_agents=n, neighbor_visible_num=k, sense_noise=None, thrust_noise_ratio=0.0,
                          episode_duration=15.0, obs_repr=rep)
    env = QuadSwarmEnv(cfg)
    env.reset()
    _load_initial_state(env, g, n)
    airborne = np.ones(n, bool)
    rows = []
    for t in range(len(g["actions"])):
        obs, _, _, _ = env.step(torch.from_numpy(g["actions"][t].astype(np.float32)).cuda())
        o = obs.double().cpu().numpy()
        want = g["obs"][t]
        airborne &= (want[:, 2] + 2.0) > 0.3
        if not airborne.any():
            break
        dp = np.abs(o[airborne, 0:3] - want[airborne, 0:3]).max()
        ds = np.abs(o[airborne, :so] - want[airborne, :so]).max()
        rows.append((t + 1, int(airborne.sum()), dp, ds))
    print(f"# {name}: {n} drones, control tick / drones airborne / max |pos err| m / max |self-obs err|")
    for r in rows:
        print(f"{r[0]:4d} {r[1]:2d} {r[2]:.3e} {r[3]:.3e}")
    pe = np.array([r[2] for r in rows])
    for bound in (1e-5, 1e-4, 1e-3):
        over = np.flatnonzero(pe > bound)
        print(f"# {name}: position error first above {bound:g} m at tick {rows[over[0]][0] if len(over) else 'never'}"
              f" (of {len(rows)} airborne ticks)")
    at100 = [r for r in rows if r[0] == 100]
    if at100:
        print(f"# {name}: position error at tick 100: {at100[0][2]:.3e} m")


def curve_a(name):
    from parity_utils import angle_columns_a
    from test_gpu_parity_a import load_golden_into_gpu, ostate

    def golden(n):
        return dict(np.load(os.path.join(ROOT, "tests", "golden", n + ".npz"), allow_pickle=False))
    g, cfg, env, oenv = load_golden_into_gpu(golden, name[len("a_traj_"):], with_oracle=True)
    n = int(g["n"])
    ang = set(angle_columns_a(cfg))
    dist_cols = [c for c in range(g["obs"].shape[-1]) if c not in ang]
    rows = []
    for t in range(len(g["actions"])):
        env.set_capture_radius(float(g["capture"][t]))
        oenv.set_capture_radius(float(g["capture"][t]))
        a = np.ascontiguousarray(g["actions"][t], dtype=np.float64).reshape(-1, 2)
        obs, _, _, _ = env.step(torch.from_numpy(a.astype(np.float32)).cuda())
        oenv.step(a)
        o = obs.double().cpu().numpy()
        dp = np.abs(env.drone_fields()["pos"].double().cpu().numpy() - ostate(oenv, "pos")).max()
        do = np.abs(o[:, dist_cols] - g["obs"][t][:, dist_cols]).max()
        dd = o[:, sorted(ang)] - g["obs"][t][:, sorted(ang)]
        da = np.abs((dd + np.pi) % (2 * np.pi) - np.pi).max() if ang else 0.0   # angles compared modulo 2 pi
        rows.append((8 * (t + 1), n, dp, do, da))
    print(f"# {name}: {n} drones, controller tick / drones / max |pos err| m (vs oracle) / max |obs err| non-angle "
          f"columns / angle columns (vs reference)")
    for r in rows:
        print(f"{r[0]:5d} {r[1]:2d} {r[2]:.3e} {r[3]:.3e} {r[4]:.3e}")
    fp = np.abs(env.drone_fields()["pos"].double().cpu().numpy() - g["final_pos"]).max()
    print(f"# {name}: final position error vs the reference after {8 * len(rows)} ticks: {fp:.3e} m")
    for col, label in ((2, "position"), (3, "obs (non-angle)"), (4, "obs (angle)")):
        e = np.array([r[col] for r in rows])
        for bound in (1e-5, 1e-4, 1e-3):
            over = np.flatnonzero(e > bound)
            print(f"# {name}: {label} error first above {bound:g} at tick {rows[over[0]][0] if len(over) else 'never'}")
        print(f"# {name}: {label} error max {e.max():.3e}")


if __name__ == "__main__":
    for nm in (sys.argv[1:] or ["traj_n8quiet", "traj_n4wallquiet", "a_traj_n4quiet"]):
        curve_a(nm) if nm.startswith("a_traj_") else curve(nm)
