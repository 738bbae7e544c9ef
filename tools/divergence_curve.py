#!/usr/bin/env python
"""Divergence-time curve (SURVEY §8c tolerance plan: "position error <= 1e-3 m after 100 control ticks for noise-off
B ... report the divergence-time curve"): the reference's own noise-free trajectories replayed on the GPU, the
largest position / self-obs error over the drones that are still airborne, per control tick.

    python tools/divergence_curve.py [traj_n8quiet traj_n4wallquiet ...]      (needs the GPU)

Prints one line per tick and a summary (the first tick each error bound is crossed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
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


if __name__ == "__main__":
    for nm in (sys.argv[1:] or ["traj_n8quiet", "traj_n4wallquiet"]):
        curve(nm)
