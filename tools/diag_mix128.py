"""Diagnostic (GPU box): which envs of a 128-drone flavor-A mix reset differ from the oracle, with their scenario,
formation and the per-env position / goal / obs error."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O  # noqa: E402
from parity_utils import oracle_params_a  # noqa: E402
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402


def main():
    N, E = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 16
    cfg = QuadSwarmConfig.sb_train(num_envs=E, seed=11, num_agents=N, neighbor_visible_num=4,
                                   neighbor_obs_type="dist_angle", quads_mode="mix")
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnvA(oracle_params_a(cfg), seed=11)
    oenv.set_capture_radius(cfg.initial_capture_radius)
    obs = env.reset().double().cpu().numpy()
    want, _ = oenv.reset()
    f = env.drone_fields()
    pos = f["pos"].double().cpu().numpy()
    goal = f["goal"].double().cpu().numpy() if "goal" in f else None
    for e in range(E):
        sl = slice(e * N, (e + 1) * N)
        sc = oenv.envs[e].scen
        opos = np.array([oenv.drones[g].pos[:] for g in range(e * N, (e + 1) * N)])
        ogoal = np.array([oenv.drones[g].goal[:] for g in range(e * N, (e + 1) * N)])
        d_obs = np.abs(obs[sl] - want[sl])
        print(f"env {e}: mode {sc.mode} form {sc.formation} size {sc.size:.4f} | pos err {np.abs(pos[sl] - opos).max():.2e}"
              f" goal err {np.abs(goal[sl] - ogoal).max() if goal is not None else float('nan'):.2e}"
              f" | obs rows off {(d_obs.max(1) > 3e-4).sum()} self-col max {d_obs[:, :7].max():.2e}")


if __name__ == "__main__":
    main()
