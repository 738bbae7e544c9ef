"""Diagnostic: flavor-A downwash, GPU vs oracle on one stacked pair (prints per-drone state differences)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O  # noqa: E402
from parity_utils import gpu_to_oracle_a, oracle_params_a, oracle_to_gpu_a  # noqa: E402
from quadswarm_amd import QuadSwarmConfig  # noqa: E402
from quadswarm_amd.env import QuadSwarmEnv  # noqa: E402

for ticks in (1, 8):
    cfg = QuadSwarmConfig.sb_train(num_envs=4, num_agents=2, neighbor_obs_type="dist_angle", use_downwash=True,
                                   seed=3, ticks_per_step=ticks)
    env = QuadSwarmEnv(cfg)
    oenv = O.OracleEnvA(oracle_params_a(cfg), seed=3)
    oenv.set_capture_radius(0.01)
    env.reset()
    oenv.reset()
    for e in range(4):
        lo, hi = oenv.drones[2 * e], oenv.drones[2 * e + 1]
        hi.pos[0], hi.pos[1], hi.pos[2] = lo.pos[0] + 0.05, lo.pos[1], lo.pos[2] + 0.3
        for c in range(3):
            lo.vel[c] = hi.vel[c] = 0.0
        oenv.envs[e].capture_radius = 0.01
    oracle_to_gpu_a(oenv, env)
    a = np.zeros((8, 2), np.float32)
    env.step(torch.from_numpy(a).cuda())
    oenv.step(a.astype(np.float64))
    f = env.drone_fields()
    gv = f["vel"].double().cpu().numpy()
    ov = np.array([oenv.drones[g].vel[:] for g in range(8)])
    gw = f["omega"].double().cpu().numpy()
    ow = np.array([oenv.drones[g].omega[:] for g in range(8)])
    print("ticks", ticks)
    print("gpu vel", gv[:4])
    print("orc vel", ov[:4])
    print("gpu om", gw[:4])
    print("orc om", ow[:4])
