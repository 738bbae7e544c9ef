#!/usr/bin/env python
"""Bitwise A/B of the flavor-B goal-scenario kernels: for each (quads_mode, drones) case, K steps of a specialised
env compiled from the current sources and from a base source directory (QS_JIT_SRC_DIR, e.g. tools/jit/base_r06 =
the kernels of an earlier commit with this library's ABI: `git show <rev>:<file>` of the six kernel headers and
include/quadswarm.h), digests of obs / rewards / dones every step plus the final env state.  Diagnostic.

    python tools/scen_bitwise.py tools/jit/base_r06 [steps] [mode:N ...]"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "quad-swarm-rl-stable-baselines3_amd"))

CASES = ["mix:8", "dynamic_formations:8", "dynamic_diff_goal:8", "swarm_vs_swarm:8", "swap_goals:8",
         "ep_rand_bezier:8", "ep_lissajous3D:8", "run_away:8", "dynamic_same_goal:8", "static_diff_goal:8",
         "mix:1", "mix:2", "swarm_vs_swarm:2", "swarm_vs_swarm:4", "swarm_vs_swarm:5", "dynamic_diff_goal:2",
         "dynamic_formations:2", "mix:4", "mix:5", "mix:16", "mix:32", "mix:64", "dynamic_formations:64",
         "swarm_vs_swarm:128", "mix:128"]


def digest(mode, n, steps, src):
    import torch
    from quadswarm_amd import QuadSwarmConfig
    from quadswarm_amd.env import QuadSwarmEnv
    if src:
        os.environ["QS_JIT_SRC_DIR"] = src
    else:
        os.environ.pop("QS_JIT_SRC_DIR", None)
    E = max(8, 2048 // n)
    cfg = QuadSwarmConfig(num_envs=E, num_agents=n, neighbor_visible_num=min(6, n - 1),
                          neighbor_obs_type="pos_vel" if n > 1 else "none", quads_mode=mode, seed=3,
                          episode_duration=7.0, specialize=True)
    env = QuadSwarmEnv(cfg, device="cuda:0")
    assert env.specialized
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    acts = (torch.rand(env.I, 4, device="cuda:0", generator=g) * 2 - 1).contiguous()
    env.reset()
    h = hashlib.sha256()
    for _ in range(steps):
        obs, rew, done, _ = env.step(acts)
        for t in (obs, rew, done):
            h.update(t.detach().cpu().numpy().tobytes())
    # the final state: drone state, env ints and env floats (the base tree has this library's ABI -- the library
    # refuses another -- so the same layout)
    h.update(env.state.cpu().numpy().tobytes())
    h.update(env.env_state.cpu().numpy().tobytes())
    h.update(env.env_f.cpu().numpy().tobytes())
    env.close()
    return h.hexdigest()


def main():
    base = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1600
    cases = sys.argv[3:] or CASES
    bad = 0
    for c in cases:
        mode, n = c.split(":")
        a = digest(mode, int(n), steps, base)
        b = digest(mode, int(n), steps, None)
        ok = a == b
        bad += not ok
        print(f"{c:24s} {'same' if ok else 'DIFF'} {a[:16]} {b[:16]}", flush=True)
    print(f"{len(cases) - bad}/{len(cases)} bitwise identical")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
