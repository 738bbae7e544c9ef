#!/usr/bin/env python
"""Bitwise A/B of the drone-pair impulse schedule (QS_PAIR_ROUNDS rounds of disjoint pairs vs one pair per iteration)
on crowded swarms: every env's drones packed into a small cube after the reset, so that many pairs collide in the same
step (chains of pairs sharing drones included); digests of obs / rewards / dones per step and the final state, for
specialised kernels compiled with and without QS_PAIR_ROUNDS.  Diagnostic.

    python tools/pair_bitwise.py [steps]"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "quad-swarm-rl-stable-baselines3_amd"))


def digest(n, steps, opts, side):
    import torch
    from quadswarm_amd import QuadSwarmConfig, _native as NAT
    from quadswarm_amd.env import QuadSwarmEnv
    os.environ["QS_JIT_OPTS"] = opts
    E = max(8, 2048 // n)
    cfg = QuadSwarmConfig(num_envs=E, num_agents=n, neighbor_visible_num=min(6, n - 1), neighbor_obs_type="pos_vel",
                          seed=4, specialize=True)
    env = QuadSwarmEnv(cfg, device="cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(7)
    pos = env.state[NAT.F_POS:NAT.F_POS + 3]
    pos.copy_(torch.rand(3, env.I, device="cuda:0", generator=g) * side + torch.tensor([[0.], [0.], [2.]], device="cuda:0"))
    vel = env.state[NAT.F_VEL:NAT.F_VEL + 3]
    vel.copy_(torch.randn(3, env.I, device="cuda:0", generator=g))
    acts = (torch.rand(env.I, 4, device="cuda:0", generator=g) * 2 - 1).contiguous()
    h = hashlib.sha256()
    events = 0
    for _ in range(steps):
        obs, rew, done, _ = env.step(acts)
        for t in (obs, rew, done):
            h.update(t.detach().cpu().numpy().tobytes())
        events += int((rew < -0.5).sum())
    h.update(env.get_state())
    env.close()
    return h.hexdigest(), events


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    bad = 0
    for n, side in ((8, 0.15), (8, 0.4), (16, 0.3), (32, 0.5), (4, 0.1)):
        a, ev = digest(n, steps, "-DQS_PAIR_ROUNDS=0", side)
        b, _ = digest(n, steps, "", side)
        bad += a != b
        print(f"N={n:3d} cube {side} m: {'same' if a == b else 'DIFF'} {a[:16]} {b[:16]} (collision-penalised rows {ev})",
              flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
