#!/usr/bin/env python
"""Diagnostic: where one rollout step of the bench's end-to-end PPO leg goes (C3 by default): the env step,
the policy forward (actor + critic towers) and its parts, each timed with HIP events over REPS calls."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    import bench
    from quadswarm_amd.env import QuadSwarmEnv
    from quadswarm_amd.ppo import SwarmActorCritic, use_gemm_table

    config = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = bench.make_cfg(bench.CONFIGS[config], seed=0, specialize=True)
    env = QuadSwarmEnv(cfg)
    obs = env.reset()
    pc, pcfg, _ = bench.e2e_settings(cfg)
    print("gemm table:", use_gemm_table())
    torch.manual_seed(0)
    pol = SwarmActorCritic(pc).cuda().eval()
    a = torch.rand(env.I, cfg.act_dim, device="cuda") * 2 - 1
    enc = pol.actor_encoder
    so, na = enc.cfg.self_obs_dim, enc.all_neighbor_obs_size
    self_obs = obs[:, :so]
    nbr = obs[:, so:so + na].reshape(obs.shape[0], enc.cfg.num_use_neighbor_obs, -1)
    with torch.no_grad():
        rows = [("env.step", lambda: env.step(a)),
                ("policy forward (actor+critic, sample)", lambda: pol(obs)),
                ("actor encoder", lambda: enc(obs)),
                ("  self encoder", lambda: enc.self_encoder(self_obs)),
                ("  neighbour encoder", lambda: enc.neighbor_encoder(self_obs, nbr)),
                ("critic value", lambda: pol.predict_values(obs))]
        from quadswarm_amd.policy_fused import FusedRolloutPolicy
        fp = FusedRolloutPolicy(pol)
        fp.refresh()
        fx = FusedRolloutPolicy(pol, precision="x3")
        fx.refresh()
        rows += [("fused policy forward (actor+critic)", lambda: fp(obs)),
                 ("  fused neighbour encoders (both towers)", lambda: fp.neighbor_encodings(obs)),
                 ("fused policy forward, x3 (split f16)", lambda: fx(obs)),
                 ("  fused neighbour encoders, x3", lambda: fx.neighbor_encodings(obs))]
        e32 = fp.neighbor_encodings(obs).clone()
        ex3 = fx.neighbor_encodings(obs).clone()
        print(f"max |x3 - fp32| encoder outputs: {(e32 - ex3).abs().max().item():.3e}")
        for name, fn in rows:
            print(f"{name:42s} {timed(fn):8.3f} ms")


if __name__ == "__main__":
    main()
