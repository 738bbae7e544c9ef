#!/usr/bin/env python
"""torch.profiler view of one PPO minibatch step at C3's update shape (262 144 samples, attention K 6, H 256, rnn 256,
fused x3 encoders): the aten ops by device time with their input shapes, to name the torch GEMMs and elementwise
passes around the fused encoder kernels.  Diagnostic.

    python tools/update_profile.py [--B 262144] [--rows 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=262144)
    ap.add_argument("--rows", type=int, default=40)
    ap.add_argument("--rollout", action="store_true", help="one rollout policy forward (FusedRolloutPolicy x3, 32768 "
                    "agents) instead of the update's minibatch step")
    a = ap.parse_args()
    from quadswarm_amd.encoder_train import FusedAttentionTrain
    from quadswarm_amd.ppo import PolicyConfig, SwarmActorCritic
    torch.manual_seed(0)
    pol = SwarmActorCritic(PolicyConfig(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=6, rnn_size=256,
                                        neighbor_hidden_size=256, act_dim=4)).cuda()
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4)
    fused = FusedAttentionTrain(pol)
    B = a.B
    obs = torch.randn(B, 54, device="cuda")
    act = torch.rand(B, 4, device="cuda") * 1.6 - 0.8
    adv = torch.randn(B, device="cuda")
    ret = torch.randn(B, device="cuda")
    old_lp = torch.randn(B, device="cuda")

    if a.rollout:
        from quadswarm_amd.policy_fused import FusedRolloutPolicy
        fp = FusedRolloutPolicy(pol, precision="x3")
        ob = obs[:32768].contiguous()

        def step():
            fp(ob)
    else:
        def step():
            _minibatch()

    def _minibatch():
        nbr = fused.encodings(obs)
        values, logp, _ = pol.evaluate_actions(obs, act, nbr=nbr, l0=fused.self_layer0, ff=fused.feed_forward)
        ad = (adv - adv.mean()) / (adv.std() + 1e-8)
        ratio = torch.exp(logp - old_lp)
        loss = -torch.min(ad * ratio, ad * torch.clamp(ratio, 0.8, 1.2)).mean() + 0.5 * F.mse_loss(ret, values.flatten())
        opt.zero_grad(set_to_none=False)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(pol.parameters(), 0.5)
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA, ProfilerActivity.CPU], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    ev = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")]
    dev = lambda e: getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)  # noqa: E731
    ev.sort(key=lambda e: -dev(e))
    tot = sum(dev(e) for e in prof.key_averages() if not e.key.startswith(("aten::", "autograd", "_Attn", "Optimizer",
                                                                         "cudaLaunch", "hipLaunch")))
    print(f"device time of the step's kernels: {tot / 1e3:.2f} ms; kernels by device time:")
    kern = [e for e in prof.key_averages() if not e.key.startswith(("aten::", "autograd", "_Attn", "Optimizer", "cudaLaunch",
                                                                     "hipLaunch", "_Feed", "_Self", "_Head"))]
    kern.sort(key=lambda e: -dev(e))
    for e in kern[:a.rows]:
        print(f"  {e.key[:70]:70s} x{e.count:3d} {dev(e) / 1e3:8.3f} ms")
    print("aten ops by device time (incl. their kernels):")
    for e in ev[:a.rows]:
        print(f"  {e.key:22s} x{e.count:3d} {dev(e) / 1e3:8.3f} ms  {str(e.input_shapes)[:150]}")


if __name__ == "__main__":
    main()
