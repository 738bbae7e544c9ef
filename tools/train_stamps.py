#!/usr/bin/env python
"""Diagnostic: per-phase cycle budget of the PPO update's fused encoder kernels (csrc/qs_policy_train.h
attn_pool_train_x3 and attn_bwd1_x3) from s_memtime stamps (the QS_STAMPS library: make -C
quad-swarm-rl-stable-baselines3_amd stamps), at C3's minibatch (262 144 agents, K 6, H 256, both towers).  Wave 0 of
every tower-0 block of the last launch of each kernel; the phases include the barrier waits of that wave.

    python tools/train_stamps.py [--B 262144]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("QUADSWARM_LIB", os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd", "quadswarm_amd", "lib",
                                                   "libquadswarm_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

POOL = ["bias / P / e2 loads", "mfma a1", "a1 tanh + stores", "mfma a2", "a2 stores + score", "softmax + e2 reload",
        "mfma v1", "v1 tanh + stores", "mfma v2", "h stores + weighted tile", "pooled out"]
EMBED = ["bias + layer-0 gather", "mfma e1", "e1 tanh + stores", "mfma e2", "e2 epilogue + e_mean", "-"]
BWD1 = ["dout / w3 / w loads", "stage dh (h loads, stores)", "mfma v2t", "dv1 epilogue (stores)", "mfma v1t + dev",
        "dscore", "stage da2 (a2 loads, stores)", "mfma a2t", "a1 loads + da1 epilogue", "mfma a1et", "de2p stores"]


def report(L, name, names, nb):
    buf = np.zeros(65536 * 32, np.uint64)
    assert L.qs_debug_stamps_policy(buf.ctypes.data, buf.size) == 0
    st = buf.reshape(65536, 32)[:nb].astype(np.int64)
    rt = st[:, 12:14]
    t0 = rt[:, 0].min()
    s_, e_ = (rt[:, 0] - t0) * 10, (rt[:, 1] - t0) * 10
    d = np.diff(st[:, :len(names) + 1], axis=1)
    tot = d.sum(1)
    print(f"{name}: {nb} blocks; block lifetime p50 {np.median(e_ - s_):.0f} ns, launch span {e_.max():.0f} ns; "
          f"wave-0 cycles median {np.median(tot):.0f}")
    for k, n in enumerate(names):
        print(f"  {n:30s} {np.median(d[:, k]):8.0f} cycles {100 * np.median(d[:, k]) / np.median(tot):5.1f} %"
              f"   p90 {np.percentile(d[:, k], 90):8.0f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=262144)
    a = ap.parse_args()
    from quadswarm_amd import _native as N
    from quadswarm_amd.encoder_train import FusedAttentionTrain
    from quadswarm_amd.ppo import PolicyConfig, SwarmActorCritic
    L = N.lib()
    L.qs_debug_stamps_policy.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    torch.manual_seed(0)
    pol = SwarmActorCritic(PolicyConfig(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=6, rnn_size=256,
                                        neighbor_hidden_size=256, act_dim=4)).cuda()
    obs = torch.randn(a.B, 54, device="cuda")
    fused = FusedAttentionTrain(pol)
    params = fused.params()
    g = [torch.randn(a.B, 256, device="cuda") * 1e-3 for _ in range(2)]
    nb = -(-a.B * 6 // 60)
    for it in range(3):
        outs = fused.encodings(obs)
        torch.cuda.synchronize()
        if it == 2:
            report(L, "attn_pool_train_x3", POOL, nb)
        torch.autograd.grad(sum((o * gi).sum() for o, gi in zip(outs, g)), params)
        torch.cuda.synchronize()
    report(L, "attn_bwd1_x3", BWD1, nb)
    r = fused.runner
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(L.qs_attn_embed_train_x3(ctypes.c_void_p(obs.data_ptr()), 54, 18, 18, a.B, 6, 6, 256, r.towers, r.trains, 2,
                                     st), "qs_attn_embed_train_x3")
    torch.cuda.synchronize()
    report(L, "attn_embed_train_x3", EMBED, nb)


if __name__ == "__main__":
    main()
