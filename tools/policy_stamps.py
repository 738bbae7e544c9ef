#!/usr/bin/env python
"""Diagnostic: per-phase cycle budget of the fused attention-encoder kernels (csrc/qs_policy.h) from
s_memtime stamps (the QS_STAMPS library: make -C quad-swarm-rl-stable-baselines3_amd stamps), C3's policy
shape (32768 agents, K 6, H 256, both towers).  Block 0 .. of the LAST launched kernel of each kind."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("QUADSWARM_LIB", os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd", "quadswarm_amd", "lib",
                                                   "libquadswarm_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

EMBED = ["stage layer-0 rows", "mfma e1 + tanh store", "mfma layer e2", "sync + tanh store", "e2 + mean store"]
POOL = ["load e2", "P + mfma a1", "sync + tanh store", "mfma a2", "sync + tanh store",
        "score/softmax/reload e2", "mfma h1", "sync + tanh store", "mfma h2", "weighted h + pool store"]


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
          f"cycles median {np.median(tot):.0f}")
    for k, n in enumerate(names):
        print(f"  {n:28s} {np.median(d[:, k]):8.0f} cycles {100 * np.median(d[:, k]) / np.median(tot):5.1f} %")


def main():
    from quadswarm_amd import _native as N
    from quadswarm_amd.policy_fused import FusedRolloutPolicy
    from quadswarm_amd.ppo import PolicyConfig, SwarmActorCritic
    B = 32768
    pc = PolicyConfig(self_obs_dim=18, neighbor_obs_dim=6, num_use_neighbor_obs=6, rnn_size=256,
                      neighbor_hidden_size=256, act_dim=4)
    pol = SwarmActorCritic(pc).cuda().eval()
    fp = FusedRolloutPolicy(pol)
    obs = torch.randn(B, 54, device="cuda")
    L = N.lib()
    L.qs_debug_stamps_policy.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    nb = -(-B * 6 // 60)
    with torch.no_grad():
        for _ in range(3):
            fp.neighbor_encodings(obs)
        torch.cuda.synchronize()
        # embed only (its stamps), then the pool kernel overwrites them
        fp.neighbor_encodings(obs)
        torch.cuda.synchronize()
    report(L, "pool", POOL, nb)
    # the embed kernel alone: launch stage 1 again
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    N.check(L.qs_attn_embed(ctypes.c_void_p(obs.data_ptr()), 54, 18, 18, B, 6, 6, 256, fp.towers, 2, st), "embed")
    torch.cuda.synchronize()
    report(L, "embed", EMBED, nb)


if __name__ == "__main__":
    main()
