"""Host-side pieces of the fused rollout forward: the matrix-core weight layout (quadswarm.h qs_attn_tower)
and the C ABI's argument checks (no device needed: they fail before any HIP call)."""
import ctypes

import torch

from quadswarm_amd import _native as N
from quadswarm_amd.policy_fused import pack_mfma_weight, supports
from quadswarm_amd.ppo import PolicyConfig, SwarmActorCritic


def test_pack_layout():
    for n, kd in ((64, 16), (256, 256), (128, 128)):
        w = torch.arange(n * kd, dtype=torch.float32).view(n, kd)
        p = pack_mfma_weight(w).view(-1)
        G = kd // 8
        for ct in range(n // 32):
            for g in range(0, G, max(1, G // 4)):
                for lane in (0, 7, 31, 32, 50, 63):
                    for u in range(4):
                        row, k = 32 * ct + (lane & 31), (lane >> 5) * (kd // 2) + 4 * g + u
                        assert p[((ct * G + g) * 64 + lane) * 4 + u] == w[row, k]
        assert p.numel() == n * kd


def test_supports():
    assert supports(SwarmActorCritic(PolicyConfig(neighbor_hidden_size=256, num_use_neighbor_obs=6,
                                                  neighbor_obs_dim=6, self_obs_dim=18)))
    assert not supports(SwarmActorCritic(PolicyConfig(neighbor_hidden_size=64)))
    assert not supports(SwarmActorCritic(PolicyConfig(neighbor_encoder_type="mean_embed")))
    assert not supports(SwarmActorCritic(PolicyConfig(neighbor_hidden_size=256, self_obs_dim=30, neighbor_obs_dim=6)))


def test_abi_argument_checks():
    L = N.lib()
    towers = (N.QsAttnTower * 2)()
    for args, msg in (((4096, 6, 100), b"hidden size"), ((4096, 0, 256), b"neighbours"),
                      ((0, 6, 256), b"B must")):
        assert L.qs_attn_pool(*args, towers, 2, None) == -1
        assert msg in L.qs_last_error()
    assert L.qs_attn_pool(4096, 6, 256, towers, 3, None) == -1
    assert L.qs_attn_pool(4096, 6, 256, towers, 1, None) == -1           # NULL tower pointers
    assert b"NULL" in L.qs_last_error()
    assert L.qs_attn_embed(ctypes.c_void_p(16), 54, 18, 18, 4096, 6, 20, 256, towers, 1, None) == -1
    assert b"features per neighbour" in L.qs_last_error()
    assert L.qs_attn_embed(ctypes.c_void_p(16), 40, 18, 18, 4096, 6, 6, 256, towers, 1, None) == -1
    assert b"outside" in L.qs_last_error()
    assert L.qs_attn_embed(ctypes.c_void_p(16), 54, 60, 18, 4096, 6, 6, 256, towers, 1, None) == -1
    assert b"self features" in L.qs_last_error()
    assert L.qs_attn_embed(ctypes.c_void_p(16), 54, 30, 18, 4096, 6, 6, 256, towers, 1, None) == -1
    assert b"<= 32" in L.qs_last_error()
