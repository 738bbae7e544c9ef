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


def test_pack_x3_layout_and_split_accuracy():
    """pack_mfma_weight_x3: lane l of (column tile ct, step s) holds hi / lo halves of
    256 W[32 ct + (l & 31)][16 s + 8 (l >> 5) + j]; (hi + lo) / 256 reproduces W to 2^-22 relative."""
    import torch
    from quadswarm_amd.policy_fused import pack_mfma_weight_x3
    g = torch.Generator().manual_seed(3)
    w = (torch.rand(64, 48, generator=g) * 2 - 1) * 0.2
    w[0, 0], w[1, 1] = 1e-6, -3.5          # tiny and large entries
    p = pack_mfma_weight_x3(w).view(torch.float16).float()   # [ct, s, l, part, j]
    assert p.shape == (2, 3, 64, 2, 8)
    for ct in range(2):
        for s in range(3):
            for lane in (0, 5, 31, 32, 63):
                n, k0 = 32 * ct + (lane & 31), 16 * s + 8 * (lane >> 5)
                rec = (p[ct, s, lane, 0] + p[ct, s, lane, 1]) / 256.0
                want = w[n, k0:k0 + 8]
                # (lo below the f16 normal range: an absolute floor of half its subnormal spacing 2^-24, / 256)
                assert torch.all((rec - want).abs() <= 2.0 ** -21 * want.abs() + 2.0 ** -25 / 256), (ct, s, lane)
                assert torch.equal(p[ct, s, lane, 0], (want * 256.0).half().float())
