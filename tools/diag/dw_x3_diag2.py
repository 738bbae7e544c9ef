"""Diagnostic: which operand elements qs_attn_dw_x3 represents inexactly (one-hot partner operand)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
import torch  # noqa: E402
from quadswarm_amd.encoder_train import dw_x3, col_scales  # noqa: E402

for H in (128, 256):
    R = H
    g = torch.Generator(device="cuda").manual_seed(H)
    G = torch.randn(R, H, device="cuda", generator=g) * torch.exp2(torch.linspace(-20, 4, H, device="cuda"))
    A = torch.tanh(torch.randn(R, H, device="cuda", generator=g) * 2)
    I = torch.eye(H, device="cuda")
    gs = col_scales(G)
    print(f"H={H}: col scales {gs[:4].tolist()} .. {gs[-4:].tolist()}; "
          f"scaled col max range {(G.abs().amax(0) * gs).min().item():.1f} .. {(G.abs().amax(0) * gs).max().item():.1f}")
    got = dw_x3(G, I, parts=1)          # [n, r] = G[r, n]
    err = (got - G.t()).abs() / G.t().abs().amax(1, keepdim=True)
    bad = (err > 1e-6).nonzero()
    print(f"  G via one-hot A: max rel {err.max().item():.2e}; {bad.shape[0]} elements > 1e-6; first (n, r) "
          f"{bad[:10].tolist()}")
    for n, r in bad[:6].tolist():
        x = G[r, n].item()
        print(f"    n={n} r={r}: G={x:.9e} got={got[n, r].item():.9e} G*s={x * gs[n].item():.6f} "
              f"rel {(got[n, r].item() - x) / abs(x):.2e}")
    got2 = dw_x3(I, A, parts=1)         # [n, k] = A[n, k]
    err2 = (got2 - A).abs()
    bad2 = (err2 > 1e-6).nonzero()
    print(f"  A via one-hot G: max abs {err2.max().item():.2e}; {bad2.shape[0]} elements > 1e-6; first "
          f"{bad2[:10].tolist()}")
    for n, k in bad2[:6].tolist():
        print(f"    n={n} k={k}: A={A[n, k].item():.9e} got={got2[n, k].item():.9e}")
