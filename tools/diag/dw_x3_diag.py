"""Diagnostic: qs_attn_dw_x3's error pattern (per part count, per output row / column block) against fp64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "quad-swarm-rl-stable-baselines3_amd"))
import torch  # noqa: E402
from quadswarm_amd.encoder_train import dw_x3  # noqa: E402


def report(tag, got, want):
    sc = want.abs().amax(1, keepdim=True).clamp_min(1e-300)
    e = (got.double() - want).abs() / sc
    H = want.shape[0]
    rows = e.amax(1)
    cols = e.amax(0)
    print(f"{tag}: max {e.max().item():.2e} median {e.median().item():.2e}; worst row {int(rows.argmax())} "
          f"col {int(cols.argmax())}; by 32-row block {[f'{x:.1e}' for x in rows.view(-1, 32).amax(1).tolist()]}; "
          f"by 32-col block {[f'{x:.1e}' for x in cols.view(-1, 32).amax(1).tolist()]}")
    big = (e > 1e-6).nonzero()
    print(f"   elements > 1e-6: {big.shape[0]} of {H * H}; first {big[:8].tolist()}")


for H, R in ((128, 777), (256, 16), (256, 4000)):
    g = torch.Generator(device="cuda").manual_seed(R)
    G = torch.randn(R, H, device="cuda", generator=g) * torch.exp2(torch.linspace(-20, 4, H, device="cuda"))
    A = torch.tanh(torch.randn(R, H, device="cuda", generator=g) * 2)
    want = G.double().t().mm(A.double())
    for parts in (1, 2, 256):
        report(f"H={H} R={R} parts={parts}", dw_x3(G, A, parts=parts), want)
    Gi = torch.randint(-3, 4, (R, H), device="cuda", generator=g).float()
    Ai = torch.randint(-1, 2, (R, H), device="cuda", generator=g).float()
    wi = Gi.double().t().mm(Ai.double())
    for parts in (1, 256):
        got = dw_x3(Gi, Ai, parts=parts)
        print(f"   integers H={H} R={R} parts={parts}: max abs err {(got.double() - wi).abs().max().item():.3e}")
