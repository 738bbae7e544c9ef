"""Time the x3 linear kernels (qs_linear_tanh_x3 / _cat / _bias / _rows) at the C3 rollout's and update's shapes with
HIP events on the launch stream; the library is whatever quadswarm_amd._native loads (QUADSWARM_LIB selects an A/B
build).  Prints one line per shape: average us per launch, achieved HBM GB/s and f16 TFLOP/s (3 products).
  python tools/linear_probe.py [--reps 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "quad-swarm-rl-stable-baselines3_amd"))
from quadswarm_amd.encoder_train import _pow2_scales  # noqa: E402
from quadswarm_amd.policy_fused import (linear_bias_x3, linear_rows_x3, linear_tanh_cat_x3, linear_tanh_x3,  # noqa: E402
                                        pack_linear_x3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"library: {os.environ.get('QUADSWARM_LIB', 'in-tree')}")
    for M in (32768, 262144):
        for K, N, kind in ((256, 256, "tanh"), (512, 512, "tanh"), (512, 512, "cat"), (256, 256, "bias"),
                           (256, 256, "rows"), (512, 256, "rows")):
            x = torch.tanh(torch.randn(M, K, device=dev, generator=g))
            w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
            b = torch.randn(N, device=dev, generator=g) * 0.1
            pw = pack_linear_x3(w)
            y = torch.empty(M, N, device=dev)
            rs = _pow2_scales(x.abs().amax(1))
            x0, x1 = x[:, :256].contiguous(), x[:, 256:].contiguous()
            if kind == "tanh":
                f = lambda: linear_tanh_x3(x, pw, b, out=y)  # noqa: E731
            elif kind == "cat":
                f = lambda: linear_tanh_cat_x3(x0, x1, pw, b, out=y)  # noqa: E731
            elif kind == "bias":
                f = lambda: linear_bias_x3(x, pw, b, out=y)  # noqa: E731
            else:
                f = lambda: linear_rows_x3(x, rs, pw, N, out=y)  # noqa: E731
            for _ in range(3):
                f()
            st = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(a.reps):
                f()
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            byts = 4.0 * M * (K + N)
            flop = 2.0 * M * K * N * 3
            print(f"M {M:7d} K {K} N {N} {kind:4s}: {us:8.1f} us  {byts / us / 1e3:7.0f} GB/s  {flop / us / 1e6:6.1f} TF/s",
                  flush=True)


if __name__ == "__main__":
    main()
