#!/usr/bin/env python
"""Timing probe for the update's [B, 256] x [256, 256] torch GEMMs (P = e_mean A_m^T + b_a1, dL/de_mean = dP A_m) under
the BLAS back ends torch offers on ROCm.  Diagnostic.

    python tools/gemm_probe.py [--B 262144]
"""
import argparse

import torch


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=262144)
    a = ap.parse_args()
    H = 256
    torch.manual_seed(0)
    x = torch.randn(a.B, H, device="cuda")
    w2 = torch.randn(H, 2 * H, device="cuda")
    am = w2[:, H:]
    amc = am.contiguous()
    b = torch.randn(H, device="cuda")
    out = torch.empty(a.B, H, device="cuda")
    for lib in ("default", "cublaslt", "cublas"):
        if lib != "default":
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as e:  # noqa: BLE001
                print(lib, "unavailable:", e)
                continue
        res = {
            "addmm strided A_m^T": timeit(lambda: torch.addmm(b, x, am.t(), out=out)),
            "addmm contiguous A_m^T": timeit(lambda: torch.addmm(b, x, amc.t(), out=out)),
            "F.linear contiguous": timeit(lambda: torch.nn.functional.linear(x, amc, b)),
            "mm contiguous A_m^T": timeit(lambda: torch.mm(x, amc.t(), out=out)),
            "mm (A_m^T)^T-contiguous": timeit(lambda: torch.mm(x, amc.t().contiguous(), out=out)),
            "mm strided A_m (dem)": timeit(lambda: torch.mm(x, am, out=out)),
            "mm contiguous A_m (dem)": timeit(lambda: torch.mm(x, amc, out=out)),
        }
        flop = 2 * a.B * H * H
        print(f"== {lib}")
        for k, us in res.items():
            print(f"  {k:28s} {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s")


if __name__ == "__main__":
    main()
