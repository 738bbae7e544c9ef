"""Diagnostic (GPU box): is a split-f16 (x3) GEMM through rocBLAS (f16 inputs, fp32 accumulate and output) faster
than torch's fp32 GEMM at the PPO update's neighbour-encoder shape, and how accurate is it?

    python tools/x3_gemm_probe.py [M]

Y = X W^T with X [M, 256] (tanh-range activations), W [256, 256]; x3 = Xh Wh^T + Xl Wh^T + Xh Wl^T on
hi = f16(s x), lo = f16(s x - hi) (s = 256), the three products accumulated in fp32 by rocblas_gemm_ex (beta = 1).
Reports ms per GEMM (fp32 torch, x3 incl. / excl. the splits) and the max error of each against an fp64 product.
"""
import ctypes
import sys
import time

import torch

RB = ctypes.CDLL("librocblas.so")
F16, F32, OP_N, OP_T = 150, 151, 111, 112


class X3:
    def __init__(self, stream):
        self.h = ctypes.c_void_p()
        assert RB.rocblas_create_handle(ctypes.byref(self.h)) == 0
        assert RB.rocblas_set_stream(self.h, ctypes.c_void_p(stream)) == 0

    def gemm(self, a, b, c, m, n, k, transa, transb, lda, ldb, ldc, alpha, beta):
        al, be = ctypes.c_float(alpha), ctypes.c_float(beta)
        rc = RB.rocblas_gemm_ex(self.h, transa, transb, m, n, k, ctypes.byref(al), ctypes.c_void_p(a.data_ptr()), F16,
                                lda, ctypes.c_void_p(b.data_ptr()), F16, ldb, ctypes.byref(be),
                                ctypes.c_void_p(c.data_ptr()), F32, ldc, ctypes.c_void_p(c.data_ptr()), F32, ldc, F32,
                                0, 0, 0)
        assert rc == 0, rc


def split(x, s):
    y = x * s
    h = y.half()
    return h, (y - h.float()).half()


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1572864
    K = N = 256
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    X = torch.tanh(torch.randn(M, K, device=dev))
    W = torch.randn(N, K, device=dev) / 16
    st = torch.cuda.current_stream().cuda_stream
    x3 = X3(st)
    Y = torch.empty(M, N, device=dev)
    s, sw = 256.0, 256.0

    def fp32():
        return X @ W.t()

    Wh, Wl = split(W, sw)

    def prod(Xh, Xl):
        # column-major view: Y^T (N x M) = W (N x K) . X^T (K x M)
        x3.gemm(Wh, Xh, Y, N, M, K, OP_T, OP_N, K, K, N, 1.0 / (s * sw), 0.0)
        x3.gemm(Wh, Xl, Y, N, M, K, OP_T, OP_N, K, K, N, 1.0 / (s * sw), 1.0)
        x3.gemm(Wl, Xh, Y, N, M, K, OP_T, OP_N, K, K, N, 1.0 / (s * sw), 1.0)
        return Y

    def x3_full():
        Xh, Xl = split(X, s)
        return prod(Xh, Xl)

    Xh, Xl = split(X, s)

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / reps * 1e3

    t32 = timeit(fp32)
    tx = timeit(x3_full)
    tp = timeit(lambda: prod(Xh, Xl))
    rows = slice(0, 65536)
    ref = X[rows].double() @ W.double().t()
    e32 = (fp32()[rows].double() - ref).abs().max().item()
    ex3 = (x3_full()[rows].double() - ref).abs().max().item()
    flop = 2.0 * M * N * K
    print(f"M={M}: fp32 {t32:.3f} ms ({flop / t32 / 1e9:.1f} TF/s) | x3 {tx:.3f} ms incl. split, {tp:.3f} ms GEMMs only "
          f"({3 * flop / tp / 1e9:.1f} TF/s f16) | max err fp32 {e32:.2e} x3 {ex3:.2e} (|Y| max {ref.abs().max().item():.2f})")


if __name__ == "__main__":
    main()
