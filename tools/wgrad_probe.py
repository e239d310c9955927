"""Weight-gradient formulations at C2 (K = 320k rows): one GEMM dyᵀ·x (with whatever split-K
solution the library / TunableOp picks) against the split-K batched GEMM + ordered sum used by
kernels.weight_grad, for the QKV (N_out = 384) and out-projection (128) shapes, fp32.

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=... python tools/wgrad_probe.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tagan_amd  # noqa: E402,F401
from tagan_amd.kernels import weight_grad  # noqa: E402

dev = torch.device("cuda")
K, H = 320_000, 128
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(K, H, device=dev, generator=g)


def bench(name, f, flops, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print("%-44s %8.1f us  %6.1f TF/s" % (name, dt * 1e6, flops / dt / 1e12), flush=True)


for n_out in (384, 128):
    dy = torch.randn(K, n_out, device=dev, generator=g)
    F = 2 * K * H * n_out
    ref = weight_grad(dy, x).double()
    one = (dy.t() @ x).double()
    print("n_out %d: max |one - splitK| / max|ref| = %.2e" % (n_out, ((one - ref).abs().max() / ref.abs().max()).item()))
    bench("dW %d: one GEMM dy^T x" % n_out, lambda: dy.t() @ x, F)
    bench("dW %d: split-K bmm + sum (weight_grad)" % n_out, lambda: weight_grad(dy, x), F)
    for rows in (5000, 10000, 20000):
        bench("dW %d: split-K rows=%d" % (n_out, rows), lambda: weight_grad(dy, x, rows), F)
