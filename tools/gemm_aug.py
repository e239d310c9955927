"""Projection-GEMM formulations at C2 (M = 320k rows, H = 128), fp32:

* QKV forward with the bias in the hipBLASLt epilogue (F.linear) against a bias-free GEMM over
  an augmented operand [h | 1 | 0 0 0] (K = H + 4) and a weight with the bias as an extra column;
* the out-projection with and without bias epilogue;
* the split-K weight gradient over the augmented operand, whose extra column is the bias gradient.

    python tools/gemm_aug.py          (PYTORCH_TUNABLEOP_ENABLED=1 ... to time tuned solutions)
"""
import time

import torch

dev = torch.device("cuda")
M, H = 320_000, 128
HA = H + 4
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(M, H, device=dev, generator=g)
h_aug = torch.zeros(M, HA, device=dev)
h_aug[:, :H] = h
h_aug[:, H] = 1.0
w_qkv = torch.randn(3 * H, H, device=dev, generator=g)
b_qkv = torch.randn(3 * H, device=dev, generator=g)
w_aug = torch.zeros(3 * H, HA, device=dev)
w_aug[:, :H] = w_qkv
w_aug[:, H] = b_qkv
w_o = torch.randn(H, H, device=dev, generator=g)
b_o = torch.randn(H, device=dev, generator=g)
ctx = torch.randn(M, H, device=dev, generator=g)
dqkv = torch.randn(M, 3 * H, device=dev, generator=g)


def bench(name, f, flops, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print("%-40s %8.1f us  %6.1f TF/s" % (name, dt * 1e6, flops / dt / 1e12), flush=True)


def split_k(dy2, x2, rows=2000):
    K, Mo = dy2.shape
    N = x2.shape[1]
    c = K // rows
    xs = x2.as_strided((c, rows, N), (rows * x2.stride(0), x2.stride(0), 1))
    return torch.bmm(dy2.view(c, rows, Mo).transpose(1, 2), xs).sum(0)


F_qkv = 2 * M * H * 3 * H
F_o = 2 * M * H * H
ref = torch.nn.functional.linear(h, w_qkv, b_qkv)
aug = h_aug @ w_aug.t()
print("max |aug - linear| = %.3g" % (aug - ref).abs().max().item())
bench("qkv F.linear (bias epilogue)", lambda: torch.nn.functional.linear(h, w_qkv, b_qkv), F_qkv)
bench("qkv mm no bias", lambda: h @ w_qkv.t(), F_qkv)
bench("qkv aug K=132 mm(h_aug, W_aug^T)", lambda: h_aug @ w_aug.t(), F_qkv)
wa_t = w_aug.t().contiguous()
bench("qkv aug K=132 NN", lambda: h_aug @ wa_t, F_qkv)
bench("out F.linear (bias epilogue)", lambda: torch.nn.functional.linear(ctx, w_o, b_o), F_o)
bench("out mm no bias", lambda: ctx @ w_o.t(), F_o)
bench("dW qkv split-K (h, N=128)", lambda: split_k(dqkv, h), F_qkv)
bench("dW qkv split-K (h_aug[:, :132])", lambda: split_k(dqkv, h_aug), F_qkv)
bench("dW qkv split-K (h_aug[:, :128] view)", lambda: split_k(dqkv, h_aug[:, :H]), F_qkv)
bench("db colsum (torch sum)", lambda: dqkv.sum(0), 0)
