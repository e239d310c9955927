"""The six GEMMs of one attention layer at C2 (M = 320k rows, H = 128), each timed alone in the
formulation the fused block uses and in alternatives, to find the inefficient ones.

    python tools/gemm_layer.py
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

dev = torch.device("cuda")
M, H = 320_000, 128
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(M, H, device=dev, generator=g)
w_qkv = torch.randn(3 * H, H, device=dev, generator=g)
b_qkv = torch.randn(3 * H, device=dev, generator=g)
w_o = torch.randn(H, H, device=dev, generator=g)
b_o = torch.randn(H, device=dev, generator=g)
ctx = torch.randn(M, H, device=dev, generator=g)
dqkv = torch.randn(M, 3 * H, device=dev, generator=g)
do = torch.randn(M, H, device=dev, generator=g)


def bench(name, f, flops, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print("%-34s %8.1f us  %6.1f TF/s" % (name, dt * 1e6, flops / dt / 1e12), flush=True)


def split_k(dy2, x2, rows):
    K, Mo = dy2.shape
    N = x2.shape[1]
    c = K // rows
    main = c * rows
    dw = torch.bmm(dy2[:main].view(c, rows, Mo).transpose(1, 2), x2[:main].view(c, rows, N)).sum(0)
    if main < K:
        dw = dw + dy2[main:].t() @ x2[main:]
    return dw


F_qkv = 2 * M * H * 3 * H
F_o = 2 * M * H * H
bench("fwd qkv addmm(b, h, Wt)", lambda: torch.addmm(b_qkv, h, w_qkv.t()), F_qkv)
bench("fwd qkv mm(h, Wt)", lambda: h @ w_qkv.t(), F_qkv)
bench("fwd qkv linear", lambda: torch.nn.functional.linear(h, w_qkv, b_qkv), F_qkv)
bench("fwd out addmm(b, ctx, Wot)", lambda: torch.addmm(b_o, ctx, w_o.t()), F_o)
bench("fwd out mm", lambda: ctx @ w_o.t(), F_o)
bench("bwd dctx = do @ Wo", lambda: do @ w_o, F_o)
bench("bwd dctx = (Wo^T do^T)^T", lambda: (w_o.t() @ do.t()).t(), F_o)
bench("bwd dh = dqkv @ Wqkv", lambda: dqkv @ w_qkv, F_qkv)
bench("bwd dh = (Wqkv^T dqkv^T)^T", lambda: (w_qkv.t() @ dqkv.t()).t(), F_qkv)
for rows in (1024, 2048, 4096, 8192):
    bench("bwd dWqkv split-K %d" % rows, lambda rows=rows: split_k(dqkv, h, rows), F_qkv)
    bench("bwd dWo split-K %d" % rows, lambda rows=rows: split_k(do, ctx, rows), F_o)
bench("bwd dWqkv mm(dqkv^T, h)", lambda: dqkv.t() @ h, F_qkv)
bench("bwd dWqkv mm(h^T, dqkv)^T", lambda: (h.t() @ dqkv).t(), F_qkv)
bench("bwd db_qkv sum(0)", lambda: dqkv.sum(0), M * 3 * H)
