"""Probe: the layer GEMMs with bf16 operands and fp32 accumulate/output (torch.mm(..., out_dtype)) vs fp32."""
import time

import torch

dev = torch.device("cuda")
M, H = 320_000, 128
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(M, H, device=dev, generator=g)
w = torch.randn(3 * H, H, device=dev, generator=g)
dqkv = torch.randn(M, 3 * H, device=dev, generator=g)


def bench(name, f, flops, reps=20):
    for _ in range(3):
        r = f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        r = f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    print("%-40s %8.1f us  %6.1f TF/s  %s" % (name, dt * 1e6, flops / dt / 1e12, tuple(r.shape)), flush=True)
    return r


F = 2 * M * H * 3 * H
ref = bench("fp32 h @ w.T", lambda: h @ w.t(), F)
hb, wb = h.bfloat16(), w.bfloat16()
bench("cast h -> bf16", lambda: h.bfloat16(), 0.0 + 1)
try:
    r = bench("bf16 mm(out_dtype=fp32)", lambda: torch.mm(hb, wb.t(), out_dtype=torch.float32), F)
    print("  rel err vs fp32: %.2e" % float((r - ref).abs().max() / ref.abs().max()))
except Exception as e:
    print("mm out_dtype failed:", e)
r = bench("bf16 mm -> bf16", lambda: hb @ wb.t(), F)
dqb = dqkv.bfloat16()
bench("fp32 dh = dqkv @ w", lambda: dqkv @ w, F)
try:
    bench("bf16 dh out fp32", lambda: torch.mm(dqb, wb, out_dtype=torch.float32), F)
except Exception as e:
    print("failed:", e)
rows = 2048
c = M // rows
bench("fp32 dW split-K", lambda: torch.bmm(dqkv.view(c, rows, 3 * H).transpose(1, 2), h.view(c, rows, H)).sum(0), F)
try:
    bench("bf16 dW split-K out fp32", lambda: torch.bmm(dqb.view(c, rows, 3 * H).transpose(1, 2), hb.view(c, rows, H),
                                                       out_dtype=torch.float32).sum(0), F)
except Exception as e:
    print("bmm out_dtype failed:", e)
bench("bf16 dW mm out fp32", lambda: torch.mm(dqb.t(), hb, out_dtype=torch.float32), F)
