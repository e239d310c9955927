"""Probe: the fp32 QKV projection (C2 geometric layer, M = 320,000, K = H + 4 = 132, N = 3H = 384) as one bf16 MFMA
GEMM over split operands -- A = [a_hi | a_lo | a_hi], B = [w_hi | w_hi | w_lo] (x_hi = bf16(x), x_lo = bf16(x - x_hi)),
K' = 3K, fp32 accumulate and fp32 output -- against the fp32 GEMM: time (HIP events) and error vs an fp64 product.

    python tools/split_bf16_probe.py
"""
import torch

dev = torch.device("cuda")
M, K, N = 320_000, 132, 384
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(M, K, device=dev, generator=g)
w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5


def split(x):
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return hi, lo


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


ah, al = split(a)
wh, wl = split(w)
A3 = torch.cat([ah, al, ah], 1).contiguous()
B3 = torch.cat([wh, wh, wl], 1).contiguous()
ref = (a.double() @ w.double().t())
f32 = a @ w.t()
s3 = torch.mm(A3, B3.t(), out_dtype=torch.float32)
b1 = torch.mm(ah, wh.t(), out_dtype=torch.float32)
scale = ref.abs().max().item()
for name, out in (("fp32", f32), ("split-bf16 x3", s3), ("bf16 x1", b1)):
    err = (out.double() - ref).abs()
    print("%-14s max abs err %.3e  max rel-to-max %.3e  mean abs %.3e" % (name, err.max().item(),
                                                                     err.max().item() / scale, err.mean().item()))
t32 = timeit(lambda: a @ w.t())
t3 = timeit(lambda: torch.mm(A3, B3.t(), out_dtype=torch.float32))
tsplit = timeit(lambda: torch.cat([*split(a)[:1], split(a)[1], split(a)[0]], 1))
flops = 2.0 * M * K * N
print("fp32 GEMM        %7.1f us  %6.1f TF/s" % (t32, flops / t32 / 1e6))
print("split GEMM (3K)  %7.1f us  %6.1f TF/s (fp32-equivalent)" % (t3, flops / t3 / 1e6))
print("split pass (torch, unfused)  %7.1f us" % tsplit)
