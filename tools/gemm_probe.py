"""Micro-probe: weight-gradient GEMM dW = dYᵀ X (K = 320k rows) via different torch formulations."""
import time
import torch

dev = torch.device("cuda")
K = 320_000
for (M, N) in [(384, 128), (128, 128), (128, 27)]:
    dy = torch.randn(K, M, device=dev)
    x = torch.randn(K, N, device=dev)
    ref = (dy.double().t() @ x.double()).float()

    def mm():
        return dy.t() @ x

    def bmm(c):
        def f():
            return torch.bmm(dy.view(c, K // c, M).transpose(1, 2), x.view(c, K // c, N)).sum(0)
        return f

    def mmT():
        return (x.t() @ dy).t()

    cands = {"mm": mm, "mmT": mmT}
    for c in (10, 40, 160, 640):
        cands["bmm%d" % c] = bmm(c)
    for name, f in cands.items():
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            r = f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        err = float((r - ref).abs().max() / ref.abs().max())
        print("M=%d N=%d %-8s %8.1f us  %6.1f TF  relerr %.1e" % (M, N, name, dt * 1e6, 2 * K * M * N / dt / 1e12, err))
# layer norm
x = torch.randn(K, 128, device=dev, requires_grad=True)
ln = torch.nn.LayerNorm(128).to(dev)
for _ in range(3):
    y = ln(x)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    y = ln(x)
torch.cuda.synchronize()
print("LN fwd %.1f us" % ((time.perf_counter() - t0) / 20 * 1e6))
