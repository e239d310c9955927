"""LayerNorm kernels at C2's shape (M = 320k rows, H = 128), each variant the model launches:
HIP-event time per launch and algorithmic GB/s.  The row-groups-per-wave factor is read once
per process from TAGAN_LN_ROWS (1|2|4), so A/B it across processes:

    for u in 1 2 4; do TAGAN_LN_ROWS=$u python tools/ln_probe.py; done
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tagan_amd  # noqa: E402,F401
from tagan_amd.fused import ln_bwd, ln_fwd  # noqa: E402

dev = torch.device("cuda")
M, H = 320_000, 128
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(M, H, device=dev, generator=g)
b = torch.randn(M, H, device=dev, generator=g)
ab = torch.randn(H, device=dev, generator=g)
gamma = torch.randn(H, device=dev, generator=g)
beta = torch.randn(H, device=dev, generator=g)
dy = torch.randn(M, H, device=dev, generator=g)
dres = torch.randn(M, H, device=dev, generator=g)
ROW = M * H * 4


def bench(name, f, nbytes, reps=50):
    for _ in range(3):
        f()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(reps):
        f()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print("U=%s %-40s %8.1f us  %7.1f GB/s" % (os.environ.get("TAGAN_LN_ROWS", "default"), name, us,
                                              nbytes / us / 1e3), flush=True)


y, s, mean, rstd = ln_fwd(a, b, 0.1, 7, gamma, beta, 1e-5, True, a_bias=ab)
bench("fwd LN(drop(a+bias)+b), keeps s", lambda: ln_fwd(a, b, 0.1, 7, gamma, beta, 1e-5, True, a_bias=ab),
      4 * ROW + 8 * M)
bench("fwd LN(a)", lambda: ln_fwd(a, None, 0.0, 0, gamma, beta, 1e-5, False), 2 * ROW + 8 * M)
bench("bwd ds(+dres), da, dsum_a", lambda: ln_bwd(s, mean, rstd, gamma, dy, dres, 0.1, 7, True, True, True),
      5 * ROW + 8 * M)
bench("bwd da only", lambda: ln_bwd(s, mean, rstd, gamma, dy, None, 0.0, 0, False, True, False), 3 * ROW + 8 * M)
