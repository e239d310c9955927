"""LayerNorm kernels at C2's shape (M = 320k rows, H = 128; LN_PROBE_M / LN_PROBE_H override), each variant the model launches:
HIP-event time per launch and algorithmic GB/s.  Compile-time variants (the row groups per wave, TAGAN_LN_ROWS) are
A/B'd as variant libraries:

    make -C temporal-asymmetric-graph-attention-network_amd/csrc variant NAME=lnu2 EXTRA=-DTAGAN_LN_ROWS=2
    TAGAN_LIB=$PWD/temporal-asymmetric-graph-attention-network_amd/libtagan_hip_lnu2.so python tools/ln_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tagan_amd  # noqa: E402,F401
from tagan_amd.fused import ln_bwd, ln_fwd  # noqa: E402

dev = torch.device("cuda")
M = int(os.environ.get("LN_PROBE_M", 320_000))
H = int(os.environ.get("LN_PROBE_H", 128))
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
    print("%s M=%d H=%d %-40s %8.1f us  %7.1f GB/s" % (os.path.basename(os.environ.get("TAGAN_LIB", "default")), M, H, name, us,
                                              nbytes / us / 1e3), flush=True)


y, s, mean, rstd = ln_fwd(a, b, 0.1, 7, gamma, beta, 1e-5, True, a_bias=ab)
bench("fwd LN(drop(a+bias)+b), keeps s", lambda: ln_fwd(a, b, 0.1, 7, gamma, beta, 1e-5, True, a_bias=ab),
      4 * ROW + 8 * M)
bench("fwd LN(a)", lambda: ln_fwd(a, None, 0.0, 0, gamma, beta, 1e-5, False), 2 * ROW + 8 * M)
bench("bwd ds(+dres), da, dsum_a", lambda: ln_bwd(s, mean, rstd, gamma, dy, dres, 0.1, 7, True, True, True),
      5 * ROW + 8 * M)
bench("bwd da only", lambda: ln_bwd(s, mean, rstd, gamma, dy, None, 0.0, 0, False, True, False), 3 * ROW + 8 * M)
