"""Time TemporalPropagation's intended compute (GRU evolution over T -> skip window -> output projection -> LN),
forward + backward, at a config's shape, with the recurrence as the csrc/gru.hip kernels and as per-step Python
(TAGAN_GRU_KERNEL=0 path), and the window aggregation kernel.

    python tools/tprop_probe.py [--config c2] [--reps 10] [--bidirectional 0]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tagan_amd  # noqa: E402,F401
from tagan_amd import synthetic  # noqa: E402
import tagan_amd.layers.temporal_propagation as tp  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--bidirectional", type=int, default=0)
    ap.add_argument("--only", default="", help="gru_kernel | python_steps: time one mode (profiling)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, _E, T, H = synthetic.CONFIGS[a.config][:4]
    torch.manual_seed(0)
    mod = tp.TemporalPropagation(H, H, dropout=0.1, bidirectional=bool(a.bidirectional)).to(dev).train()
    g = torch.Generator(device=dev).manual_seed(1)
    xt = torch.randn(T, N, H, device=dev, generator=g).requires_grad_()
    ts = (torch.rand(N, T, device=dev, generator=g).cumsum(1) * 3.0)
    dy = torch.randn(T, N, H, device=dev, generator=g)
    res = {"config": a.config, "rows": N, "T": T, "H": H, "bidirectional": bool(a.bidirectional)}
    for name, kern in (("gru_kernel", True), ("python_steps", False)):
        if a.only and name != a.only:
            continue
        tp.USE_GRU_KERNEL = kern
        for _ in range(2):
            mod.zero_grad(set_to_none=True)
            (mod.forward_intended(xt, ts) * dy).sum().backward()
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf = tb = 0.0
        for _ in range(a.reps):
            mod.zero_grad(set_to_none=True)
            xt.grad = None
            e[0].record()
            y = mod.forward_intended(xt, ts)
            e[1].record()
            (y * dy).sum().backward()
            e[2].record()
            e[2].synchronize()
            tf += e[0].elapsed_time(e[1])
            tb += e[1].elapsed_time(e[2])
        res[name] = {"ms_fwd": round(tf / a.reps, 3), "ms_bwd": round(tb / a.reps, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
