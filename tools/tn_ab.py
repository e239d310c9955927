"""A/B of the two weight-gradient kernels (csrc/stream_gemm.hip): k_sgemm_tn2 (16-byte rows) against k_sgemm_tn
(rows of stride N + 2, same values), fp32 three-plane and the LN-recomputing form, H = 128 / 256.
Usage: python tools/tn_ab.py [--M 320000] [--H 128]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tagan_amd  # noqa: E402,F401
from tagan_amd import stream_gemm as sg  # noqa: E402


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for i in range(reps):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
    return ts[reps // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=320000)
    ap.add_argument("--H", type=int, default=128)
    a = ap.parse_args()
    M, H = a.M, a.H
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(M, H, device=dev)
    mean, rstd = x.mean(1), x.var(1, unbiased=False).add(1e-5).rsqrt()
    lg, lb = torch.randn(H, device=dev), torch.randn(H, device=dev)
    for N in (3 * H, H):
        wide = torch.randn(M, N + 2, device=dev)
        dy_old = wide[:, :N]
        dy = dy_old.contiguous()
        mb = M * (N + H) * 4 / 1e6
        for P in (3, 1):
            r = {"H": H, "N": N, "K": H, "planes": P, "MB": round(mb, 1)}
            r["tn2_us"] = round(timeit(lambda: sg.tn(dy, x, P)), 1)
            r["tn_us"] = round(timeit(lambda: sg.tn(dy_old, x, P)), 1)
            if N == 3 * H:
                r["tn2_ln_us"] = round(timeit(lambda: sg.tn_ln(dy, x, lg, lb, mean, rstd, P)), 1)
                r["tn_ln_us"] = round(timeit(lambda: sg.tn_ln(dy_old, x, lg, lb, mean, rstd, P)), 1)
            d2, b2 = sg.tn(dy, x, P)
            d1, b1 = sg.tn(dy_old, x, P)
            r["rel_diff"] = float((d2 - d1).norm() / d1.norm())
            r["db_rel_diff"] = float((b2 - b1).norm() / b1.norm())
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
