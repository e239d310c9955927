"""Weight-gradient kernel timing (csrc/stream_gemm.hip k_sgemm_tn) at the block shapes, fp32 three-plane and one-plane,
plain and LN-recomputing forms; run it under TAGAN_LIB=<variant library> to A/B a compile-time switch.
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
        dy = torch.randn(M, N, device=dev)
        for P in (3, 1):
            r = {"lib": os.path.basename(tagan_amd._lib.LIB_PATH), "H": H, "N": N, "K": H, "planes": P,
                 "MB": round(M * (N + H) * 4 / 1e6, 1), "tn_us": round(timeit(lambda: sg.tn(dy, x, P)), 1)}
            if N == 3 * H and sg.ln_supported(H, P, False, "in"):
                r["tn_ln_us"] = round(timeit(lambda: sg.tn_ln(dy, x, lg, lb, mean, rstd, P)), 1)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
