"""Time the fused projection kernels (csrc/proj_gemm.hip) at a C2-sized block (M = 320,000 rows, H = 128)
against the unfused hipBLASLt + LayerNorm-kernel chain they replace.  HIP events on the launch stream.

    python tools/proj_probe.py [--M 320000] [--reps 20] [--only ln_qkv,proj_ln,mm_k,ln_bwd]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=320_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import tagan_amd  # noqa: F401
    import tagan_amd.fused as fu
    dev = torch.device("cuda:0")
    M, H = a.M, 128
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g, device=dev)  # noqa: E731
    x, c, dy, dres = r(M, H), r(M, H), r(M, H), r(M, H)
    dqkv = r(M, 3 * H)
    wq, bq, wo, bo = r(3 * H, H) * 0.08, r(3 * H), r(H, H) * 0.08, r(H)
    lw, lb = 1 + 0.1 * r(H), 0.1 * r(H)
    mean, rstd = x.mean(-1), 1 / torch.sqrt(x.var(-1, unbiased=False) + 1e-5)
    only = set(a.only.split(",")) if a.only else None
    res = {}

    def run(name, fn, flop, bytes_):
        if only and name.split(":")[0] not in only:
            return
        us = timeit(fn, a.reps)
        res[name] = {"us": round(us, 1), "TFs": round(flop / us / 1e6, 1), "TBs": round(bytes_ / us / 1e6, 2)}
        print("%-28s %8.1f us  %6.1f TF/s  %5.2f TB/s" % (name, us, flop / us / 1e6, bytes_ / us / 1e6), flush=True)

    f = 4
    run("ln_qkv", lambda: fu.proj_ln_qkv(x, lw, lb, 1e-5, wq, bq, False), 2 * M * H * 3 * H, f * M * (H + 3 * H))
    run("ln_qkv:h_aug", lambda: fu.proj_ln_qkv(x, lw, lb, 1e-5, wq, bq, True), 2 * M * H * 3 * H,
        f * M * (H + 3 * H + H + 4))
    run("proj_ln", lambda: fu.proj_ln_out(c, wo, bo, x, 0.1, 7, lw, lb, 1e-5), 2 * M * H * H, f * M * 4 * H)
    run("mm_k", lambda: fu.proj_mm(dy, wo, True), 2 * M * H * H, f * M * 2 * H)
    run("mm_k:384", lambda: fu.proj_mm(dqkv, wq, True), 2 * M * 3 * H * H, f * M * 4 * H)
    run("ln_bwd", lambda: fu.proj_ln_bwd(dqkv, wq, x, mean, rstd, lw, dres), 2 * M * 3 * H * H, f * M * (3 * H + 3 * H))
    # the unfused chain they replace (hipBLASLt + csrc/layernorm.hip)
    run("ref:ln_fwd", lambda: fu.ln_fwd(x, None, 0.0, 0, lw, lb, 1e-5, False), 0, f * M * 2 * H)
    run("ref:qkv_gemm", lambda: torch.nn.functional.linear(x, wq, bq), 2 * M * H * 3 * H, f * M * 4 * H)
    run("ref:out_gemm", lambda: c @ wo.t(), 2 * M * H * H, f * M * 2 * H)
    run("ref:dc_gemm", lambda: dy @ wo, 2 * M * H * H, f * M * 2 * H)
    run("ref:dh_gemm", lambda: dqkv @ wq, 2 * M * 3 * H * H, f * M * 4 * H)
    run("ref:ln_bwd", lambda: fu.ln_bwd(x, mean, rstd, lw, dy, dres, 0.0, 0, True, False, False), 0, f * M * 4 * H)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
