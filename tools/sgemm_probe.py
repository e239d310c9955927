"""Probe: the streaming projection GEMMs (csrc/stream_gemm.hip) against torch's GEMMs at the C2 block shapes.

Per shape: kernel time (HIP events, median of 20 after 5 warm-ups), the same product through torch (with the bench's
TunableOp table), and the error of both against fp64 (max-abs / max|ref| and normwise) on the same inputs.
Usage: python tools/sgemm_probe.py [--M 320000] [--H 128] [--planes 3,1] [--cases ...] ; TAGAN_LIB=<variant library> times another build.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tagan_amd  # noqa: E402,F401
from tagan_amd import stream_gemm as sg  # noqa: E402
from tagan_amd.gemm_tuning import use_tuned_gemms  # noqa: E402


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    ts = []
    for i in range(reps):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ts = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
    return ts[reps // 2] * 1e3   # us


def err(x, ref):
    x = x.double()
    d = x - ref
    return {"max_rel": float(d.abs().max() / ref.abs().max()), "norm_rel": float(d.norm() / ref.norm())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=320000)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--check-rows", type=int, default=40000)
    ap.add_argument("--no-tuned", action="store_true")
    ap.add_argument("--cases", default="", help="comma list of case names to run (default: all), e.g. qkv_fwd,dw_qkv")
    ap.add_argument("--planes", default="3,1", help="plane counts to run (3 = fp32, 1 = bf16)")
    args = ap.parse_args()
    only = set(c for c in args.cases.split(",") if c)
    if not args.no_tuned:
        use_tuned_gemms()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M, H = args.M, args.H
    R = min(M, args.check_rows)
    out = {"variant": os.path.basename(os.environ.get("TAGAN_LIB", "libtagan_hip.so")), "M": M, "H": H, "cases": []}

    def want(name):
        return not only or name.split(" ")[-1] in only

    def rec(name, bytes_, flops, t_k, t_t, e_k, e_t, extra=None):
        r = {"case": name, "us_kernel": round(t_k, 1), "us_torch": round(t_t, 1),
             "TBps_kernel": round(bytes_ / t_k / 1e6, 3), "TFps_kernel": round(flops / t_k / 1e6, 1),
             "err_kernel": e_k, "err_torch": e_t}
        if extra:
            r.update(extra)
        out["cases"].append(r)
        print(json.dumps(r), flush=True)

    x = torch.randn(M, H, device=dev)
    w_qkv = torch.randn(3 * H, H, device=dev) / H ** 0.5
    b_qkv = torch.randn(3 * H, device=dev) * 0.1
    w_o = torch.randn(H, H, device=dev) / H ** 0.5
    dq = torch.randn(M, 3 * H, device=dev)

    for planes in [int(p) for p in args.planes.split(",")]:
        tag = "fp32x3" if planes == 3 else "bf16x1"
        if want("qkv_fwd"):
            wp = sg.wprep(w_qkv, False, planes)
            c = sg.nt(x, wp, 3 * H, planes, b_qkv)
            ref = (x[:R].double() @ w_qkv.double().t() + b_qkv.double())
            ct = torch.nn.functional.linear(x, w_qkv, b_qkv)
            rec(tag + " qkv_fwd", 4 * M * 4 * H, 2 * M * H * 3 * H,
                timeit(lambda: sg.nt(x, wp, 3 * H, planes, b_qkv, out=c)),
                timeit(lambda: torch.nn.functional.linear(x, w_qkv, b_qkv)), err(c[:R], ref), err(ct[:R], ref))
        if want("qkv_fwd_ln"):   # LN1 in the prologue (the step's form)
            lw, lb = torch.ones(H, device=dev), torch.zeros(H, device=dev)
            wp = sg.wprep(w_qkv, False, planes)
            c, _, _ = sg.nt_ln_in(x, lw, lb, 1e-5, wp, 3 * H, planes, bias=b_qkv)
            h = torch.nn.functional.layer_norm(x[:R].double(), (H,), lw.double(), lb.double(), 1e-5)
            ref = h @ w_qkv.double().t() + b_qkv.double()
            rec(tag + " qkv_fwd_ln", 4 * M * 4 * H, 2 * M * H * 3 * H,
                timeit(lambda: sg.nt_ln_in(x, lw, lb, 1e-5, wp, 3 * H, planes, bias=b_qkv)), 0.0, err(c[:R], ref), {})
        if want("out_fwd"):
            wpo = sg.wprep(w_o, False, planes)
            c = sg.nt(x, wpo, H, planes)
            ref = x[:R].double() @ w_o.double().t()
            ct = x @ w_o.t()
            rec(tag + " out_fwd", 2 * M * H * 4, 2 * M * H * H, timeit(lambda: sg.nt(x, wpo, H, planes, out=c)),
                timeit(lambda: x @ w_o.t()), err(c[:R], ref), err(ct[:R], ref))
        if want("dc"):
            wpd = sg.wprep(w_o, True, planes)
            c = sg.nt(x, wpd, H, planes)
            ref = x[:R].double() @ w_o.double()
            ct = x @ w_o
            rec(tag + " dc", 2 * M * H * 4, 2 * M * H * H, timeit(lambda: sg.nt(x, wpd, H, planes, out=c)),
                timeit(lambda: x @ w_o), err(c[:R], ref), err(ct[:R], ref))
        if want("dh"):
            wph = sg.wprep(w_qkv, True, planes)
            c = sg.nt(dq, wph, H, planes)
            ref = dq[:R].double() @ w_qkv.double()
            ct = dq @ w_qkv
            rec(tag + " dh", 4 * M * 4 * H, 2 * M * H * 3 * H, timeit(lambda: sg.nt(dq, wph, H, planes, out=c)),
                timeit(lambda: dq @ w_qkv), err(c[:R], ref), err(ct[:R], ref))
        if want("dw_qkv"):
            dw, db = sg.tn(dq, x, planes)
            ref = dq.double().t() @ x.double()
            refb = dq.double().sum(0)
            dwt = dq.t() @ x
            rec(tag + " dw_qkv", 4 * M * 4 * H, 2 * M * H * 3 * H, timeit(lambda: sg.tn(dq, x, planes)),
                timeit(lambda: dq.t() @ x), err(dw, ref), err(dwt, ref), {"err_db": err(db, refb)})
        if want("dw_o"):
            do = dq[:, :H]
            dw, db = sg.tn(do, x, planes)
            ref = do.double().t() @ x.double()
            dwt = do.t() @ x
            rec(tag + " dw_o", 2 * M * H * 4, 2 * M * H * H, timeit(lambda: sg.tn(do, x, planes)),
                timeit(lambda: do.t() @ x), err(dw, ref), err(dwt, ref))
        if want("ln2_bwd_out") and sg.ln2_bwd_out_supported(H, planes, False):
            # LN2 backward + dC + dW_o + db_o (5 row passes: dy, s, c in; dres, dc out)
            s2 = dq[:, H:2 * H].contiguous()
            dy = dq[:, 2 * H:].contiguous()
            st = torch.ones(2, M, device=dev)
            lw = torch.ones(H, device=dev)
            wpd = sg.wprep(w_o, True, planes)
            rec(tag + " ln2_bwd_out", 5 * M * H * 4, 4 * M * H * H,
                timeit(lambda: sg.ln2_bwd_out(dy, s2, st[0], st[1], lw, 0.1, 7, x, wpd, planes)), 0.0, {}, {})
    if not only or "bf16io" in only:
        xb, dqb = x.bfloat16(), dq.bfloat16()
        wp = sg.wprep(w_qkv, False, 1)
        c = sg.nt(xb, wp, 3 * H, 1, b_qkv, out_dtype=torch.bfloat16)
        ref = xb[:R].double() @ w_qkv.bfloat16().double().t() + b_qkv.double()
        ct = torch.addmm(b_qkv.bfloat16(), xb, w_qkv.bfloat16().t())
        rec("bf16io qkv_fwd", 2 * M * 4 * H, 2 * M * H * 3 * H,
            timeit(lambda: sg.nt(xb, wp, 3 * H, 1, b_qkv, out=c)),
            timeit(lambda: torch.addmm(b_qkv.bfloat16(), xb, w_qkv.bfloat16().t())), err(c[:R].float(), ref),
            err(ct[:R].float(), ref))
        dw, db = sg.tn(dqb, xb, 1)
        ref = dqb.double().t() @ xb.double()
        rec("bf16io dw_qkv", 2 * M * 4 * H, 2 * M * H * 3 * H, timeit(lambda: sg.tn(dqb, xb, 1)),
            timeit(lambda: torch.mm(dqb.t(), xb, out_dtype=torch.float32)), err(dw, ref),
            err(torch.mm(dqb.t(), xb, out_dtype=torch.float32), ref))
    path = os.environ.get("SGEMM_PROBE_OUT")
    if path:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
