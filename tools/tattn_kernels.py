"""Time the temporal attention kernels (fwd, bwd) alone at a config's shape.

    python tools/tattn_kernels.py [--config c2] [--p 0.1] [--reps 20]

Layout as in the model: Q|K|V of the time-major [T, N, 3H] projection (row stride 3H,
step stride N*3H), the folded [heads, 2T-1] bias table, bias-table gradient on.
Algorithmic bytes: fwd reads Q,K,V and writes O (+ LSE); bwd reads Q,K,V,O,dO (+ LSE)
and writes dQ,dK,dV (the matrix-core v4/v5 paths do not read O).  FLOPs: 2 (fwd) and 5 (bwd) T x T x d
products per (row, head).  TAGAN_LIB=<path> selects an alternative build.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tagan_amd  # noqa: E402,F401
from tagan_amd import _lib, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--causal", type=int, default=0)
    ap.add_argument("--keep", type=int, default=1, help="dropout keep-bit cache between fwd and bwd (as the model)")
    ap.add_argument("--bf16", action="store_true", help="bf16 storage of q, k, v, out, dout, dq, dk, dv (the bf16 step)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N, _E, T, H, heads = synthetic.CONFIGS[a.config][:5]
    d = H // heads
    g = torch.Generator(device=dev).manual_seed(3)
    dt = torch.bfloat16 if a.bf16 else torch.float32
    qkv = torch.randn(T, N, 3 * H, device=dev, generator=g).to(dt)
    out = torch.empty(T, N, H, device=dev, dtype=dt)
    dout = torch.randn(T, N, H, device=dev, generator=g).to(dt)
    dqkv = torch.empty_like(qkv)
    lse = torch.empty(N, heads, T, device=dev)
    table = torch.randn(heads, 2 * T - 1, device=dev, generator=g) * 0.1
    dtable = torch.empty_like(table)
    L = _lib.lib()
    wsb = L.tagan_temporal_attn_bwd_workspace(N, T, heads, d)
    ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    b, db, es = qkv.data_ptr(), dqkv.data_ptr(), qkv.element_size()
    code = 1 if a.bf16 else 0
    sr, st = 3 * H, N * 3 * H

    kb = int(L.tagan_temporal_attn_keep_bytes(N, T, heads, d, a.causal, 0, 0, a.p)) if a.keep else 0
    keep = torch.empty(max(kb // 4, 1), dtype=torch.int32, device=dev)
    written = ctypes.c_int32(0)

    def fwd():
        _lib.check(L.tagan_temporal_attn_fwd_keep(code, N, T, heads, d, b, b + H * es, b + 2 * H * es, sr, st,
                                                  _lib.ptr(table), None, 0, None, 0, 0, a.causal, a.p, 99,
                                                  _lib.ptr(out), H, N * H, _lib.ptr(lse), None,
                                                  _lib.ptr(keep) if kb else None, kb, ctypes.byref(written), sp),
                   "fwd")

    def bwd():
        kp = _lib.ptr(keep) if written.value else None
        _lib.check(L.tagan_temporal_attn_bwd_keep(code, N, T, heads, d, b, b + H * es, b + 2 * H * es, sr, st,
                                                  _lib.ptr(table), None, 0, None, 0, 0, a.causal, a.p, 99,
                                                  _lib.ptr(out), H, N * H, _lib.ptr(lse), _lib.ptr(dout), H, N * H,
                                                  db, db + H * es, db + 2 * H * es, sr, st, _lib.ptr(dtable), None,
                                                  None, kp, kb if written.value else 0, _lib.ptr(ws), wsb, sp), "bwd")

    for _ in range(3):
        fwd()
        bwd()
    stream = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(a.reps):
        ev[0].record(stream)
        fwd()
        ev[1].record(stream)
        bwd()
        ev[2].record(stream)
        ev[2].synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    tf, tb = tf / a.reps, tb / a.reps
    unit = N * T * H * es
    bf = 4 * unit + N * heads * T * 4
    v4 = os.environ.get("TAGAN_TATTN_V4", "1") != "0" and T <= 32 and d in (16, 32)
    v5 = os.environ.get("TAGAN_TATTN_V5", "1") != "0" and 16 < T <= 128 and d in (16, 32)
    bb = (7 if (v4 or v5) else 8) * unit + N * heads * T * 4   # v4/v5 take delta from P·dP and never read O
    mm = 2.0 * T * T * d * N * heads   # flops of one T x T x d product over all units
    chk = [float(out.double().abs().sum()), float(dqkv.double().abs().sum()), float(dtable.double().abs().sum())]
    print(json.dumps({"lib": os.environ.get("TAGAN_LIB", "default"), "config": a.config, "dtype": "bf16" if a.bf16 else "f32", "rows": N, "T": T,
                      "heads": heads, "d": d, "p": a.p, "keep_bits": bool(written.value), "ms_fwd": round(tf, 4), "ms_bwd": round(tb, 4),
                      "gbs_fwd": round(bf / tf / 1e6, 1), "gbs_bwd": round(bb / tb / 1e6, 1),
                      "frac_hbm": round((bf + bb) / (tf + tb) / 1e6 / bench.HBM_PEAK_GBS, 4),
                      "tflops_fwd": round(2 * mm / tf / 1e9, 1), "tflops_bwd": round(5 * mm / tb / 1e9, 1),
                      "checksums": chk}), flush=True)


if __name__ == "__main__":
    main()
