"""Time the edge-softmax kernels (fwd, bwd) alone on a config's synthetic graph.

    python tools/geo_kernels.py [--config c2] [--snapshots T] [--chunk 128] [--metric 0] [--reps 20]

Prints one JSON line: ms_fwd, ms_bwd, algorithmic GB/s (bench.geo_bytes) and the
fraction of the 8 TB/s HBM peak.  TAGAN_LIB=<path> selects an alternative build of
libtagan_hip.so (kernel-variant sweeps).  The synthetic graph of C4 (1M nodes, 20M
uniform edges per snapshot) is the SURVEY §8(d) roofline configuration.
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
from tagan_amd.kernels import CHUNK, build_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--snapshots", type=int, default=None)
    ap.add_argument("--chunk", type=int, default=None)
    ap.add_argument("--metric", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--p", type=float, default=0.1)
    ap.add_argument("--bf16", action="store_true", help="bf16 activation storage (TAGAN_BF16)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N0, E0, T, H, heads = synthetic.CONFIGS[a.config][:5]
    T = a.snapshots or T
    seq = synthetic.make_sequence(a.config, dev, seed=1000, snapshots=T)
    graph = build_graph([ei for _, ei, _, _ in seq], [int(x.shape[0]) for x, _, _, _ in seq], chunk=a.chunk or CHUNK)
    del seq
    N, d = graph.num_nodes, H // heads
    E = graph.nnz_host()
    g = torch.Generator(device=dev).manual_seed(7)
    adt = torch.bfloat16 if a.bf16 else torch.float32
    qkv = torch.randn(N, 3 * H, device=dev, generator=g).to(adt)
    dout = torch.randn(N, H, device=dev, generator=g).to(adt)
    out = torch.empty(N, H, device=dev, dtype=adt)
    lse = torch.empty(N, heads, device=dev)
    dqkv = torch.empty_like(qkv)
    prm = torch.ones(heads, device=dev)
    dprm = torch.zeros(heads, device=dev)
    L = _lib.lib()
    gs = graph.struct()
    fwb = L.tagan_geo_attn_fwd_workspace(gs, heads, d)
    fws = torch.empty(max(int(fwb), 1), dtype=torch.uint8, device=dev)
    wsb = L.tagan_geo_attn_bwd_workspace(gs, heads, d)
    ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    b, db, es = qkv.data_ptr(), dqkv.data_ptr(), qkv.element_size()
    dt = _lib.TAGAN_BF16 if a.bf16 else 0
    learn = a.metric in (7, 8)
    pp, dpp = (_lib.ptr(prm), _lib.ptr(dprm)) if learn else (None, None)

    def fwd():
        _lib.check(L.tagan_geo_attn_fwd(dt, a.metric, gs, heads, d, b, b + H * es, b + 2 * H * es, 3 * H, pp, a.p,
                                        1234, _lib.ptr(out), _lib.ptr(lse), None, _lib.ptr(fws), fwb, sp), "fwd")

    def bwd():
        _lib.check(L.tagan_geo_attn_bwd(dt, a.metric, gs, heads, d, b, b + H * es, b + 2 * H * es, 3 * H, pp, a.p,
                                        1234, _lib.ptr(out), _lib.ptr(lse), _lib.ptr(dout), db, db + H * es,
                                        db + 2 * H * es, 3 * H, dpp, _lib.ptr(ws), wsb, sp), "bwd")

    for _ in range(3):
        fwd()
        bwd()
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
    bf, bb = bench.geo_bytes(E, N, H, heads, s=es)
    print(json.dumps({"lib": os.environ.get("TAGAN_LIB", "default"), "config": a.config, "snapshots": T,
                      "chunk": a.chunk or CHUNK, "dtype": "bf16" if a.bf16 else "f32", "metric": a.metric, "nodes": N, "edges": E, "H": H, "heads": heads,
                      "ms_fwd": round(tf, 4), "ms_bwd": round(tb, 4),
                      "gbs_fwd": round(bf / tf / 1e6, 1), "gbs_bwd": round(bb / tb / 1e6, 1),
                      "frac": round((bf + bb) / (tf + tb) / 1e6 / bench.HBM_PEAK_GBS, 4)}), flush=True)


if __name__ == "__main__":
    main()
