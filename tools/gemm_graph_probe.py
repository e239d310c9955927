"""Probe: the C2 projection GEMM shapes launched eagerly vs replayed from a captured HIP graph, with the bench's
TunableOp table (the graph-replayed step's rocprof summary shows the out-projection GEMM at ~170 us per call against
~95 us eager).  HIP events around 20 calls on fresh operands per call (no cache reuse across calls).

    python tools/gemm_graph_probe.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tagan_amd.gemm_tuning import use_tuned_gemms  # noqa: E402

use_tuned_gemms()
dev = torch.device("cuda")
M, R = 320_000, 6
g = torch.Generator(device=dev).manual_seed(0)
SHAPES = {
    "out_fwd  a[M,128]@W^T[128,128]": (lambda a, w: a @ w.t(), (M, 128), (128, 128)),
    "out_dgrad a[M,128]@W[128,128]": (lambda a, w: a @ w, (M, 128), (128, 128)),
    "qkv_fwd  a[M,132]@W^T[132,384]": (lambda a, w: a @ w.t(), (M, 132), (384, 132)),
    "qkv_dgrad a[M,384]@W[384,128]": (lambda a, w: a @ w, (M, 384), (384, 128)),
}


def run(name, fn, sa, sw):
    As = [torch.randn(*sa, device=dev, generator=g) for _ in range(R)]
    w = torch.randn(*sw, device=dev, generator=g) / sw[1] ** 0.5
    outs = [None] * R

    def calls():
        for i in range(R):
            outs[i] = fn(As[i], w)

    for _ in range(2):
        calls()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        calls()
    e1.record()
    e1.synchronize()
    t_eager = e0.elapsed_time(e1) / (3 * R) * 1e3
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        calls()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        calls()
    graph.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(3):
        graph.replay()
    e1.record()
    e1.synchronize()
    t_graph = e0.elapsed_time(e1) / (3 * R) * 1e3
    print("%-34s eager %7.1f us   graph %7.1f us" % (name, t_eager, t_graph), flush=True)


for name, (fn, sa, sw) in SHAPES.items():
    run(name, fn, sa, sw)
