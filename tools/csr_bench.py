"""Time the snapshot CSR/CSC build (kernels.build_graph: tagan_csr_build + the chunk work lists) on the BASELINE
workloads' edge lists, HIP events on the launch stream, mean of ``--reps`` after 2 warm-ups.

    python tools/csr_bench.py [--configs c2,c4] [--reps 10] [--out profiles/x.json]

Reports per config: snapshots in the batch, raw edges, unique CSR entries (nnz), build ms, and the build's
algorithmic rate in raw edges per second.
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
from tagan_amd.kernels import build_graph  # noqa: E402


def time_build(eis, counts, reps):
    for _ in range(2):
        build_graph(eis, counts)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g = build_graph(eis, counts)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps, g.nnz_host()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda")
    res = []
    for name in args.configs.split(","):
        N, E, T = synthetic.CONFIGS[name][:3]
        for snaps in sorted({1, T}):
            seq = synthetic.make_sequence(name, dev, seed=1000, snapshots=snaps)
            eis = [ei for _, ei, _, _ in seq]
            counts = [int(x.shape[0]) for x, _, _, _ in seq]
            del seq
            ms, nnz = time_build(eis, counts, args.reps)
            rec = {"config": name, "snapshots": snaps, "nodes": sum(counts), "raw_edges": E * snaps, "nnz": nnz,
                   "build_ms": round(ms, 4), "raw_edges_per_s": round(E * snaps / ms * 1e3, 1)}
            print(json.dumps(rec), flush=True)
            res.append(rec)
            del eis
            torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
