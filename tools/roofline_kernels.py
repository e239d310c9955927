"""Run only the edge-softmax kernels (fwd + bwd) on the bench graph (bench.roofline_cache_assisted: all 32 C2
snapshots as one graph) — target for rocprofv3 --pmc passes (profiles/pmc_c2.json via tools/pmc_summary.py).

    rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d OUT -- python tools/roofline_kernels.py [c2]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import tagan_amd  # noqa: E402
from tagan_amd import synthetic  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    dev = torch.device("cuda")
    cfg = synthetic.config_for(name)
    seq = synthetic.make_sequence(name, dev, seed=1000)
    print(bench.roofline_cache_assisted(seq, cfg, reps=5))


if __name__ == "__main__":
    main()
