"""Phase timings of the fused head kernels: run the C2 head (T = 32, H = 128, C = 1, B = 1, BCE, dropout 0.1) a few
times forward + backward.  With TAGAN_LIB pointing at a build of csrc/head.hip instrumented with per-barrier
wall-clock stamps (printf "HEADPROF fwd|bwd line:ticks ..."; 100 MHz ticks) the kernels print their phase costs;
with the shipped library it times the two launches.
    python tools/head_probe.py [--T 32 --H 128 --reps 5]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32)
    ap.add_argument("--H", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import bench  # noqa: F401  (registers the tagan_amd package alias)
    import tagan_amd  # noqa: F401
    from tagan_amd.layers.classification import ClassificationModule, fused_head
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = ClassificationModule(hidden_dim=a.H, task_configs={"output_dim": 1, "task_type": "classification"},
                             multi_task=False, num_layers=2, dropout=0.1, use_layer_norm=True).to(dev).train()
    pooled = (torch.randn(a.T, a.H, device=dev) * 0.5).requires_grad_()
    labels = torch.ones(1, device=dev)
    for _ in range(a.reps):
        logits, preds, loss = fused_head(m, pooled, 1, labels, 1, seed=7)
        loss.backward()
        torch.cuda.synchronize()
    print("done", float(loss))


if __name__ == "__main__":
    main()
