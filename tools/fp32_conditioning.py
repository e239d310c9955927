"""How well can ANY fp32 implementation match fp64 at C2?  Runs the CPU oracle (oracle/tagan_oracle.py) on the
C2 workload in fp32 and in fp64 from the same parameters/inputs and reports every gradient tensor whose fp32
normwise relative error exceeds 2e-5.  Test infrastructure (not the product): the result justifies the
tensor-specific tolerance exceptions of tests/test_gpu_fullsize.py.

    python tools/fp32_conditioning.py [--out profiles/r2_fp32_conditioning.json]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import tagan_amd  # noqa: E402,F401
from tagan_amd import TAGAN, synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    cfg = synthetic.config_for("c2", dropout=0.0, device="cpu")
    torch.manual_seed(0)
    model = TAGAN(cfg)
    seq = synthetic.make_sequence("c2", "cpu", seed=1000)
    lab = torch.tensor([1.0])
    grads, secs = {}, {}
    for dt in (torch.float32, torch.float64):
        P = {k: v.detach().to(dt).requires_grad_(v.is_floating_point()) for k, v in model.state_dict().items()}
        s = [(x.to(dt), ei, None, ids) for x, ei, _, ids in seq]
        t0 = time.time()
        out = oracle.tagan_forward(P, cfg.to_dict(), s, lab.to(dt))
        out["loss"].backward()
        secs[str(dt)] = round(time.time() - t0, 1)
        grads[dt] = {k: v.grad.double() for k, v in P.items() if v.grad is not None}
    rows = {}
    for k, want in grads[torch.float64].items():
        got = grads[torch.float32][k]
        nr = float((got - want).norm() / want.norm().clamp_min(1e-300))
        rows[k] = {"normwise_rel": nr, "max_abs": float((got - want).abs().max()), "norm": float(want.norm())}
    worst = {k: v for k, v in rows.items() if v["normwise_rel"] > 2e-5}
    for k, v in sorted(worst.items()):
        print("%-70s normwise %.2e  max_abs %.2e  |g| %.2e" % (k, v["normwise_rel"], v["max_abs"], v["norm"]))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"what": "CPU oracle fp32 vs fp64 at C2 (10k nodes, 32 snapshots, H=128, 8 heads, dropout 0)",
                       "threads": a.threads, "seconds": secs, "above_2e-5": worst, "all": rows}, f, indent=1)


if __name__ == "__main__":
    main()
