"""Host launch time vs device time of one C2 training step (is the step launch-bound?).

For each step: sync, t0, step() returns (host has issued everything) -> t1, sync -> t2.
host = t1 - t0, wall = t2 - t0.  If host ~ wall the step is bound by host-side launch work.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tagan_amd  # noqa: E402,F401
from tagan_amd import TAGAN, synthetic  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    dev = torch.device("cuda")
    cfg = synthetic.config_for(name)
    torch.manual_seed(0)
    model = TAGAN(cfg).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay)
    seq = synthetic.make_sequence(name, dev, seed=1000)
    labels = torch.tensor([1.0], device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        out = model(seq, labels=labels)
        out["loss"].backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.gradient_clip_val)
        opt.step()

    for _ in range(3):
        step()
    hs, ws = [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        hs.append(t1 - t0)
        ws.append(t2 - t0)
    print("host launch ms/step: %.3f   wall ms/step: %.3f" % (1e3 * sorted(hs)[5], 1e3 * sorted(ws)[5]))
    # forward alone
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = model(seq, labels=labels)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("forward host %.3f wall %.3f" % (1e3 * (t1 - t0), 1e3 * (t2 - t0)))
    t0 = time.perf_counter()
    out["loss"].backward()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("backward host %.3f wall %.3f" % (1e3 * (t1 - t0), 1e3 * (t2 - t0)))


if __name__ == "__main__":
    main()
