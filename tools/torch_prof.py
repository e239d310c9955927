"""torch.profiler view of one C2 training step: which framework ops launch the small fills/copies/adds.

    python tools/torch_prof.py [--config c2]
"""
import os
import sys

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
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    keys = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::sum", "aten::cat", "aten::clone",
            "aten::contiguous", "aten::to", "aten::mul")
    for e in prof.key_averages(group_by_stack_n=6):
        if any(e.key.startswith(k) for k in keys):
            print("%-22s calls=%3d  dev_us=%8.1f" % (e.key, e.count, e.device_time_total))
            for fr in (e.stack or [])[:6]:
                print("      ", fr)
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=40))
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in ("aten::add", "aten::add_", "aten::copy_", "aten::fill_", "aten::zero_", "aten::sum",
                     "aten::mul", "aten::cat", "aten::clone", "aten::mm", "aten::addmm", "aten::bmm",
                     "aten::linear", "aten::_efficientzerotensor"):
            print("%-14s calls=%3d dev_us=%8.1f shapes=%s" % (e.key, e.count, e.device_time_total, e.input_shapes))


if __name__ == "__main__":
    main()
