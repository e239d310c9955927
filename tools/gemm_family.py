"""The C2 training step's GEMM family, per shape: device time per step (torch.profiler over one eager step, the
bench's TunableOp table enabled), FLOPs, TF/s and the fraction of the dense MFMA peak of the operand type
(fp32 157.3 TF/s, bf16 2.5 PF/s; MI355X_MICROARCH.md).  Eager launches, warm stream; the graph-replayed step's
kernel times are in the rocprof summaries (profiles/r2g_c2_kernel_stats.csv).

    python tools/gemm_family.py [--precision fp32|bf16]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tagan_amd  # noqa: E402,F401
from tagan_amd import TAGAN, synthetic  # noqa: E402
from tagan_amd.gemm_tuning import use_tuned_gemms  # noqa: E402

PEAK = {"fp32": 157.3, "bf16": 2500.0}


def flops(key, shapes):
    if key in ("aten::mm",):
        (m, k), (_, n) = shapes[0], shapes[1]
        return 2.0 * m * n * k
    if key == "aten::addmm":
        (m, k), (_, n) = shapes[1], shapes[2]
        return 2.0 * m * n * k
    if key == "aten::bmm":
        (b, m, k), (_, _, n) = shapes[0], shapes[1]
        return 2.0 * b * m * n * k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="fp32", choices=("fp32", "bf16"))
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    use_tuned_gemms()
    dev = torch.device("cuda")
    cfg = synthetic.config_for(args.config)
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=args.precision).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay)
    seq = synthetic.make_sequence(args.config, dev, seed=1000)
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
    reps = 3
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(reps):
            step()
        torch.cuda.synchronize()
    rows, tot_t, tot_f = [], 0.0, 0.0
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key not in ("aten::mm", "aten::addmm", "aten::bmm"):
            continue
        shapes = [s for s in e.input_shapes if s]
        f = flops(e.key, shapes)
        if not f:
            continue
        us = e.device_time_total / reps
        calls = e.count / reps
        tf = f * calls / (us * 1e-6) / 1e12 if us > 0 else 0.0
        rows.append((us, calls, e.key, shapes, f * calls, tf))
        tot_t += us
        tot_f += f * calls
    peak = PEAK[args.precision]
    print("# %s, %s step, GEMM family per shape (us per step, calls per step, GFLOP per step, TF/s, of %.1f TF/s)"
          % (args.config, args.precision, peak))
    for us, calls, key, shapes, f, tf in sorted(rows, reverse=True):
        if f < 1e8:
            continue
        print("%9.1f us %4.1f  %-11s %-44s %7.2f GF %7.1f TF/s  %5.1f %%" % (us, calls, key, shapes, f / 1e9, tf,
                                                                           100 * tf / peak))
    print("total %.1f us per step, %.1f GFLOP, %.1f TF/s = %.1f %% of the %s MFMA peak"
          % (tot_t, tot_f / 1e9, tot_f / (tot_t * 1e-6) / 1e12, 100 * tot_f / (tot_t * 1e-6) / 1e12 / peak,
             args.precision))


if __name__ == "__main__":
    main()
