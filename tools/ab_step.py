"""Same-process A/B of fused-LayerNorm variants of the C2 training step (graph replays, interleaved).

Each variant sets ``fused.SG_LN_OPS`` (the ops of the LN-fused stream GEMMs) before its own HIP-graph capture of the
bench step; the graphs are then replayed round-robin, HIP events around each block of replays, and the median per
variant is reported.  Box-to-box (DVFS) differences cancel, which separate-process A/Bs do not guarantee.

    python tools/ab_step.py [--precision fp32|bf16] [--rounds 7] [--reps 10] none in in+out all default
"""
import argparse
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--config", default="c2")
    args = ap.parse_args()
    import bench
    from tagan_amd import TAGAN, fused, synthetic
    from tagan_amd.gemm_tuning import use_tuned_gemms
    use_tuned_gemms()
    dev = torch.device("cuda", 0)
    cfg = synthetic.config_for(args.config)
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=args.precision).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay, capturable=True,
                           fused=True)
    seq = synthetic.make_sequence(args.config, dev, seed=1000)
    labels = torch.tensor([1.0], device=dev)

    def fwd():
        return model(seq, labels=labels)

    DEFAULT_OPS = dict(fused.SG_LN_OPS)
    graphs = {}
    for v in args.variants:
        # "<ln ops>": the LayerNorm-fused stream-GEMM op set of this precision (fused.SG_LN_OPS) for this variant's
        # capture: none, all, default, or a "+"-list of in / out / bwd
        bf = args.precision != "fp32"
        default = DEFAULT_OPS[bf]
        fused.SG_LN_OPS[bf] = (frozenset() if v == "none" else frozenset({"in", "out", "bwd", "ln2bwd"}) if v == "all" else
                               default if v == "default" else frozenset(v.replace("+", ",").split(",")))
        fused._SG_LN_OK.clear()
        graphs[v] = bench.graphed(model, opt, cfg, fwd)
    times = {v: [] for v in args.variants}
    st = torch.cuda.current_stream()
    for _ in range(args.rounds):
        for v in args.variants:
            g = graphs[v]
            g()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.reps):
                g()
            e1.record(st)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.reps)
    for v in args.variants:
        print("%s %s median %.3f ms  (min %.3f, max %.3f)" % (args.precision, v, statistics.median(times[v]),
                                                              min(times[v]), max(times[v])), flush=True)
    for g in graphs.values():
        g.close()


if __name__ == "__main__":
    main()
