"""Condition numbers of the C2 model with respect to the bf16 stores of the bf16 activation mode.

The bf16 mode (fused.py "bf16") rounds, per attention block, five tensors in the forward -- h = LN1(x), Q|K|V, the
attention output, the two weight operands W_qkv and W_o -- and three in the backward -- d(out-projection output),
d(context), dQ|dK|dV.  A round-to-nearest store perturbs every element by an independent relative error of RMS
U_RMS = 2^-8 / sqrt(3).  To first order the error of an output tensor t is a sum over the store sites s:

    delta_t = sum_s J_{t,s} (xi_s * v_s) U_RMS,     xi_s i.i.d. unit-RMS per element,
    E ||delta_t||^2 / ||t||^2 = U_RMS^2 sum_s kappa_{t,s}^2,   kappa_{t,s} = ||J_{t,s} diag(v_s)||_F / ||t||

(kappa_{t,s} is the relative condition number of t for elementwise relative perturbations at site s).  This script
measures sqrt(sum_s kappa_{t,s}^2) with the fp64 oracle (oracle/tagan_oracle.py, test infrastructure): forward +
backward runs with every site's values perturbed at once by independent eps * xi (xi uniform on [-sqrt 3, sqrt 3],
eps = 1e-6, the linear regime), kappa_rss = RMS over --joint draws of ||t - t_0|| / (eps ||t_0||), on the C2
workload of the test (the bench's generator and model initialisation, on the CPU); --per-site adds kappa_{t,s}
from one draw per site.  It writes tests/golden/bf16_conditioning.json, which
tests/test_gpu_fullsize.py::test_c2_bf16_vs_oracle turns into its bound.

Usage: python tools/bf16_conditioning.py [--nodes 10000] [--edges 100000] [--out tests/golden/bf16_conditioning.json]
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import oracle.tagan_oracle as O  # noqa: E402

BLOCKS = ("geometric_attention_layers.0.geometric_attention", "geometric_attention_layers.1.geometric_attention",
          "temporal_attention")
KINDS = ("h", "qkv", "ctx", "w_qkv", "w_o", "d_o", "d_ctx", "d_qkv")


class _GradNoise(torch.autograd.Function):
    """Identity forward; backward multiplies the incoming gradient by (1 + noise)."""

    @staticmethod
    def forward(ctx, x, noise):
        ctx.save_for_backward(noise)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        (noise,) = ctx.saved_tensors
        return g * (1.0 + noise), None


def _classify(name):
    for b in BLOCKS:
        if name.startswith(b + "."):
            tail = name[len(b) + 1:]
            if tail in ("q_linear", "k_linear", "v_linear"):
                return b, "qkv"
            if tail == "output_proj":
                return b, "o"
    return None, None


def run(P, cfg, seq, labels, site=None, eps=0.0, seed=0):
    """One fp64 forward + backward; ``site`` = (block, kind) perturbed by eps * xi, or "all": every site at once
    (independent noise per site and element)."""
    gen = torch.Generator().manual_seed(seed)
    shared = {}

    def noise_like(t):
        return (torch.rand(t.shape, generator=gen, dtype=t.dtype) * 2.0 - 1.0) * (math.sqrt(3.0) * eps)

    def lin(x, Pm, name):
        block, kind = _classify(name)
        if block is None or (site != "all" and (site is None or block != site[0])):
            return F.linear(x, Pm[name + ".weight"], Pm.get(name + ".bias"))
        on = (lambda s: True) if site == "all" else (lambda s: s == site[1])
        W = Pm[name + ".weight"]
        if kind == "qkv" and on("h"):   # h is stored once and read by the three consecutive projections
            if shared.get("x") is not x:
                shared["x"], shared["h"] = x, x * (1.0 + noise_like(x))
            x = shared["h"]
        if kind == "o" and on("ctx"):
            x = x * (1.0 + noise_like(x))
        if kind == "o" and on("d_ctx"):
            x = _GradNoise.apply(x, noise_like(x))
        if (kind == "qkv" and on("w_qkv")) or (kind == "o" and on("w_o")):
            W = W * (1.0 + noise_like(W))
        y = F.linear(x, W, Pm.get(name + ".bias"))
        if kind == "qkv" and on("qkv"):
            y = y * (1.0 + noise_like(y))
        if (kind == "qkv" and on("d_qkv")) or (kind == "o" and on("d_o")):
            y = _GradNoise.apply(y, noise_like(y))
        return y

    saved = O._lin
    O._lin = lin
    try:
        for v in P.values():
            v.grad = None
        xs = [(x.detach().clone().requires_grad_(True), ei, None, ids) for x, ei, _, ids in seq]
        out = O.tagan_forward(P, cfg, xs, labels)
        out["loss"].backward()
    finally:
        O._lin = saved
    res = {"logits": out["logits"].detach().clone(), "loss": out["loss"].detach().reshape(1).clone()}
    for k, v in P.items():
        if v.grad is not None:
            res["grad " + k] = v.grad.detach().clone()
    res["grad x"] = torch.cat([x.grad.detach().reshape(-1) for x, _, _, _ in xs])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10_000)
    ap.add_argument("--edges", type=int, default=100_000)
    ap.add_argument("--eps", type=float, default=1e-6)
    ap.add_argument("--joint", type=int, default=16, help="draws of the all-sites-at-once estimate")
    ap.add_argument("--per-site", action="store_true", help="also the per-site breakdown (one draw per site)")
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "bf16_conditioning.json"))
    a = ap.parse_args()
    torch.set_num_threads(max(1, os.cpu_count() or 1))
    from tagan_amd import TAGAN, synthetic
    cfg = synthetic.config_for("c2", dropout=0.0)
    torch.manual_seed(0)
    model = TAGAN(cfg)
    P = {k: v.detach().double().requires_grad_(v.is_floating_point()) for k, v in model.state_dict().items()}
    seq = synthetic.make_sequence("c2", torch.device("cpu"), seed=1000, nodes=a.nodes, edges=a.edges)
    seq = [(x.double(), ei, None, ids) for x, ei, _, ids in seq]
    labels = torch.tensor([1.0], dtype=torch.float64)
    cd = cfg.to_dict()
    t0 = time.time()
    base = run(P, cd, seq, labels)
    print("baseline %.1f s" % (time.time() - t0), flush=True)
    # every site perturbed at once, independently: E||t - t0||^2 = U^2 ||t0||^2 sum_s kappa_{t,s}^2 to first order,
    # so the RMS over draws estimates kappa_rss directly (one draw of a scalar output is a single |N(0, 1)| sample:
    # the per-site single-draw figures below are a breakdown, not the bound)
    acc = {k: 0.0 for k in base}
    for r in range(a.joint):
        t1 = time.time()
        got = run(P, cd, seq, labels, "all", a.eps, seed=10_000 + r)
        for k, v0 in base.items():
            acc[k] += float((got[k] - v0).norm()) ** 2
        print("joint draw %d %.1f s" % (r, time.time() - t1), flush=True)
    kappa_rss = {k: math.sqrt(acc[k] / a.joint) / (a.eps * float(v0.norm()))
                 for k, v0 in base.items() if float(v0.norm()) > 0}
    kappa = {k: {} for k in base}
    for bi, b in enumerate(BLOCKS if a.per_site else ()):
        for ki, s in enumerate(KINDS):
            t1 = time.time()
            got = run(P, cd, seq, labels, (b, s), a.eps, seed=1 + 16 * bi + ki)
            for k, v0 in base.items():
                n0 = float(v0.norm())
                if n0 > 0:
                    kappa[k]["%s:%s" % (b, s)] = float((got[k] - v0).norm()) / (a.eps * n0)
            print("%-52s %-6s %.1f s" % (b, s, time.time() - t1), flush=True)
    out = {"note": "relative condition numbers of each output tensor w.r.t. elementwise relative perturbations at "
                   "each bf16 store site of the bf16 activation mode (tools/bf16_conditioning.py, fp64 oracle)",
           "workload": {"config": "c2", "nodes": a.nodes, "edges": a.edges, "snapshots": len(seq), "seed": 1000,
                        "model_seed": 0, "eps": a.eps},
           "sites": ["%s:%s" % (b, s) for b in BLOCKS for s in KINDS],
           "joint_draws": a.joint,
           "kappa_rss": kappa_rss,
           "kappa": {k: d for k, d in kappa.items() if d}}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote %s (%.0f s)" % (a.out, time.time() - t0))


if __name__ == "__main__":
    main()
