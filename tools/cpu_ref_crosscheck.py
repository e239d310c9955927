"""CONTAINER-ONLY: time the literal reference CPU path and the oracle's restatements at C1.

BASELINE.md §CPU-baseline plan step 2: the oracle's ``dense_faithful`` mode (dense N×N mask plus the
per-(head, node) distance loop of geometric_attention.py:386-401 / graph_attention.py:96-105) must match
the literal reference's C1 throughput within ~10 % on the same cores before its GPU-box timings are
quoted as "reference CPU path".  This script imports the read-only reference from /root/reference
(scratch cwd, stdout/stderr swallowed, bytecode off — SURVEY.md §8c), runs TAGAN.forward + backward
on the C1 workload (example.py:35-48 shapes, N = 500, T = 10, train mode, dropout 0.1) and times, with
the same threads, the oracle in ``dense_faithful`` and ``sparse`` mode on the same inputs and weights.

    python tools/cpu_ref_crosscheck.py [--threads 8] [--reps 3] [--out profiles/r2_cpu_crosscheck.json]
    python tools/cpu_ref_crosscheck.py --sweep [--out profiles/r2_cpu_crosscheck_c2sweep.json]

``--sweep``: the C2 shape (H = 128, 8 heads, F = 27, euclidean, dropout 0.1) at N = 250 / 500 / 1000 with E = 10 N
and 1 snapshot (best of 2), literal reference against ``dense_faithful`` (bench.py's sweep, same inputs and weights), both
power laws fitted and extrapolated to C2's N = 10,000: the check behind the bench's extrapolated C2
``cpu_baseline.dense_faithful``.

Never runs on the GPU box (the reference does not travel); the result is committed under profiles/.
"""
import argparse
import contextlib
import io
import json
import os
import platform
import sys
import tempfile
import time

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


def _quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        return fn(*a, **k)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _fit(pts):
    import math
    xs = [math.log(n) for n, _ in pts]
    ys = [math.log(t) for _, t in pts]
    mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
    p = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    return p, math.exp(my - p * mx)


def sweep(args):
    import torch
    torch.set_num_threads(args.threads)
    sys.path.insert(0, ROOT)
    import oracle
    from tagan_amd import synthetic
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp(prefix="tagan_xcheck_"))
    nodes, snaps = (250, 500, 1000), 1
    try:
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            from src.tagan.model import TAGAN as RefTAGAN
            from src.tagan.utils.config import TAGANConfig as RefConfig
        N2, E2, T2, H, heads, F, De, _ = synthetic.CONFIGS["c2"]
        kw = dict(hidden_dim=H, num_heads=heads, node_feature_dim=F, edge_feature_dim=De, use_edge_features=True,
                  output_dim=1, loss_type="bce", dropout=0.1, device="cpu")
        torch.manual_seed(0)
        model = _quiet(RefTAGAN, _quiet(RefConfig, **kw)).train()
        P = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in model.state_dict().items()}
        labels = torch.tensor([1.0])
        small = synthetic.make_sequence("c2", "cpu", seed=1, snapshots=1, nodes=100, edges=1000)
        _quiet(lambda: model(small, labels=labels)["loss"].backward())          # warm-up
        oracle.tagan_forward(P, dict(kw), small, labels, mode="dense_faithful")["loss"].backward()
        lit, dfa = [], []
        for n in nodes:
            seq = synthetic.make_sequence("c2", "cpu", seed=7, snapshots=snaps, nodes=n, edges=10 * n)
            tl = td = float("inf")
            for _ in range(2):                     # best of 2, interleaved (as bench.py's sweep)
                t0 = time.perf_counter()
                _quiet(lambda: model(seq, labels=labels)["loss"].backward())
                tl = min(tl, time.perf_counter() - t0)
                t0 = time.perf_counter()
                oracle.tagan_forward(P, dict(kw), seq, labels, mode="dense_faithful")["loss"].backward()
                td = min(td, time.perf_counter() - t0)
            lit.append((n, tl / snaps))
            dfa.append((n, td / snaps))
            print(n, lit[-1][1], dfa[-1][1], flush=True)
    finally:
        os.chdir(cwd)
    pl, al = _fit(lit)
    pd, ad = _fit(dfa)
    ext_l, ext_d = 1.0 / (al * N2 ** pl), 1.0 / (ad * N2 ** pd)
    rec = {"workload": "C2 shape (H=128, 8 heads, F=27, euclidean, train, dropout 0.1), N = 250/500/1000, E = 10 N, "
                       "1 snapshot (best of 2), TAGAN.forward + loss.backward(); seconds per snapshot",
           "host": {"cpu_model": _cpu_model(), "nproc": os.cpu_count(), "threads": args.threads},
           "torch": torch.__version__,
           "reference_literal": {str(n): round(t, 3) for n, t in lit},
           "oracle_dense_faithful": {str(n): round(t, 3) for n, t in dfa},
           "fit_exponent": {"reference_literal": round(pl, 3), "oracle_dense_faithful": round(pd, 3)},
           "extrapolated_c2_snapshots_per_s": {"reference_literal": float("%.3g" % ext_l),
                                               "oracle_dense_faithful": float("%.3g" % ext_d)},
           "dense_faithful_over_literal_per_N": {str(n): round(tl / td, 3) for (n, tl), (_, td) in zip(lit, dfa)},
           "dense_faithful_over_literal_at_c2": round(ext_d / ext_l, 3)}
    out = args.out or os.path.join(ROOT, "profiles", "r2_cpu_crosscheck_c2sweep.json")
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.sweep:
        return sweep(args)
    if args.out is None:
        args.out = os.path.join(ROOT, "profiles", "r2_cpu_crosscheck.json")
    import torch
    torch.set_num_threads(args.threads)
    sys.path.insert(0, ROOT)
    import oracle
    from tagan_amd import synthetic
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp(prefix="tagan_xcheck_"))
    try:
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            from src.tagan.model import TAGAN as RefTAGAN
            from src.tagan.utils.config import TAGANConfig as RefConfig
        N, E, T, H, heads, F, De, _ = synthetic.CONFIGS["c1"]
        kw = dict(hidden_dim=H, num_heads=heads, node_feature_dim=F, edge_feature_dim=De, use_edge_features=True,
                  output_dim=1, loss_type="bce", dropout=0.1, device="cpu")
        torch.manual_seed(0)
        ref = _quiet(RefConfig, **kw)
        model = _quiet(RefTAGAN, ref).train()
        seq = synthetic.make_sequence("c1", "cpu", seed=42)
        labels = torch.tensor([1.0])

        def ref_step():
            out = _quiet(model, seq, labels=labels)
            _quiet(out["loss"].backward)

        P = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in model.state_dict().items()}

        def oracle_step(mode):
            out = oracle.tagan_forward(P, dict(kw), seq, labels, mode=mode)
            out["loss"].backward()

        fns = (("reference_literal", ref_step), ("oracle_dense_faithful", lambda: oracle_step("dense_faithful")),
               ("oracle_sparse", lambda: oracle_step("sparse")))
        for _, fn in fns:
            fn()                                                    # warm-up
        times = {name: [] for name, _ in fns}
        for _ in range(args.reps):                                  # interleaved: host drift hits every mode alike
            for name, fn in fns:
                t0 = time.perf_counter()
                fn()
                times[name].append(time.perf_counter() - t0)
        res = {}
        for name, ts in times.items():
            ts.sort()
            res[name] = {"snapshots_per_s_best": round(T / ts[0], 4), "snapshots_per_s_median": round(T / ts[len(ts) // 2], 4),
                         "seconds": [round(t, 3) for t in ts]}
    finally:
        os.chdir(cwd)
    lit = res["reference_literal"]["snapshots_per_s_best"]          # best of reps, as BASELINE.md
    dfa = res["oracle_dense_faithful"]["snapshots_per_s_best"]
    rec = {"workload": "C1: example.py shapes, N=500, E=1000, T=10, H=64, 4 heads, euclidean, train mode, dropout 0.1, "
                       "TAGAN.forward + loss.backward()",
           "host": {"cpu_model": _cpu_model(), "nproc": os.cpu_count(), "threads": args.threads},
           "torch": torch.__version__, "reps": args.reps, "results": res,
           "dense_faithful_over_literal_best": round(dfa / lit, 4),
           "dense_faithful_over_literal_median": round(res["oracle_dense_faithful"]["snapshots_per_s_median"]
                                                       / res["reference_literal"]["snapshots_per_s_median"], 4),
           "within_10pct": abs(dfa / lit - 1.0) <= 0.10}
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
