"""TAGAN training-step benchmark on MI355X (graph-snapshots/s, fwd+bwd+optimizer).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--shard] [--roofline-only]
  (N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N ... bench.py --gpus N)

One step = one TAGAN sequence (all T snapshots) per rank: forward, BCE loss,
backward, gradient all-reduce (N>1, RCCL), clip_grad_norm_(1.0), Adam step —
the reference trainer's step (trainer.py:295-311).  Inputs are synthetic, seeded
per rank and resident in HBM before timing; the snapshot CSR is rebuilt inside
every step.  Prints ONE JSON line on rank 0.

``--gpus N`` with N > 1 outside torchrun re-launches itself under ``torch.distributed.run`` with N ranks
(before anything touches the GPU); under torchrun (the driver's form) WORLD_SIZE must equal N.

roofline: the edge-softmax + aggregate kernels (tagan_geo_attn fwd, bwd-row, bwd-col;
geometric_attention.py:332-516 + :579-583) on a cache-cold C4 snapshot (SURVEY §8(d)'s roofline
configuration: 1M nodes, 20M uniform edges, H=128, 4 heads, fp32), timed with HIP events on the launch
stream; achieved = SURVEY §8(d)'s algorithmic bytes ÷ time, peak = 8.0 TB/s; traffic = the PMC HBM bytes
of the same launches (profiles/pmc_c4.json).  The same kernels on the bench's own C2 graph are reported
beside it as ``cache_assisted`` (C2's gathers are served partly by L2 / Infinity Cache).
cpu_baseline: the CPU oracle (oracle/, restatements of the reference algorithm) on bounded samples,
rank 0, N=1 only: sparse CSR at C2 (the headline ratio); dense_faithful (the reference's own dense N×N mask +
per-(head, node) loop) at C2 extrapolated from a measured N = 250/500/1000 sweep (labelled as such;
tools/cpu_ref_crosscheck.py --sweep sets the same sweep beside the literal reference); and at C1 both sparse and
dense_faithful (cross-checked against the literal reference in profiles/r2_cpu_crosscheck.json), next to a GPU
C1 step measured here.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-sample-snapshots", type=int, default=8)
    ap.add_argument("--precision", default="fp32", choices=("fp32", "bf16-gemm", "bf16"),
                    help="fp32 (parity mode); bf16-gemm: bf16 GEMM operands; bf16: bf16 activations between "
                         "kernels, fp32 math (BASELINE's C2 dtype)")
    ap.add_argument("--no-alt-precision", action="store_true",
                    help="skip the extra bf16-activation measurement reported as alt_precision")
    ap.add_argument("--no-tuned-gemms", action="store_true",
                    help="library-default GEMM solutions instead of the shipped TunableOp table (gemm_tuning.py)")
    ap.add_argument("--tune-gemms", action="store_true",
                    help="time every GEMM solution of the shapes missing from the table; write the table at exit")
    ap.add_argument("--gemm-table", default=None, help="TunableOp table path (default: the shipped one)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the C4 roofline launches (for rocprofv3 kernel-trace / PMC passes of the same kernels)")
    ap.add_argument("--roofline-reps", type=int, default=10)
    ap.add_argument("--no-c1", action="store_true", help="skip the GPU C1 line beside the C1 CPU baselines")
    ap.add_argument("--launch", default="auto", choices=("auto", "graph", "eager"),
                    help="graph: replay the step as a HIP graph (graph_step.py); eager: launch every kernel from "
                         "Python; auto (default): time a short trial of both and keep the faster")
    ap.add_argument("--no-graph", action="store_true", help="same as --launch eager")
    ap.add_argument("--sub-records", default="auto",
                    help="BASELINE multi-GPU workloads measured beside the headline: auto (c3_dp at N = 2, 4; "
                         "c5_shard at N = 8), none, or a comma list of c3_dp, c5_shard")
    ap.add_argument("--c5-shard-size", default=None,
                    help="NODES,EDGES per snapshot for the c5_shard sub-record (a reduced rehearsal; default C5's)")
    ap.add_argument("--shard", action="store_true",
                    help="one sequence sharded by snapshot over all ranks (strong scaling; C5 mode) instead of "
                         "one sequence per rank (data parallel, weak scaling)")
    return ap.parse_args()


def geo_bytes(E, N, H, heads=None, s=4):
    """SURVEY §8(d)'s algorithmic HBM bytes of one geometric layer over N nodes / E' CSR entries:
    B_fwd = s·H·(2E' + 2N) + 4(E' + N) (K_j, V_j gathered per edge; Q_i read, O_i written; CSR col + rowptr);
    B_bwd = s·H·(4E' + 8N) + 8(E' + N) (CSR pass gathers K_j, V_j; CSC pass gathers Q_i, dO_i; per node Q, K, V,
    O, dO read and dQ, dK, dV written; CSR + CSC indices)."""
    fwd = s * H * (2 * E + 2 * N) + 4 * (E + N)
    bwd = s * H * (4 * E + 8 * N) + 8 * (E + N)
    return fwd, bwd


class EdgeKernels:
    """The edge-softmax + aggregate launches of one geometric layer (fwd; bwd row + col passes) through the
    C-ABI on a graph, random Q|K|V and dO, launched on the current stream."""

    def __init__(self, graph, H, heads, p_drop, metric=0):
        import ctypes
        from tagan_amd import _lib
        dev = graph.rowptr.device
        self.graph, self.H, self.heads, self.p, self.metric = graph, H, heads, float(p_drop), metric
        self.N, self.d = graph.num_nodes, H // heads
        self.E = graph.nnz_host()
        g = torch.Generator(device=dev).manual_seed(7)
        self.qkv = torch.randn(self.N, 3 * H, device=dev, generator=g)
        self.dout = torch.randn(self.N, H, device=dev, generator=g)
        self.out = torch.empty(self.N, H, device=dev)
        self.lse = torch.empty(self.N, heads, device=dev)
        self.dqkv = torch.empty_like(self.qkv)
        L = self.L = _lib.lib()
        self.gs = graph.struct()
        self.fwb = L.tagan_geo_attn_fwd_workspace(self.gs, heads, self.d)
        self.fws = torch.empty(max(int(self.fwb), 1), dtype=torch.uint8, device=dev)
        self.wsb = L.tagan_geo_attn_bwd_workspace(self.gs, heads, self.d)
        self.ws = torch.empty(max(int(self.wsb), 1), dtype=torch.uint8, device=dev)
        self.stream = torch.cuda.current_stream(dev)
        self.sp = ctypes.c_void_p(self.stream.cuda_stream)

    def fwd(self):
        from tagan_amd import _lib
        b, es, H = self.qkv.data_ptr(), 4, self.H
        _lib.check(self.L.tagan_geo_attn_fwd(0, self.metric, self.gs, self.heads, self.d, b, b + H * es, b + 2 * H * es,
                                             3 * H, None, self.p, 1234, _lib.ptr(self.out), _lib.ptr(self.lse), None,
                                             _lib.ptr(self.fws), self.fwb, self.sp), "fwd")

    def bwd(self):
        from tagan_amd import _lib
        b, db, es, H = self.qkv.data_ptr(), self.dqkv.data_ptr(), 4, self.H
        _lib.check(self.L.tagan_geo_attn_bwd(0, self.metric, self.gs, self.heads, self.d, b, b + H * es, b + 2 * H * es,
                                             3 * H, None, self.p, 1234, _lib.ptr(self.out), _lib.ptr(self.lse),
                                             _lib.ptr(self.dout), db, db + H * es, db + 2 * H * es, 3 * H, None,
                                             _lib.ptr(self.ws), self.wsb, self.sp), "bwd")

    def time(self, reps):
        """Mean fwd / bwd launch-group durations (s), HIP events on the launch stream, after 2 warm-ups."""
        for _ in range(2):
            self.fwd()
            self.bwd()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tf = tb = 0.0
        for _ in range(reps):
            ev[0].record(self.stream)
            self.fwd()
            ev[1].record(self.stream)
            self.bwd()
            ev[2].record(self.stream)
            ev[2].synchronize()
            tf += ev[0].elapsed_time(ev[1])
            tb += ev[1].elapsed_time(ev[2])
        return tf / reps * 1e-3, tb / reps * 1e-3


def _pmc_traffic(config):
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % config)
    if os.path.exists(pmc):
        with open(pmc) as f:
            return json.load(f).get("hbm_bytes_per_launch_group")
    return None


def roofline_c4(reps=10):
    """The ≥40 %-of-HBM gate configuration: one C4 snapshot, 1M nodes, 20M uniform-random edges
    (worst-case gather locality; Q|K|V = 1.5 GB, far beyond the 256 MB Infinity Cache), H=128, 4 heads, fp32,
    dropout 0.1, euclidean metric."""
    from tagan_amd import synthetic
    from tagan_amd.kernels import build_graph
    dev = torch.device("cuda", torch.cuda.current_device())
    N, E, _T, H, heads = synthetic.CONFIGS["c4"][:5]
    seq = synthetic.make_sequence("c4", dev, seed=4000, snapshots=1)
    graph = build_graph([seq[0][1]], [N])
    del seq
    k = EdgeKernels(graph, H, heads, 0.1)
    tf, tb = k.time(reps)
    bf, bb = geo_bytes(k.E, k.N, H)
    achieved = (bf + bb) / (tf + tb) / 1e9
    traffic = _pmc_traffic("c4")
    rec = {"kernel": "tagan_geo_attn fwd (k_geo_fwd_chunk + k_geo_fwd_merge) + bwd in the column-first order this "
                     "graph takes (k_geo_bwd_delta + k_geo_bwd_col_chunk + k_geo_bwd_row_ds + 2 k_geo_sum_parts): "
                     "edge-softmax + aggregate of one layer, one C4 snapshot",
           "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
           "traffic_source": ("profiles/pmc_c4.json: rocprofv3 --pmc FETCH_SIZE x 2 + WRITE_SIZE of these launches, "
                              "collected by the builder (tools/pmc_summary.py), not measured in this run")
           if traffic else None,
           "algorithmic_bytes": int(bf + bb), "bytes_fwd": int(bf), "bytes_bwd": int(bb),
           "edges": k.E, "nodes": k.N, "H": H, "heads": heads, "dtype": "fp32",
           "ms_fwd": round(tf * 1e3, 4), "ms_bwd": round(tb * 1e3, 4), "reps": reps,
           "formula": "SURVEY 8(d): B_fwd = s*H*(2E'+2N) + 4(E'+N), B_bwd = s*H*(4E'+8N) + 8(E'+N), s = 4",
           "config": "c4 (1M nodes, 20M uniform edges, cache-cold)"}
    if traffic:
        rec["traffic_frac"] = round(traffic / (tf + tb) / 1e9 / HBM_PEAK_GBS, 4)
    del k, graph
    torch.cuda.empty_cache()
    return rec


def temporal_kernels(config, reps=10):
    """The temporal attention kernels alone (forward + backward, HIP events) on a config's [T, N, 3H] time-major
    projection with the folded bias table, its gradient and dropout 0.1 -- the kernel VERDICT r01 named furthest
    below the roofline.  Algorithmic bytes: forward Q, K, V in + O out; backward Q, K, V, dO in + dQ, dK, dV out
    (O is not read: delta comes from P·dP); + the LSE rows."""
    from tagan_amd import _lib, synthetic
    dev = torch.device("cuda", torch.cuda.current_device())
    N, _E, T, H, heads = synthetic.CONFIGS[config][:5]
    d = H // heads
    g = torch.Generator(device=dev).manual_seed(3)
    qkv = torch.randn(T, N, 3 * H, device=dev, generator=g)
    out = torch.empty(T, N, H, device=dev)
    dout = torch.randn(T, N, H, device=dev, generator=g)
    dqkv = torch.empty_like(qkv)
    lse = torch.empty(N, heads, T, device=dev)
    table = torch.randn(heads, 2 * T - 1, device=dev, generator=g) * 0.1
    dtable = torch.empty_like(table)
    L = _lib.lib()
    wsb = L.tagan_temporal_attn_bwd_workspace(N, T, heads, d)
    ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    b, db, es = qkv.data_ptr(), dqkv.data_ptr(), 4
    sr, stt = 3 * H, N * 3 * H

    def fwd():
        _lib.check(L.tagan_temporal_attn_fwd(0, N, T, heads, d, b, b + H * es, b + 2 * H * es, sr, stt,
                                             _lib.ptr(table), None, 0, None, 0, 0, 0, 0.1, 99,
                                             _lib.ptr(out), H, N * H, _lib.ptr(lse), None, sp), "fwd")

    def bwd():
        _lib.check(L.tagan_temporal_attn_bwd(0, N, T, heads, d, b, b + H * es, b + 2 * H * es, sr, stt,
                                             _lib.ptr(table), None, 0, None, 0, 0, 0, 0.1, 99,
                                             _lib.ptr(out), H, N * H, _lib.ptr(lse), _lib.ptr(dout), H, N * H,
                                             db, db + H * es, db + 2 * H * es, sr, stt, _lib.ptr(dtable), None, None,
                                             _lib.ptr(ws), wsb, sp), "bwd")
    for _ in range(2):
        fwd()
        bwd()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(reps):
        ev[0].record(st)
        fwd()
        ev[1].record(st)
        bwd()
        ev[2].record(st)
        ev[2].synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    tf, tb = tf / reps / 1e3, tb / reps / 1e3
    unit = N * T * H * 4
    bf, bb = 4 * unit + N * heads * T * 4, 7 * unit + N * heads * T * 4
    del qkv, out, dout, dqkv, lse, ws
    torch.cuda.empty_cache()
    return {"config": config, "rows": N, "T": T, "heads": heads, "head_dim": d,
            "ms_fwd": round(tf * 1e3, 4), "ms_bwd": round(tb * 1e3, 4),
            "gbs_fwd": round(bf / tf / 1e9, 1), "gbs_bwd": round(bb / tb / 1e9, 1),
            "frac_fwd": round(bf / tf / 1e9 / HBM_PEAK_GBS, 4), "frac_bwd": round(bb / tb / 1e9 / HBM_PEAK_GBS, 4)}


def roofline_cache_assisted(seq, cfg, reps=20):
    """The same launches on the bench's own C2 graph (all 32 snapshots): L2 / Infinity Cache serve part of the
    gathered K|V rows, so algorithmic bytes / time can pass the HBM peak -- an effective bandwidth, not a
    roofline fraction."""
    from tagan_amd.kernels import build_graph
    graph = build_graph([ei for _, ei, _, _ in seq], [int(x.shape[0]) for x, _, _, _ in seq])
    k = EdgeKernels(graph, cfg.hidden_dim, cfg.num_heads, cfg.dropout, 6 if cfg.learnable_distance else 0)
    tf, tb = k.time(reps)
    bf, bb = geo_bytes(k.E, k.N, cfg.hidden_dim)
    eff = (bf + bb) / (tf + tb) / 1e9
    return {"effective_gbs": round(eff, 1), "effective_over_peak": round(eff / HBM_PEAK_GBS, 4),
            "traffic": _pmc_traffic("c2"), "algorithmic_bytes": int(bf + bb), "edges": k.E, "nodes": k.N,
            "ms_fwd": round(tf * 1e3, 4), "ms_bwd": round(tb * 1e3, 4)}


def breakdown(model, seq, fwd, bwd, opt, cfg, reps=5):
    """Per-phase time of one step (CSR build and optimizer reported separately), measured
    after the timed region with HIP events on the current stream, mean of ``reps`` (all ranks in lockstep)."""
    from tagan_amd.kernels import build_graph
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    acc = [0.0] * 4
    eis = [ei for _, ei, _, _ in seq]
    counts = [int(x.shape[0]) for x, _, _, _ in seq]
    for _ in range(reps):
        opt.zero_grad(set_to_none=True)
        ev[0].record(stream)
        build_graph(eis, counts)
        ev[1].record(stream)
        out = fwd()
        ev[2].record(stream)
        bwd(out)
        ev[3].record(stream)
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.gradient_clip_val)
        opt.step()
        ev[4].record(stream)
        ev[4].synchronize()
        for i in range(4):
            acc[i] += ev[i].elapsed_time(ev[i + 1])
    names = ("csr_build_ms", "forward_ms", "backward_ms", "optimizer_ms")
    res = {n: round(a / reps, 3) for n, a in zip(names, acc)}
    res["note"] = ("forward includes its own CSR build; backward includes the gradient exchange; "
                   "optimizer = clip_grad_norm_ + Adam")
    return res


def _host_cores():
    """Threads for the CPU legs: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the pool) or the affinity
    mask, whichever is smaller; plus what the host reports (nproc, CPU model) for the record."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(aff, omp) if omp > 0 else aff
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return threads, {"nproc": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": omp or None,
                     "cpu_model": model}


def _oracle_rate(P, c, seq, lab, mode, min_seconds, max_reps=1000):
    import oracle
    n = len(seq)
    done, t0 = 0, time.perf_counter()
    reps = 0
    while True:
        out = oracle.tagan_forward(P, c, seq, lab, mode=mode)
        out["loss"].backward()
        done += n
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= min_seconds or reps >= max_reps:
            return done / dt, done, dt


DF_SWEEP_N = (250, 500, 1000)


def dense_faithful_sweep(P, c, name, lab, nodes=DF_SWEEP_N, snapshots=1, reps=2):
    """The reference's own algorithm (oracle ``dense_faithful``: dense N×N mask, per-(head, node) distance loop,
    geometric_attention.py:386-401) on ``name``-shaped sequences at small N (E = 10 N, ``snapshots`` snapshots,
    fwd+bwd, best of ``reps``: single runs of this loop-heavy path see occasional 2-3x host stalls), and the power
    law t = a·N^p fitted to the per-snapshot times (the loop's backward is ≈N³, so a whole C2 snapshot, ≈3 h, is
    out of reach).  Returns ([(N, seconds per snapshot)], p, a)."""
    import math
    import oracle
    from tagan_amd import synthetic
    pts = []
    for n in nodes:
        seq = synthetic.make_sequence(name, "cpu", seed=7, snapshots=snapshots, nodes=n, edges=10 * n)
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            oracle.tagan_forward(P, c, seq, lab, mode="dense_faithful")["loss"].backward()
            best = min(best, time.perf_counter() - t0)
        pts.append((n, best / snapshots))
    xs = [math.log(n) for n, _ in pts]
    ys = [math.log(t) for _, t in pts]
    mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
    p = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a = math.exp(my - p * mx)
    return pts, p, a


def cpu_baseline(cfg, name, model_state, n_snap, gpu_c1=None, gpu_value=None, min_seconds=8.0):
    """CPU oracle on bounded samples of the workloads, fwd+bwd (no optimizer), fp32, on the host's cores:

    * ``value``: sparse CSR restatement on ``n_snap``-snapshot sequences of the bench's own config (C2) — the
      strong CPU baseline of the headline;
    * ``c1.dense_faithful``: the reference's own algorithm and cost model (dense N×N mask, per-(head, node)
      distance loop; geometric_attention.py:386-401, graph_attention.py:96-105) on one whole C1 sequence —
      matched to the literal reference within 10 % in this container (profiles/r2_cpu_crosscheck.json);
    * ``c1.sparse``: the sparse restatement on the same C1 sequence.
    """
    from tagan_amd import synthetic
    threads, host = _host_cores()
    torch.set_num_threads(threads)
    lab = torch.tensor([1.0])
    seq = synthetic.make_sequence(name, "cpu", seed=42, snapshots=n_snap)
    P = {k: v.detach().cpu().clone().requires_grad_(v.is_floating_point()) for k, v in model_state.items()}
    c = cfg.to_dict()
    small = synthetic.make_sequence(name, "cpu", seed=1, snapshots=1, nodes=500, edges=2000)
    import oracle
    oracle.tagan_forward(P, c, small, lab)["loss"].backward()            # warm-up
    rate, done, dt = _oracle_rate(P, c, seq, lab, "sparse", min_seconds)
    rec = {"value": round(rate, 4), "unit": "graph-snapshots/s", "cores": threads, "kind": "port",
           "sample": "oracle sparse-CSR restatement, fwd+bwd (no optimizer), %s shape, %d-snapshot sequences "
                     "x %d (%d snapshots) in %.1f s, fp32, %d threads" % (name, n_snap, done // n_snap, done, dt, threads),
           "host": host}
    if gpu_value:
        rec["gpu_over_cpu"] = round(gpu_value / rate, 1)
    # the headline config against the reference's own algorithm: measured at small N, extrapolated to the config's N
    pts, p, a = dense_faithful_sweep(P, c, name, lab)
    n_full = synthetic.CONFIGS[name][0]
    df_ext = 1.0 / (a * n_full ** p)
    rec["dense_faithful"] = {
        "value": float("%.3g" % df_ext), "unit": "graph-snapshots/s", "kind": "port", "extrapolated": True,
        "sample": "oracle dense_faithful (the reference's dense N×N per-(head, node) loop), fwd+bwd, %s shape with "
                  "N = %s, E = 10 N, one snapshot each (best of 2), %d threads; t = a·N^p fitted (p = %.2f) and extrapolated to "
                  "N = %d: an upper bound on the CPU rate (the loop's ≈N³ backward takes over above N ≈ 1000, BASELINE.md, "
                  "so the true exponent at C2 is larger)" % (name, "/".join(str(n) for n, _ in pts), threads, p, n_full),
        "sweep_s_per_snapshot": {str(n): round(t, 3) for n, t in pts},
        "fit_exponent": round(p, 3)}
    if gpu_value:
        rec["gpu_over_dense_faithful"] = float("%.3g" % (gpu_value / df_ext))
    # C1: the reference's own configuration (example.py), the only one the literal reference runs in full
    c1cfg = synthetic.config_for("c1")
    torch.manual_seed(0)
    from tagan_amd import TAGAN
    m1 = TAGAN(c1cfg)
    P1 = {k: v.detach().clone().requires_grad_(v.is_floating_point()) for k, v in m1.state_dict().items()}
    seq1 = synthetic.make_sequence("c1", "cpu", seed=42)
    c1 = c1cfg.to_dict()
    oracle.tagan_forward(P1, c1, seq1[:2], lab, mode="dense_faithful")["loss"].backward()   # warm-up
    df_rate, df_done, df_dt = _oracle_rate(P1, c1, seq1, lab, "dense_faithful", 0.0, max_reps=1)
    sp_rate, sp_done, sp_dt = _oracle_rate(P1, c1, seq1, lab, "sparse", 2.0)
    c1rec = {"dense_faithful": {"value": round(df_rate, 4), "unit": "graph-snapshots/s", "kind": "port",
                                "sample": "one C1 sequence (10 snapshots of 500 nodes) in %.1f s" % df_dt},
             "sparse": {"value": round(sp_rate, 4), "unit": "graph-snapshots/s", "kind": "port",
                        "sample": "%d C1 sequences in %.1f s" % (sp_done // 10, sp_dt)},
             "literal_reference_crosscheck": "profiles/r2_cpu_crosscheck.json (container, 8 threads)"}
    if gpu_c1:
        c1rec["gpu"] = gpu_c1
        c1rec["gpu_over_dense_faithful"] = round(gpu_c1["value"] / df_rate, 1)
        c1rec["gpu_over_sparse"] = round(gpu_c1["value"] / sp_rate, 1)
    rec["c1"] = c1rec
    return rec


def make_step(model, opt, cfg, fwd, bwd):
    def step():
        opt.zero_grad(set_to_none=True)
        out = fwd()
        bwd(out)
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.gradient_clip_val)
        opt.step()
        return out["loss"]
    return step


def graphed(model, opt, cfg, fwd, exchange=None, warmup=3):
    """The bench step as ONE replayable HIP graph (graph_step.GraphedStep): forward, backward, the gradient
    exchange (N > 1: ``exchange()`` = the static RCCL bucket all-reduce, captured into the same graph), clip, Adam."""
    from tagan_amd.graph_step import GraphedStep

    def whole():
        out = fwd()
        out["loss"].backward()
        if exchange is not None:
            exchange()
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.gradient_clip_val)
        opt.step()
        return out["loss"]
    return GraphedStep(model, whole, optimizer=opt, warmup=warmup)


def gpu_c1_line(dev, precision, steps=20, warmup=5, graph=True):
    """The same training step on C1 (example.py: 500 nodes, 1000 edges, 10 snapshots, H=64, 4 heads) on this GPU,
    beside the C1 CPU baselines (host-launch-bound at this size)."""
    from tagan_amd import TAGAN, synthetic
    cfg = synthetic.config_for("c1")
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=precision).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay, capturable=graph,
                           fused=True)
    seq = synthetic.make_sequence("c1", dev, seed=1000)
    labels = torch.tensor([1.0], device=dev)
    step = make_step(model, opt, cfg, lambda: model(seq, labels=labels), lambda out: out["loss"].backward())
    g = graphed(model, opt, cfg, lambda: model(seq, labels=labels)) if graph else None
    if g is not None:
        step = g
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    T = len(seq)
    if g is not None:
        g.close()
    return {"value": round(T * steps / el, 3), "unit": "graph-snapshots/s", "ms_per_step": round(el / steps * 1e3, 3),
            "steps": steps, "dtype": precision, "launch": "hip-graph" if graph else "eager"}


EXCHANGE_PHASES = ("grad_allreduce", "all_to_all", "pool_allreduce")


def sub_record(workload, step, world, group=None, steps=5, warmup=3, snapshots_per_step=1, extra=None):
    """One measured multi-GPU sub-record of the bench line (DESIGN.md §4 'sub-records'): ``warmup`` untimed calls
    of ``step``, then ``steps`` timed ones between two barriers + device syncs on ``group`` (a gloo group of host
    tensors), wall time = the MAX over ranks; the collectives inside the step are timed per phase by
    ``distributed.ExchangeTimer`` (HIP events around each call on the current stream; wall clock for host
    tensors) and reported per step, each phase its MAX over ranks.  Runs on CPU too (gloo tests)."""
    from tagan_amd import distributed as D
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    timer = D.ExchangeTimer()
    D.TIMER = timer
    try:
        for _ in range(warmup):
            step()
        sync()
        if world > 1:
            dist.barrier(group=group)
        timer.reset()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        sync()
        if world > 1:
            dist.barrier(group=group)
        el = time.perf_counter() - t0
        tot = timer.totals()
    finally:
        D.TIMER = None
    vals = torch.tensor([el] + [tot.get(k, 0.0) for k in EXCHANGE_PHASES], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(vals, dist.ReduceOp.MAX, group=group)
    el = float(vals[0])
    rec = {"workload": workload, "value": round(snapshots_per_step * steps / el, 3), "unit": "graph-snapshots/s",
           "ms_per_step": round(el / steps * 1e3, 3), "steps": steps, "warmup": warmup, "n_ranks": world,
           "exchange_ms_per_step": {k: round(float(v) / steps, 4) for k, v in zip(EXCHANGE_PHASES, vals[1:].tolist())
                                    if tot.get(k) is not None or float(v) > 0}}
    if extra:
        rec.update(extra)
    return rec


def sub_records_for(spec, world):
    """``--sub-records``: "auto" = c3_dp at N in {2, 4} (BASELINE configs[2]: "snapshot-batch DP over 2 then 4
    GPUs"), c5_shard at N = 8 (configs[4]: "8x snapshot-sharded ... scaling-curve config"); "none"; or a comma
    list of c3_dp / c5_shard (any N, e.g. a one-GPU rehearsal of the code path)."""
    spec = (spec or "auto").strip().lower()
    if spec == "none":
        return []
    if spec == "auto":
        return ["c3_dp"] if world in (2, 4) else (["c5_shard"] if world == 8 else [])
    out = [x.strip() for x in spec.split(",") if x.strip()]
    bad = [x for x in out if x not in ("c3_dp", "c5_shard")]
    if bad:
        raise SystemExit("bench.py: unknown sub-record(s) %s" % bad)
    return out


def c3_dp_record(dev, rank, world, ctl, backend, steps=5, warmup=3):
    """BASELINE configs[2] at N ranks: 100k nodes / 2M edges per snapshot, 64 snapshots, hidden 256, 8 heads, fp32,
    one sequence per rank (snapshot-batch data parallel), the flagged gradient bucket over RCCL; eager launches
    (a 0.6-s step: launch overhead is noise, and a captured graph would double the 195-GB working set)."""
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.distributed import GradBucket, broadcast_parameters
    cfg = synthetic.config_for("c3")
    torch.manual_seed(0)
    model = TAGAN(cfg).to(dev).train()
    broadcast_parameters(model)
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay, fused=True)
    seq = synthetic.make_sequence("c3", dev, seed=2000 + rank)
    labels = torch.tensor([1.0 if rank % 2 == 0 else 0.0], device=dev)
    bucket = GradBucket(model.parameters())

    def bwd(out):
        out["loss"].backward()
        bucket.allreduce_mean()
    step = make_step(model, opt, cfg, lambda: model(seq, labels=labels), bwd)
    N, E, T, H, heads = synthetic.CONFIGS["c3"][:5]
    rec = sub_record("c3 (BASELINE configs[2]): %d nodes, %d edges/snapshot, %d snapshots, hidden %d, %d heads, fp32, "
                     "one sequence per rank" % (N, E, T, H, heads), step, world, ctl, steps, warmup, T * world,
                     {"parallelism": "dp%d" % world, "scaling": "weak", "launch": "eager", "dtype": "fp32",
                      "n_ranks_rccl": world if backend == "nccl" else 0,
                      "grad_bucket_mb": round(4 * (bucket.n + len(bucket.params)) / 1e6, 3)})
    rec["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    return rec


def c5_shard_record(dev, rank, world, ctl, backend, steps=5, warmup=3, nodes=None, edges=None):
    """BASELINE configs[4] over N ranks: ONE sequence of 128 snapshots (100k nodes / 2M edges each, hidden 256,
    16 heads, fp32) sharded by snapshot (sharded.py): the geometric stage on each rank's 128/N snapshots, one
    all-to-all to node rows, the temporal stage on the rank's rows, one pooling all-reduce, one gradient
    all-reduce.  ``nodes`` / ``edges`` shrink the snapshots (same T, H, heads) for a rehearsal of several ranks on
    one GPU (tests/test_gpu_sharded.py, ``--c5-shard-size``).  Launch: the whole sharded step captured as one HIP
    graph (the all-to-all, the pooling all-reduce and the static gradient sync inside it,
    tests/test_gpu_rccl.py::test_rccl_world1_graph_step_sharded) when the data plane can be captured (RCCL, or one
    rank) and the eager step's peak memory leaves room for the graph's own pool (under 45 % of the device: the full
    C5 share at N = 8 is ~240 GB and runs eagerly); a short trial of both then keeps the faster."""
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.distributed import broadcast_parameters
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
    cfg = synthetic.config_for("c5")
    N, E, T, H, heads = synthetic.CONFIGS["c5"][:5]
    N, E = nodes or N, edges or E
    torch.manual_seed(0)
    model = TAGAN(cfg).to(dev).train()
    broadcast_parameters(model)
    can_graph = world == 1 or backend == "nccl"   # the data plane can be captured (see the docstring)
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay,
                           capturable=can_graph, fused=True)
    t0, t1 = blocks(T, world)[rank]
    full = synthetic.make_sequence("c5", dev, seed=5000, nodes=N, edges=E)   # the same sequence on every rank
    seq = synthetic.take(full, t0, t1)
    del full
    counts_all = [N] * T
    sharded = SnapshotShardedTAGAN.for_model(model)
    sync = ShardGradSync(list(model.named_parameters()))
    labels = torch.tensor([1.0], device=dev)

    def bwd(out):
        out["loss"].backward()
        sync.sync()
    step = make_step(model, opt, cfg, lambda: sharded(seq, counts_all, labels), bwd)
    launch, trial_ms, gstep = "eager", None, None
    if can_graph:
        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
        peak = torch.cuda.max_memory_allocated(dev)
        fits = torch.tensor([1.0 if peak < 0.45 * torch.cuda.get_device_properties(dev).total_memory else 0.0])
        if world > 1:
            dist.all_reduce(fits, dist.ReduceOp.MIN, group=ctl)
        if float(fits) > 0:
            def t(fn, n=3):
                fn()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(n):
                    fn()
                torch.cuda.synchronize(dev)
                x = torch.tensor([(time.perf_counter() - t0) / n], dtype=torch.float64)
                if world > 1:
                    dist.all_reduce(x, dist.ReduceOp.MAX, group=ctl)
                return float(x)
            te = t(step)
            torch.cuda.empty_cache()
            gstep = graphed(model, opt, cfg, lambda: sharded(seq, counts_all, labels),
                            (lambda: sync.sync(static=True)) if world > 1 else None)
            tg = t(gstep)
            trial_ms = {"graph_ms": round(tg * 1e3, 3), "eager_ms": round(te * 1e3, 3)}
            if tg < te:
                launch, step = "hip-graph", gstep
            else:
                gstep.close()
                gstep = None
    rec = sub_record("c5 (BASELINE configs[4]): one sequence of %d snapshots (%d nodes, %d edges each), hidden %d, "
                     "%d heads, fp32, sharded by snapshot over %d ranks" % (T, N, E, H, heads, world),
                     step, world, ctl, steps, warmup, T,
                     {"parallelism": "snapshot-shard%d" % world, "scaling": "strong", "launch": launch,
                      "dtype": "fp32", "n_ranks_rccl": world if backend == "nccl" else 0})
    if trial_ms:
        rec["launch_trial"] = trial_ms
    rec["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    if gstep is not None:
        gstep.close()
    return rec


def _relaunch(n):
    """``--gpus N`` outside torchrun: run this script under torch.distributed.run with N ranks (no GPU call has
    happened in this process) and exit with its status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_relaunch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    # rehearsal knobs (never set by the driver): TAGAN_BENCH_BACKEND=gloo + TAGAN_BENCH_DEVICE=0 run the N-rank data-
    # parallel flow with every rank on one GPU (RCCL refuses two ranks per device), e.g. on a one-GPU box
    backend = os.environ.get("TAGAN_BENCH_BACKEND", "nccl")
    if os.environ.get("TAGAN_BENCH_DEVICE"):
        local = int(os.environ["TAGAN_BENCH_DEVICE"])
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        from tagan_amd.distributed import init_process_group   # RCCL event recycling off (graph capture)
        if backend == "nccl":
            init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            init_process_group(backend)
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import tagan_amd
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.distributed import GradBucket, all_reduce_, broadcast_parameters
    from tagan_amd.gemm_tuning import use_tuned_gemms
    if args.roofline_only:
        print(json.dumps({"roofline": roofline_c4(args.roofline_reps)}), flush=True)
        return
    gemm_table = None if args.no_tuned_gemms else use_tuned_gemms(args.gemm_table, tune=args.tune_gemms)
    os.environ["TAGAN_BENCH_CONFIG"] = args.config
    cfg = synthetic.config_for(args.config)
    N, E, T, H, heads = synthetic.CONFIGS[args.config][:5]
    # control plane (N > 1): timing maxima and the barriers around the timed region go over a gloo group of host
    # tensors, so no eager device work sits between two replays of the step graph
    ctl = dist.new_group(backend="gloo") if world > 1 else None
    # every form of the step is captured whole (the RCCL all-reduce inside the graph); only a gloo data plane
    # (the one-GPU rehearsal knob) cannot be captured and launches eagerly
    capturable = world == 1 or backend == "nccl"
    # --shard captures too: the all-to-all, the pooling all-reduce and the static gradient sync are graph-safe
    # (tests/test_gpu_rccl.py::test_rccl_world1_graph_step_sharded)
    launch = "eager" if (args.no_graph or not capturable) else args.launch
    use_graph = launch != "eager"   # capturable optimizer whenever a graph may be captured
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=args.precision).to(dev).train()
    broadcast_parameters(model)
    # the reference trainer's Adam (trainer.py); fused=True: the same update as ONE multi-tensor kernel
    # (capturable into the step graph), instead of ~15 foreach launches
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay,
                           capturable=use_graph, fused=True)
    init_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    if args.shard:
        from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
        full = synthetic.make_sequence(args.config, dev, seed=1000)
        counts_all = [int(x.shape[0]) for x, _, _, _ in full]
        t0, t1 = blocks(len(full), world)[rank]
        seq = synthetic.take(full, t0, t1)
        del full
        sharded = SnapshotShardedTAGAN.for_model(model)
        sync = ShardGradSync(list(model.named_parameters()))
        labels = torch.tensor([1.0], device=dev)

        def fwd():
            return sharded(seq, counts_all, labels)

        def bwd(out):
            out["loss"].backward()
            sync.sync()

        def exchange():
            sync.sync(static=True)
    else:
        bucket = GradBucket(model.parameters())
        seq = synthetic.make_sequence(args.config, dev, seed=1000 + rank)
        labels = torch.tensor([1.0 if rank % 2 == 0 else 0.0], device=dev)

        def fwd():
            return model(seq, labels=labels)

        def bwd(out):
            out["loss"].backward()
            bucket.allreduce_mean()

        def exchange():
            bucket.allreduce_mean(static=True)

    step = make_step(model, opt, cfg, fwd, bwd)
    eager_step = step

    def host_max(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, dist.ReduceOp.MAX, group=ctl)
        return float(t.item())

    def trial(fn, n=5):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return host_max(time.perf_counter() - t0) / n   # every rank takes the same decision

    launch_trial = None
    gstep = None
    if use_graph:
        # eager trial first, then ONE capture that is kept when it wins (no capture / destroy / re-capture)
        te = trial(eager_step) if launch == "auto" else None
        gstep = graphed(model, opt, cfg, fwd, exchange if world > 1 else None)
        if launch == "auto":
            tg = trial(gstep)
            launch_trial = {"graph_ms": round(tg * 1e3, 3), "eager_ms": round(te * 1e3, 3)}
            if tg >= te:
                gstep.close()
                gstep = None
    if gstep is not None:
        step = gstep

    def timed(steps, warmup):
        """W untimed steps, then exactly K steps between barrier + sync; max over ranks."""
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier(group=ctl)
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier(group=ctl)
        el = host_max(time.perf_counter() - t0)
        assert torch.isfinite(loss).item(), "non-finite loss"
        return el

    elapsed = timed(args.steps, args.warmup)

    seqs_per_step = 1 if args.shard else world
    value = seqs_per_step * T * args.steps / elapsed
    rec = {
        "metric": "graph-snapshots/sec (fwd+bwd) at 1/2/4/8 MI355X; achieved HBM GB/s vs peak",
        "value": round(value, 3), "unit": "graph-snapshots/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong" if args.shard else "weak", "vs_baseline": None,
        "dtype": {"fp32": "fp32", "bf16-gemm": "fp32 (bf16 GEMM operands, fp32 accumulate)",
                  "bf16": "bf16 (activations; fp32 math and accumulation)"}[args.precision],
        "data": "synthetic (seeded social-media-shaped temporal graph per rank; no dataset offline)",
        "config": {"workload": "%s: %d nodes, %d edges/snapshot, %d snapshots, hidden %d, %d heads, euclidean "
                               "metric, dropout %.1f, train step = fwd+bwd+clip+Adam"
                               % (args.config, N, E, T, H, heads, cfg.dropout),
                   "sequences_per_step": seqs_per_step, "snapshots_per_sequence": T,
                   "parallelism": ("snapshot-shard%d" % world) if args.shard else ("dp%d" % world)},
        "backend": ("nccl (RCCL over xGMI)" if backend == "nccl" else backend) if world > 1 else "none (single rank)",
        "n_ranks_rccl": world if (world > 1 and backend == "nccl") else 0,
        "parallelism": ("snapshot-shard%d" % world) if args.shard else ("dp%d" % world),
    }
    rec["config"]["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    from tagan_amd import fused as _fused
    lib_gemms = ("hipBLASLt/rocBLAS solutions from the TunableOp table %s" % os.path.basename(gemm_table)
                 if gemm_table else "library-default heuristic")
    if _fused._sg_use(H, args.precision != "fp32", args.precision == "bf16"):
        lib_gemms = ("attention-block projections: hand-written bf16-matrix-core kernels (csrc/stream_gemm.hip; "
                     "fp32 mode as three bf16 planes, six plane products, fp32 accumulate; the N = 128 products on "
                     "row-owner kernels; LN1 fused into the QKV projection's prologue, dropout + residual + LN2 into "
                     "the out-projection's epilogue, in bf16 mode also LN1's backward into the QKV input gradient's "
                     "epilogue); node embedding: exact-f32 matrix-core kernels (csrc/narrow.hip, weight and bias "
                     "gradients in one pass); head and GRU GEMMs: " + lib_gemms)
    rec["config"]["gemms"] = lib_gemms
    rec["launch"] = (("hip-graph (one replay per step)" if world == 1 else
                      "hip-graph (one replay per step; the RCCL gradient all-reduce captured inside it)")
                     if gstep is not None else "eager")
    if launch_trial:
        rec["launch_trial"] = dict(launch_trial, note="5-step trial of both launch modes; the faster one is timed")
    if gstep is not None:
        gstep.close()
        step = make_step(model, opt, cfg, fwd, bwd)
    rec["breakdown"] = breakdown(model, seq, fwd, bwd, opt, cfg)
    if args.precision == "fp32" and not args.no_alt_precision:
        # the same step with bf16 activations between kernels (BASELINE's C2 dtype), fp32 math inside
        # every kernel; held to the fp64 oracle at the full C2 workload by
        # tests/test_gpu_fullsize.py::test_c2_bf16_vs_oracle (per-tensor normwise bf16 bound)
        model.precision = "bf16"
        te = trial(eager_step) if (use_graph and launch == "auto") else None
        gstep = graphed(model, opt, cfg, fwd, exchange if world > 1 else None) if use_graph else None
        if gstep is not None and launch == "auto":
            tg = trial(gstep)
            if tg >= te:
                gstep.close()
                gstep = None
            alt_launch = {"graph_ms": round(tg * 1e3, 3), "eager_ms": round(te * 1e3, 3)}
        else:
            alt_launch = None
        if gstep is not None:
            step = gstep
        alt = timed(args.steps, args.warmup)
        if gstep is not None:
            gstep.close()
            step = make_step(model, opt, cfg, fwd, bwd)
        model.precision = args.precision
        rec["alt_precision"] = {"precision": "bf16", "value": round(seqs_per_step * T * args.steps / alt, 3),
                                "ms_per_step": round(alt / args.steps * 1e3, 3),
                                "launch": "hip-graph" if gstep is not None else "eager", "launch_trial": alt_launch,
                                "dtype": "bf16 (activations; fp32 math and accumulation)",
                                "parity": "tests/test_gpu_fullsize.py::test_c2_bf16_vs_oracle (full C2 workload vs the "
                                          "fp64 oracle, per-tensor normwise bf16-rounding bound, DESIGN.md section 5)"}
    subs = sub_records_for(args.sub_records, world)
    if subs:
        # BASELINE's multi-GPU workloads beside the C2 headline (DESIGN.md §4 'sub-records'): every rank takes part
        if gstep is not None:
            gstep.close()
        step = gstep = None
        torch.cuda.empty_cache()
        for name in subs:
            fn = {"c3_dp": c3_dp_record, "c5_shard": c5_shard_record}[name]
            kw = {}
            if name == "c5_shard" and args.c5_shard_size:
                kw = dict(zip(("nodes", "edges"), (int(x) for x in args.c5_shard_size.split(","))))
            rec[name] = fn(dev, rank, world, ctl, backend, **kw)
            torch.cuda.empty_cache()
    if rank == 0 and not args.no_roofline:
        roof = roofline_c4(args.roofline_reps)
        roof["cache_assisted"] = dict(roofline_cache_assisted(seq, cfg), config=args.config)
        rec["roofline"] = roof
        # the temporal kernels: C4 (v6 head-group slabs) and C2 (v6 forward, v4 backward: 64-B per-head slices,
        # at the bandwidth that access pattern allows)
        rec["temporal_kernels"] = [temporal_kernels("c4"), temporal_kernels("c2")]
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        c1 = None if args.no_c1 else gpu_c1_line(dev, args.precision, graph=launch != "eager")
        rec["cpu_baseline"] = cpu_baseline(cfg, args.config, init_state, args.cpu_sample_snapshots, gpu_c1=c1,
                                           gpu_value=value)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        # every graph that captured a collective is closed (GraphedStep.close resets it) before the process group
        # is destroyed: the order tests/test_gpu_rccl.py's graph cases run
        if gstep is not None:
            gstep.close()
        dist.barrier(group=ctl)
        torch.cuda.synchronize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
