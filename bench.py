"""TAGAN training-step benchmark on MI355X (graph-snapshots/s, fwd+bwd+optimizer).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]
  (N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N ... bench.py --gpus N)

One step = one TAGAN sequence (all T snapshots) per rank: forward, BCE loss,
backward, gradient all-reduce (N>1, RCCL), clip_grad_norm_(1.0), Adam step —
the reference trainer's step (trainer.py:295-311).  Inputs are synthetic, seeded
per rank and resident in HBM before timing; the snapshot CSR is rebuilt inside
every step.  Prints ONE JSON line on rank 0.

roofline: the edge-softmax + aggregate kernels (tagan_geo_attn fwd, bwd-row,
bwd-col) re-launched on the benchmark's own graph and Q/K/V, timed with HIP
events on the launch stream; achieved = algorithmic bytes ÷
time, peak = 8.0 TB/s.  cpu_baseline: the CPU oracle (oracle/, sparse CSR
restatement of the reference algorithm) on a bounded sample, rank 0, N=1 only.
"""
import argparse
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
    ap.add_argument("--shard", action="store_true",
                    help="one sequence sharded by snapshot over all ranks (strong scaling; C5 mode) instead of "
                         "one sequence per rank (data parallel, weak scaling)")
    return ap.parse_args()


def geo_bytes(E, N, H, heads, s=4):
    """Algorithmic HBM bytes of one geometric-attention layer pass (fwd, bwd) over N nodes / E CSR entries."""
    fwd = s * H * (2 * E + 2 * N) + 4 * (E + N) + 4 * heads * N
    bwd_row = s * H * (2 * E + 4 * N) + 4 * (E + N) + 8 * heads * N
    bwd_col = s * H * (2 * E + 4 * N) + 8 * E + 4 * N + 8 * heads * E
    return fwd, bwd_row + bwd_col


def roofline(model, seq, cfg, reps=20):
    """Time the three edge kernels on the benchmark graph with HIP events on the launch stream."""
    import ctypes
    import tagan_amd
    from tagan_amd import _lib
    from tagan_amd.kernels import build_graph
    dev = seq[0][0].device
    counts = [int(x.shape[0]) for x, _, _, _ in seq]
    graph = build_graph([ei for _, ei, _, _ in seq], counts)
    N, H, heads = graph.num_nodes, cfg.hidden_dim, cfg.num_heads
    d = H // heads
    E = graph.nnz_host()
    g = torch.Generator(device=dev).manual_seed(7)
    qkv = torch.randn(N, 3 * H, device=dev, generator=g)
    dout = torch.randn(N, H, device=dev, generator=g)
    out = torch.empty(N, H, device=dev)
    lse = torch.empty(N, heads, device=dev)
    dqkv = torch.empty_like(qkv)
    L = _lib.lib()
    gs = graph.struct()
    fwb = L.tagan_geo_attn_fwd_workspace(gs, heads, d)
    fws = torch.empty(max(int(fwb), 1), dtype=torch.uint8, device=dev)
    wsb = L.tagan_geo_attn_bwd_workspace(gs, heads, d)
    ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)
    b, es = qkv.data_ptr(), 4
    db = dqkv.data_ptr()
    metric = 6 if cfg.learnable_distance else 0
    p = float(cfg.dropout)

    def fwd():
        _lib.check(L.tagan_geo_attn_fwd(0, metric, gs, heads, d, b, b + H * es, b + 2 * H * es, 3 * H, None, p,
                                        1234, _lib.ptr(out), _lib.ptr(lse), None, _lib.ptr(fws), fwb, sp), "fwd")

    def bwd():
        _lib.check(L.tagan_geo_attn_bwd(0, metric, gs, heads, d, b, b + H * es, b + 2 * H * es, 3 * H, None, p,
                                        1234, _lib.ptr(out), _lib.ptr(lse), _lib.ptr(dout), db, db + H * es,
                                        db + 2 * H * es, 3 * H, None, _lib.ptr(ws), wsb, sp), "bwd")

    for _ in range(3):
        fwd()
        bwd()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(reps):
        ev[0].record(stream)
        fwd()
        ev[1].record(stream)
        bwd()
        ev[2].record(stream)
        ev[2].synchronize()
        tf += ev[0].elapsed_time(ev[1])
        tb += ev[1].elapsed_time(ev[2])
    tf, tb = tf / reps * 1e-3, tb / reps * 1e-3
    bf, bb = geo_bytes(E, N, H, heads)
    achieved = (bf + bb) / (tf + tb) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % os.environ.get("TAGAN_BENCH_CONFIG", "c2"))
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch_group")
    return {"kernel": "tagan_geo_attn fwd+bwd_row+bwd_col (edge-softmax + aggregate, one layer)",
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes": int(bf + bb), "edges": E, "nodes": N,
            "ms_fwd": round(tf * 1e3, 4), "ms_bwd": round(tb * 1e3, 4),
            "note": "achieved = algorithmic bytes / kernel time; at C2 the L2 and Infinity Cache serve part of "
                    "the gathered K|V rows (traffic = PMC HBM bytes), so achieved can pass the HBM peak; C4 is "
                    "the cache-cold case (DESIGN.md section 4)"}


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


def cpu_baseline(cfg, name, model_state, n_snap, min_seconds=10.0):
    """CPU oracle (sparse CSR restatement of the reference) on a bounded sample of the same workload:
    whole sequences of ``n_snap`` snapshots, fwd+bwd, repeated until ``min_seconds`` of CPU work."""
    import oracle
    from tagan_amd import synthetic
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    seq = synthetic.make_sequence(name, "cpu", seed=42, snapshots=n_snap)
    P = {k: v.detach().cpu().clone().requires_grad_(v.is_floating_point()) for k, v in model_state.items()}
    c = cfg.to_dict()
    lab = torch.tensor([1.0])
    small = synthetic.make_sequence(name, "cpu", seed=1, snapshots=1, nodes=500, edges=2000)
    oracle.tagan_forward(P, c, small, lab)["loss"].backward()            # warm-up
    done, t0 = 0, time.perf_counter()
    while True:
        out = oracle.tagan_forward(P, c, seq, lab)
        out["loss"].backward()
        done += n_snap
        dt = time.perf_counter() - t0
        if dt >= min_seconds:
            break
    return {"value": round(done / dt, 4), "unit": "graph-snapshots/s", "cores": threads, "kind": "port",
            "sample": "oracle sparse-CSR restatement, fwd+bwd (no optimizer), %s shape, %d-snapshot sequences "
                      "x %d (%d snapshots) in %.1f s, fp32" % (name, n_snap, done // n_snap, done, dt)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    import tagan_amd
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.distributed import GradBucket, broadcast_parameters
    from tagan_amd.gemm_tuning import use_tuned_gemms
    gemm_table = None if args.no_tuned_gemms else use_tuned_gemms(args.gemm_table, tune=args.tune_gemms)
    os.environ["TAGAN_BENCH_CONFIG"] = args.config
    cfg = synthetic.config_for(args.config)
    N, E, T, H, heads = synthetic.CONFIGS[args.config][:5]
    torch.manual_seed(0)
    model = TAGAN(cfg, precision=args.precision).to(dev).train()
    broadcast_parameters(model)
    opt = torch.optim.Adam(model.parameters(), lr=cfg.learning_rate, weight_decay=cfg.weight_decay)
    init_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    if args.shard:
        from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, blocks
        full = synthetic.make_sequence(args.config, dev, seed=1000)
        counts_all = [int(x.shape[0]) for x, _, _, _ in full]
        t0, t1 = blocks(len(full), world)[rank]
        seq = full[t0:t1]
        del full
        sharded = SnapshotShardedTAGAN.for_model(model)
        sync = ShardGradSync(list(model.named_parameters()))
        labels = torch.tensor([1.0], device=dev)

        def fwd():
            return sharded(seq, counts_all, labels)

        def bwd(out):
            out["loss"].backward()
            sync.sync()
    else:
        bucket = GradBucket(model.parameters())
        seq = synthetic.make_sequence(args.config, dev, seed=1000 + rank)
        labels = torch.tensor([1.0 if rank % 2 == 0 else 0.0], device=dev)

        def fwd():
            return model(seq, labels=labels)

        def bwd(out):
            out["loss"].backward()
            bucket.allreduce_mean()

    def forward_backward():
        out = fwd()
        bwd(out)
        return out

    def step():
        opt.zero_grad(set_to_none=True)
        out = forward_backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), cfg.gradient_clip_val)
        opt.step()
        return out["loss"]

    def timed(steps, warmup):
        """W untimed steps, then exactly K steps between barrier + sync; max over ranks."""
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
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
    }
    rec["config"]["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
    rec["config"]["gemms"] = ("hipBLASLt/rocBLAS solutions from the TunableOp table %s" % os.path.basename(gemm_table)
                              if gemm_table else "library-default heuristic")
    rec["breakdown"] = breakdown(model, seq, fwd, bwd, opt, cfg)
    if args.precision == "fp32" and not args.no_alt_precision:
        # the same step with bf16 activations between kernels (BASELINE's C2 dtype), fp32 math inside
        # every kernel; held to the fp32 mode by tests/test_gpu_bf16.py (loss 2e-2, gradients 8e-2)
        model.precision = "bf16"
        alt = timed(args.steps, args.warmup)
        model.precision = args.precision
        rec["alt_precision"] = {"precision": "bf16", "value": round(seqs_per_step * T * args.steps / alt, 3),
                                "ms_per_step": round(alt / args.steps * 1e3, 3),
                                "dtype": "bf16 (activations; fp32 math and accumulation)"}
    if rank == 0 and not args.no_roofline:
        rec["roofline"] = roofline(model, seq, cfg)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(cfg, args.config, init_state, args.cpu_sample_snapshots)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
