"""The RCCL code path (backend "nccl") executed on one MI355X at world size 1.

The driver's 8-GPU runs are the only place several RCCL ranks meet; every other multi-rank test uses gloo.
This test makes the RCCL calls themselves run once on the device — the snapshot-shard all-to-all
(`sharded._all_to_all`, all_to_all_single on device buffers), the pooling all-reduce, and both gradient
buckets (`GradBucket.allreduce_mean`, `ShardGradSync.sync`, forced at world size 1) — and checks that a
one-rank collective leaves every value exactly as the unsharded model computed it (sum over one rank = identity).

Each case runs in a child process (``python tests/test_gpu_rccl.py <case>``).  The graph cases close the captured
step (``GraphedStep.close``: graph reset first) and then destroy the process group and exit normally -- the order whose
absence aborted a round-3 suite run after a graph had captured the group's collective.  The
graph cases create the group through ``tagan_amd.distributed.init_process_group`` (ProcessGroupNCCL's event cache
off) and ``GraphedStep`` waits for the watchdog to retire every eager Work before it captures -- the fix of the
watchdog's hipErrorCapturedEvent abort, which ``capture_after_eager_collective`` forces open.  The parent test
asserts the child's exit status and its completion marker.
"""
import os
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

COUNTS = [40, 57, 33, 57, 49, 21]


def _setup(dev):
    from tagan_amd import TAGAN, TAGANConfig
    cfg = TAGANConfig(node_feature_dim=8, edge_feature_dim=0, hidden_dim=64, num_heads=4, num_layers=2,
                      dropout=0.0, output_dim=1, window_size=3)
    torch.manual_seed(21)
    model = TAGAN(cfg).to(dev)
    g = torch.Generator().manual_seed(4)
    seq = [(torch.randn(n, 8, generator=g).to(dev), torch.randint(0, n, (2, 4 * n), generator=g).to(dev), None,
            list(range(n))) for n in COUNTS]
    return model, seq


def _case_shard_and_buckets():
    import tagan_amd  # noqa: F401
    from tagan_amd.distributed import GradBucket
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN, _all_to_all
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    import tempfile
    store = os.path.join(tempfile.mkdtemp(prefix="tagan_rccl_"), "store")   # file rendezvous: no TCP port race
    from tagan_amd.distributed import init_process_group
    init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        # raw all_to_all_single over device buffers
        a = torch.arange(12, dtype=torch.float32, device=dev).view(3, 4)
        (b,) = _all_to_all([a], [(3, 4)], None)
        assert torch.equal(a, b)

        labels = torch.tensor([1.0], device=dev)
        ref_model, seq = _setup(dev)
        ref = ref_model(seq, labels)
        ref["loss"].backward()
        ref_grads = {k: p.grad.clone() for k, p in ref_model.named_parameters() if p.grad is not None}

        model, seq = _setup(dev)
        out = SnapshotShardedTAGAN.for_model(model)(seq, COUNTS, labels)
        out["loss"].backward()
        ShardGradSync(list(model.named_parameters())).sync(force=True)
        torch.cuda.synchronize()
        torch.testing.assert_close(out["loss"], ref["loss"], rtol=1e-5, atol=1e-6)
        for k, p in model.named_parameters():
            if k in ref_grads:
                torch.testing.assert_close(p.grad, ref_grads[k], rtol=1e-4, atol=1e-5, msg=k)
            else:
                assert p.grad is None, k
        before = {k: p.grad.clone() for k, p in model.named_parameters() if p.grad is not None}
        GradBucket(model.parameters()).allreduce_mean(force=True)
        torch.cuda.synchronize()
        for k, p in model.named_parameters():
            if k in before:
                assert torch.equal(p.grad, before[k]), k
            else:
                assert p.grad is None, k
    finally:
        dist.destroy_process_group()


def _graph_vs_eager(dev, seq, steps_eager=6, replays=3, seed=3):
    """bench.py's N > 1 step at world size 1: forward, backward, the static gradient bucket's RCCL all-reduce
    (forced), clip and Adam captured as ONE HIP graph -- replayed, against the same step launched eagerly with the
    flagged bucket (dropout off): the same loss trajectory and weights."""
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.distributed import GradBucket
    from tagan_amd.graph_step import GraphedStep
    cfg = synthetic.config_for("c2", dropout=0.0)
    labels = torch.tensor([1.0], device=dev)

    def setup():
        torch.manual_seed(seed)
        m = TAGAN(cfg).to(dev).train()
        o = torch.optim.Adam(m.parameters(), lr=1e-3, capturable=True)
        return m, o, GradBucket(m.parameters())

    m1, o1, b1 = setup()
    eager = []
    for _ in range(steps_eager):
        o1.zero_grad(set_to_none=True)
        out = m1(seq, labels=labels)
        out["loss"].backward()
        b1.allreduce_mean(force=True)
        torch.nn.utils.clip_grad_norm_(m1.parameters(), 1.0)
        o1.step()
        eager.append(float(out["loss"]))

    m2, o2, b2 = setup()

    def whole():
        out = m2(seq, labels=labels)
        out["loss"].backward()
        b2.allreduce_mean(force=True, static=True)
        torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
        o2.step()
        return out["loss"]

    g = GraphedStep(m2, whole, optimizer=o2, warmup=steps_eager - replays)
    try:
        graphed = [float(g()) for _ in range(replays)]
    finally:
        g.close()
    torch.cuda.synchronize()
    for a, b in zip(eager[steps_eager - replays:], graphed):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (eager, graphed)
    for (k, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(p2, p1, atol=1e-5, rtol=1e-4, msg=k)


def _case_graph_step_sharded():
    """The snapshot-sharded step (sharded.py) captured as ONE HIP graph at world size 1 over RCCL, its exchanges
    forced: the all-to-all (snapshots -> node rows and back), the pooling all-reduce and the static ShardGradSync
    all-reduce all inside the graph; replays against the same step launched eagerly (the flagged ShardGradSync):
    the same loss trajectory and weights."""
    import tagan_amd  # noqa: F401
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.graph_step import GraphedStep
    from tagan_amd.sharded import ShardGradSync, SnapshotShardedTAGAN
    dev = torch.device("cuda:0")
    _init_nccl(dev, "gsh")
    try:
        cfg = synthetic.config_for("c5", dropout=0.0)
        seq = synthetic.make_sequence("c5", dev, seed=11, snapshots=8, nodes=300, edges=2400)
        counts = [int(x.shape[0]) for x, _, _, _ in seq]
        labels = torch.tensor([1.0], device=dev)
        steps_eager, replays = 6, 3

        def setup():
            torch.manual_seed(5)
            m = TAGAN(cfg).to(dev).train()
            o = torch.optim.Adam(m.parameters(), lr=1e-3, capturable=True)
            return (m, o, SnapshotShardedTAGAN.for_model(m, force_collectives=True),
                    ShardGradSync(list(m.named_parameters())))

        m1, o1, sh1, sy1 = setup()
        eager = []
        print("sharded case: eager steps", flush=True)
        for _ in range(steps_eager):
            o1.zero_grad(set_to_none=True)
            out = sh1(seq, counts, labels)
            out["loss"].backward()
            sy1.sync(force=True)
            torch.nn.utils.clip_grad_norm_(m1.parameters(), 1.0)
            o1.step()
            eager.append(float(out["loss"]))
        m2, o2, sh2, sy2 = setup()

        def whole():
            out = sh2(seq, counts, labels)
            out["loss"].backward()
            sy2.sync(force=True, static=True)
            torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
            o2.step()
            return out["loss"]

        print("sharded case: eager done %s; capture" % eager, flush=True)
        g = GraphedStep(m2, whole, optimizer=o2, warmup=steps_eager - replays)
        print("sharded case: captured; replays", flush=True)
        try:
            graphed = []
            for _ in range(replays):
                graphed.append(float(g()))
                print("sharded case: replay", graphed[-1], flush=True)
        finally:
            g.close()
        torch.cuda.synchronize()
        for a, b in zip(eager[steps_eager - replays:], graphed):
            assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (eager, graphed)
        for (k, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            torch.testing.assert_close(p2, p1, atol=1e-5, rtol=1e-4, msg=k)
    except BaseException:
        # a failed capture can leave the group unable to shut down: report and leave without destroying it
        import traceback
        traceback.print_exc()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)
    dist.destroy_process_group()


def _init_nccl(dev, tag):
    import tempfile
    torch.cuda.set_device(dev)
    store = os.path.join(tempfile.mkdtemp(prefix="tagan_rccl_%s_" % tag), "store")
    from tagan_amd.distributed import init_process_group   # RCCL event recycling off before the group exists
    init_process_group("nccl", init_method="file://" + store, rank=0, world_size=1)


def _case_graph_step_small():
    import tagan_amd  # noqa: F401
    from tagan_amd import synthetic
    dev = torch.device("cuda:0")
    _init_nccl(dev, "gs")
    seq = synthetic.make_sequence("c2", dev, seed=7, snapshots=6, nodes=400, edges=3000)
    _graph_vs_eager(dev, seq)
    dist.destroy_process_group()


def _case_graph_step_c2():
    """The same at the full C2 workload (10k nodes, 100k Zipf edges per snapshot, 32 snapshots): the size at which
    the round-2 split capture (an eager all-reduce between two captured segments) faulted on replay."""
    import tagan_amd  # noqa: F401
    from tagan_amd import synthetic
    dev = torch.device("cuda:0")
    _init_nccl(dev, "gc2")
    seq = synthetic.make_sequence("c2", dev, seed=1000)
    _graph_vs_eager(dev, seq, steps_eager=7, replays=4)
    dist.destroy_process_group()


def _capture_after_eager_collective():
    """The watchdog race made deterministic: the warm-up steps' eager all-reduces record their end events on the
    stream that is captured next, and the capture (only the capture) holds the host for 0.45 s (several 100-ms
    watchdog polls).  Without
    ``retire_pending_works`` a Work still on the watchdog's list is polled during the capture and the watchdog aborts
    the process (hipErrorCapturedEvent); with it, the capture and the replays are clean."""
    import time
    import tagan_amd  # noqa: F401
    from tagan_amd.graph_step import GraphedStep
    dev = torch.device("cuda:0")
    _init_nccl(dev, "race")
    lin = torch.nn.Linear(4, 4).to(dev)
    x = torch.ones(1 << 14, device=dev)
    out = torch.empty_like(x)

    def step():
        out.copy_(x * 2)
        dist.all_reduce(out)           # eager in the warm-up, captured afterwards
        if torch.cuda.is_current_stream_capturing():
            time.sleep(0.45)           # host time inside the capture only: the warm-up's Works stay un-retired
        return out.sum()

    try:
        g = GraphedStep(lin, step, warmup=3)
        try:
            vals = [float(g()) for _ in range(3)]
        finally:
            g.close()
        assert vals == [2.0 * x.numel()] * 3, vals
    finally:
        dist.destroy_process_group()


def _case_capture_race_unfixed():
    """NOT a test: the same case with ``retire_pending_works`` reduced to a device sync (the round-4 state), used by
    ``tools/runs/r5b.sh`` to show the abort the fix removes.  Expected: rc -6 / 134, the watchdog message."""
    import tagan_amd.distributed as D
    D.retire_pending_works = lambda device=None: torch.cuda.synchronize(device) or 0
    _capture_after_eager_collective()


CASES = {"shard_and_buckets": _case_shard_and_buckets, "graph_step_small": _case_graph_step_small,
         "graph_step_c2": _case_graph_step_c2, "capture_after_eager_collective": _capture_after_eager_collective,
         "capture_race_unfixed": _case_capture_race_unfixed, "graph_step_sharded": _case_graph_step_sharded}
OK = "RCCL_CASE_OK"


def _run_case(name, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), name], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    tail = (p.stdout[-3000:] + "\n" + p.stderr[-3000:])
    assert p.returncode == 0 and OK in p.stdout, "case %s: rc %s\n%s" % (name, p.returncode, tail)


def test_rccl_world1_shard_and_buckets():
    _run_case("shard_and_buckets")


def test_rccl_world1_graph_step_small():
    _run_case("graph_step_small")


def test_rccl_world1_graph_step_c2():
    """The graph-step case at the full C2 workload (10k nodes, 100k Zipf edges per snapshot, 32 snapshots): the size
    at which the round-2 split capture (an eager all-reduce between two captured segments) faulted on replay."""
    _run_case("graph_step_c2", timeout=280)


def test_rccl_world1_graph_step_sharded():
    """The snapshot-sharded step (all-to-all, pooling all-reduce, static gradient sync over RCCL) captured whole."""
    _run_case("graph_step_sharded", timeout=100)


def test_rccl_capture_after_eager_collective():
    """The capture-time watchdog race forced open: eager collectives on the capture stream right
    before a capture that holds the host across several watchdog polls.  Passes only because GraphedStep waits for the
    watchdog to retire every eager Work first."""
    _run_case("capture_after_eager_collective", timeout=120)


if __name__ == "__main__":
    if os.environ.get("TAGAN_CASE_STACK_AFTER"):   # diagnostics: dump every thread's stack, then exit, after N s
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["TAGAN_CASE_STACK_AFTER"]), exit=True)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    CASES[sys.argv[1]]()
    torch.cuda.synchronize()
    print(OK, flush=True)
