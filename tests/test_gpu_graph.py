"""The whole training step captured as one HIP graph (graph_step.GraphedStep) against the same step run eagerly:
identical trajectory with dropout off (same kernels, same order), fresh dropout masks on every replay with
dropout on (the device seed counter), and eager launches unchanged once the counter is unregistered."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _setup(dev, dropout, seed=3, config="c2", snapshots=6, nodes=400, edges=3000):
    from tagan_amd import TAGAN, synthetic
    cfg = synthetic.config_for(config, dropout=dropout)
    torch.manual_seed(seed)
    model = TAGAN(cfg).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=True)
    seq = synthetic.make_sequence(config, dev, seed=7, snapshots=snapshots, nodes=nodes, edges=edges)
    labels = torch.tensor([1.0], device=dev)

    def step():
        out = model(seq, labels=labels)
        out["loss"].backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return out["loss"]
    return model, opt, step


def test_graph_matches_eager_without_dropout(dev):
    from tagan_amd.graph_step import GraphedStep
    m1, o1, s1 = _setup(dev, 0.0)
    m2, o2, s2 = _setup(dev, 0.0)
    eager = []
    for _ in range(6):
        o1.zero_grad(set_to_none=True)
        eager.append(float(s1()))
    g = GraphedStep(m2, s2, optimizer=o2, warmup=3)    # 3 eager warm-up steps, then the capture
    try:
        graphed = [float(g()) for _ in range(3)]
    finally:
        g.close()
    torch.cuda.synchronize()
    # warm-up steps 1-3 ran eagerly on m2; replays are steps 4-6
    for a, b in zip(eager[3:], graphed):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (eager, graphed)
    for (k, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(p2, p1, atol=1e-5, rtol=1e-4, msg=k)


def test_graph_replays_draw_fresh_dropout(dev):
    from tagan_amd.graph_step import GraphedStep
    model, opt, step = _setup(dev, 0.1)
    for p in model.parameters():
        p.requires_grad_(True)
    g = GraphedStep(model, step, optimizer=opt, warmup=2)
    try:
        c0 = int(g.counter.item())
        losses = [float(g()) for _ in range(4)]
        assert int(g.counter.item()) == c0 + 4
    finally:
        g.close()
    assert all(torch.isfinite(torch.tensor(losses)))
    assert len(set(losses)) == len(losses), losses   # different masks (and weights) every replay


def test_counter_unregistered_restores_eager_seeds(dev):
    """A train-mode (dropout on) eager forward with fixed seeds gives bitwise the same logits before a graph was
    captured and after close(): the advanced device counter no longer enters the masks."""
    from tagan_amd import synthetic
    from tagan_amd.graph_step import GraphedStep
    model, opt, step = _setup(dev, 0.1, seed=5)
    seq = synthetic.make_sequence("c2", dev, seed=9, snapshots=4, nodes=300, edges=2000)
    state = {k: v.clone() for k, v in model.state_dict().items()}

    def fwd():
        model.load_state_dict(state)
        torch.manual_seed(123)
        with torch.no_grad():
            return model(seq)["logits"].clone()
    before = fwd()
    g = GraphedStep(model, step, optimizer=opt, warmup=1)
    g()
    g()
    g.close()
    assert int(g.counter.item()) >= 2
    assert torch.equal(fwd(), before)


def test_graph_intended_propagation_matches_eager(dev):
    """TAGAN with the intended TemporalPropagation (matrix-core GRU kernels, skip-window kernel) captured as one
    graph: replays 4-6 follow the eager trajectory (dropout off)."""
    from tagan_amd import TAGAN, synthetic
    from tagan_amd.graph_step import GraphedStep
    cfg = synthetic.config_for("c2", dropout=0.0)
    seq = synthetic.make_sequence("c2", dev, seed=7, snapshots=6, nodes=400, edges=3000)
    labels = torch.tensor([1.0], device=dev)

    def setup():
        torch.manual_seed(3)
        m = TAGAN(cfg, temporal_propagation="intended").to(dev).train()
        o = torch.optim.Adam(m.parameters(), lr=1e-3, capturable=True)

        def step():
            out = m(seq, labels=labels)
            out["loss"].backward()
            o.step()
            return out["loss"]
        return m, o, step
    m1, o1, s1 = setup()
    eager = []
    for _ in range(6):
        o1.zero_grad(set_to_none=True)
        eager.append(float(s1()))
    m2, o2, s2 = setup()
    g = GraphedStep(m2, s2, optimizer=o2, warmup=3)
    try:
        graphed = [float(g()) for _ in range(3)]
    finally:
        g.close()
    torch.cuda.synchronize()
    for a, b in zip(eager[3:], graphed):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (eager, graphed)


def test_graph_keeps_offset_table_through_cache_eviction(dev):
    """The snapshot offset table a captured step reads by address is pinned: flooding the LRU cache with 300 other
    shapes between replays (kernels._ptr_table evicts beyond 256) neither frees it nor changes the trajectory."""
    from tagan_amd import kernels
    from tagan_amd.graph_step import GraphedStep
    m1, o1, s1 = _setup(dev, 0.0)
    m2, o2, s2 = _setup(dev, 0.0)
    eager = []
    for _ in range(6):
        o1.zero_grad(set_to_none=True)
        eager.append(float(s1()))
    g = GraphedStep(m2, s2, optimizer=o2, warmup=3)
    try:
        assert len(kernels._PTR_PINNED) >= 1
        pinned = dict(kernels._PTR_PINNED)
        graphed = [float(g())]
        for i in range(300):                      # evict every unpinned entry, allocating over the freed blocks
            kernels._ptr_table(dev, [0, i + 1, 2 * i + 7])
        junk = torch.full((1 << 20,), -1, dtype=torch.int64, device=dev)
        graphed += [float(g()) for _ in range(2)]
        del junk
        assert all(kernels._PTR_PINNED[k] is t for k, t in pinned.items())
    finally:
        g.close()
    torch.cuda.synchronize()
    for a, b in zip(eager[3:], graphed):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (eager, graphed)


def test_graphed_step_has_no_split_form(dev):
    from tagan_amd.graph_step import GraphedStep
    m, o, s = _setup(dev, 0.0)
    with pytest.raises(TypeError):
        GraphedStep(m, s, optimizer=o, warmup=1, between=lambda: None, post=lambda: None)


def test_graph_keep_cache_matches_hash_path_at_t128(dev, monkeypatch):
    """C5's temporal shape (T = 128, 16 heads, H = 256) with attention dropout, captured: the replays with the
    keep-bit cache (the forward stores its dropout decisions, the backward reads them) against the same replays with
    the backward re-hashing the counters -- the same masks, so the same trajectory to fp32 rounding (the cached
    backward applies 1 / (1 - p) per output instead of per element)."""
    import ctypes
    from tagan_amd import fused
    from tagan_amd.graph_step import GraphedStep

    def run():
        model, opt, step = _setup(dev, 0.1, config="c5", snapshots=128, nodes=200, edges=1200)
        g = GraphedStep(model, step, optimizer=opt, warmup=2)
        try:
            losses = [float(g()) for _ in range(3)]
        finally:
            g.close()
        torch.cuda.synchronize()
        return losses, [p.detach().clone() for p in model.parameters()]

    written = []
    real = fused._keep_cache

    def spy(*args):
        out = real(*args)
        written.append(out[0] is not None)
        return out
    monkeypatch.setattr(fused, "_keep_cache", spy)
    la, pa = run()
    assert any(written), "the T = 128 temporal forward allocates the keep-bit cache"
    monkeypatch.setattr(fused, "_keep_cache", lambda *args: (None, 0, ctypes.c_int32(0)))
    lb, pb = run()
    for a, b in zip(la, lb):
        assert abs(a - b) <= 1e-5 * max(1.0, abs(a)), (la, lb)
    for x, y in zip(pa, pb):
        torch.testing.assert_close(x, y, atol=1e-5, rtol=1e-4)
