"""GPU parity of the fused classification head + loss (csrc/head.hip) against a plain PyTorch fp64 restatement
of the reference's head (classification.py:856-966: attention pooling over T, Linear -> LayerNorm -> ReLU ->
Dropout -> Linear) and loss forms (model.py:430-459: BCE-with-logits mean through TemporalLossModule, cross
entropy for output_dim > 1 with 1-D labels), on graph_features with row 0 = the pooled means and rows 1..B-1 zero
(model.py:382-394).  Gradients flow through all three outputs (logits, predictions, loss).  With dropout the
fp64 reference uses the kernel's counter-hash mask regenerated on the host (tagan_uniform(seed, row, feature))."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 1e-4


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    return torch.device("cuda:0")


def _module(H, C, p, seed):
    from tagan_amd.layers.classification import ClassificationModule
    torch.manual_seed(seed)
    m = ClassificationModule(hidden_dim=H, task_configs={"output_dim": C, "task_type": "classification"},
                             multi_task=False, num_layers=2, dropout=p, use_layer_norm=True)
    with torch.no_grad():   # non-trivial biases / LN affine
        for name, prm in m.named_parameters():
            if prm.dim() == 1:
                prm.add_(0.1 * torch.randn_like(prm))
    return m


def _ref(m, pooled, B, labels, kind, mask):
    """fp64 restatement; mask [B, H] of kept-and-scaled dropout factors (ones without dropout)."""
    head = m.classification_head
    P = {k: v.detach().double().clone().requires_grad_() for k, v in head.named_parameters()}
    x0 = pooled.detach().double().clone().requires_grad_()
    T, H = x0.shape
    gf = torch.cat([x0.unsqueeze(0), x0.new_zeros(B - 1, T, H)]) if B > 1 else x0.unsqueeze(0)
    s = torch.tanh(gf @ P["attention.0.weight"].t() + P["attention.0.bias"]) @ P["attention.2.weight"].t()
    pooled_b = (gf * torch.softmax(s, dim=1)).sum(1)
    u = pooled_b @ P["classifier.0.weight"].t() + P["classifier.0.bias"]
    n = torch.nn.functional.layer_norm(u, (H,), P["classifier.1.weight"], P["classifier.1.bias"], 1e-5)
    h2 = torch.relu(n) * mask
    logits = h2 @ P["classifier.4.weight"].t() + P["classifier.4.bias"]
    C = logits.shape[1]
    preds = torch.sigmoid(logits) if C == 1 else torch.softmax(logits, 1)
    loss = None
    if kind == "bce":
        lab = labels.double().reshape(logits.shape) if C == 1 else labels.double()
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, lab)
    elif kind == "ce":
        loss = torch.nn.functional.cross_entropy(logits, labels.long())
    return x0, P, logits, preds, loss


CASES = [  # T, H, C, B, kind, label shape
    (10, 64, 1, 1, "bce", "1d"),
    (32, 128, 1, 3, "bce", "1d"),
    (32, 128, 1, 2, "bce", "2d"),
    (16, 128, 3, 2, "ce", "1d"),
    (16, 128, 3, 2, "bce", "2d"),
    (5, 64, 2, 1, "none", None),
    (128, 64, 1, 1, "bce", "1d"),
    (32, 256, 1, 2, "bce", "1d"),     # T·H = 8192: the largest head the kernel takes, 4 step groups
    (20, 96, 4, 2, "ce", "1d"),       # H not a power of two: 10 step groups, 64 idle threads
    (16, 128, 3, 4, "ce_ignore", "1d"),   # nn.CrossEntropyLoss's ignore_index -100 on one row
]


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("T,H,C,B,kind,lshape", CASES)
def test_fused_head(dev, T, H, C, B, kind, lshape, p):
    from tagan_amd import _lib
    from tagan_amd.layers.classification import fused_head
    m = _module(H, C, p, seed=T + H + C).to(dev).train()
    g = torch.Generator().manual_seed(5)
    pooled = (torch.randn(T, H, generator=g) * 0.5).to(dev).requires_grad_()
    labels = None
    if kind == "bce":
        labels = (torch.rand(B, generator=g) > 0.5).float() if lshape == "1d" else \
            (torch.rand(B, C, generator=g) > 0.5).float()
    elif kind in ("ce", "ce_ignore"):
        labels = torch.randint(0, C, (B,), generator=g)
        if kind == "ce_ignore":
            labels[1] = -100
    labels = labels.to(dev) if labels is not None else None
    seed = 12345
    out = fused_head(m, pooled, B, labels, C, seed=seed)
    assert out is not None, "fused path not taken"
    logits, preds, loss = out
    keep = 1.0 / (1.0 - p) if p > 0 else 1.0
    mask = torch.ones(B, H, dtype=torch.float64)
    if p > 0:
        L = _lib.lib()
        for b in range(B):
            for j in range(H):
                mask[b, j] = keep if L.tagan_uniform(seed, b, j) >= p else 0.0
    import copy
    x0, P, rl, rp, rloss = _ref(copy.deepcopy(m).cpu(), pooled.detach().cpu(), B,
                                labels.cpu() if labels is not None else None, "ce" if kind == "ce_ignore" else kind,
                                mask)
    torch.testing.assert_close(logits.double().cpu(), rl.detach(), atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(preds.double().cpu(), rp.detach(), atol=ATOL, rtol=RTOL)
    if kind == "none":
        assert loss is None
    else:
        torch.testing.assert_close(loss.double().cpu(), rloss.detach(), atol=ATOL, rtol=RTOL)
    # upstream gradient into all three outputs
    r1 = torch.randn(B, C, generator=g, dtype=torch.float64)
    r2 = torch.randn(B, C, generator=g, dtype=torch.float64)
    obj = (logits * r1.to(dev).float()).sum() + (preds * r2.to(dev).float()).sum() + (loss if loss is not None else 0)
    obj.backward()
    robj = (rl * r1).sum() + (rp * r2).sum() + (rloss if rloss is not None else 0)
    robj.backward()
    torch.testing.assert_close(pooled.grad.double().cpu(), x0.grad, atol=ATOL, rtol=RTOL, msg="d pooled")
    for name, prm in m.classification_head.named_parameters():
        torch.testing.assert_close(prm.grad.double().cpu().reshape(P[name].shape), P[name].grad, atol=ATOL,
                                   rtol=RTOL, msg=name)


def test_fused_head_in_model_matches_module_path(dev):
    """TAGAN.head with the fused kernel against TAGAN_FUSED_HEAD=0 (the torch modules), eval mode, B = 3."""
    import tagan_amd.model as M
    from tagan_amd import TAGAN, TAGANConfig
    cfg = TAGANConfig(hidden_dim=128, num_heads=8, node_feature_dim=27, edge_feature_dim=2, output_dim=1,
                      loss_type="bce", dropout=0.1, device="cuda")
    torch.manual_seed(4)
    model = TAGAN(cfg).to(dev).eval()
    pooled = torch.randn(32, 128, device=dev)
    labels = torch.tensor([1.0, 0.0, 1.0], device=dev)
    res = {}
    for fused in (True, False):
        M.FUSED_HEAD = fused
        try:
            x = pooled.clone().requires_grad_()
            out = model.head(x, labels)
            out["loss"].backward()
            res[fused] = (out["logits"].detach(), out["predictions"].detach(), out["loss"].detach(), x.grad.clone(),
                          {k: p.grad.clone() for k, p in model.classification_head.named_parameters()})
            model.zero_grad(set_to_none=True)
        finally:
            M.FUSED_HEAD = True
    for a, b in zip(res[True][:4], res[False][:4]):
        torch.testing.assert_close(a, b, atol=ATOL, rtol=RTOL)
    for k in res[True][4]:
        torch.testing.assert_close(res[True][4][k], res[False][4][k], atol=ATOL, rtol=RTOL, msg=k)


def test_fused_head_misaligned_pooled_view(dev):
    """A pooled [T, H] view 4 bytes into its storage (the kernels read x0 as float4 runs): the wrapper copies it, and
    the results equal the aligned call's bit for bit."""
    from tagan_amd.layers.classification import fused_head
    T, H = 32, 128
    m = _module(H, 1, 0.0, seed=3).to(dev).train()
    g = torch.Generator().manual_seed(9)
    base = (torch.randn(T * H + 1, generator=g) * 0.5).to(dev)
    odd = base[1:].view(T, H).detach().requires_grad_()
    assert odd.data_ptr() % 16 != 0
    even = odd.detach().clone().requires_grad_()
    labels = torch.ones(1, device=dev)
    outs = []
    for x in (odd, even):
        m.zero_grad()
        logits, preds, loss = fused_head(m, x, 1, labels, 1, seed=1)
        loss.backward()
        outs.append((logits.detach().clone(), loss.detach().clone(), x.grad.clone(),
                     m.classification_head.attention[0].weight.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
