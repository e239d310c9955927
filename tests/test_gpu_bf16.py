"""bf16-GEMM mode (TAGAN(gemm_precision="bf16")): projection GEMMs take bf16 operands with fp32
accumulation; everything else fp32.  Not bit-compatible with the reference; checked against the
fp32 HIP model on the same inputs with a bf16-level tolerance (loss 1e-2 relative, every
gradient within 3e-2 relative of its norm, floored at 1e-3 of the largest gradient norm)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bf16_gemm_mode_tracks_fp32(dev=None):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import tagan_amd  # noqa: F401
    from tagan_amd import TAGAN, TAGANConfig
    dev = torch.device("cuda:0")
    cfg = TAGANConfig(node_feature_dim=16, edge_feature_dim=0, hidden_dim=128, num_heads=8, dropout=0.0,
                      output_dim=1)
    g = torch.Generator().manual_seed(5)
    seq = [(torch.randn(n, 16, generator=g).to(dev), torch.randint(0, n, (2, 6 * n), generator=g).to(dev), None,
            list(range(n))) for n in (300, 280, 310, 295, 300, 305)]
    labels = torch.tensor([1.0], device=dev)
    out = {}
    for mode in ("fp32", "bf16"):
        torch.manual_seed(1)
        m = TAGAN(cfg, gemm_precision=mode).to(dev)
        r = m(seq, labels)
        r["loss"].backward()
        out[mode] = (float(r["loss"]), {k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    l32, g32 = out["fp32"]
    l16, g16 = out["bf16"]
    assert abs(l16 - l32) <= 1e-2 * abs(l32)
    assert sorted(g16) == sorted(g32)
    scale = max(float(g.norm()) for g in g32.values())
    for k in g32:   # floor: gradients that vanish analytically (e.g. key biases under softmax) are noise
        err = float((g16[k] - g32[k]).norm()) / max(float(g32[k].norm()), 1e-3 * scale)
        assert err < 3e-2, (k, err)
