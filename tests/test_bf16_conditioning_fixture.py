"""The bf16 tolerance fixture (tests/golden/bf16_conditioning.json, written by tools/bf16_conditioning.py) covers
every tensor tests/test_gpu_fullsize.py::test_c2_bf16_vs_oracle bounds: logits, loss, d(node features) and the
gradient of every C2 parameter, each with a finite positive condition number (CPU only)."""
import json
import math
import os

import torch


def test_fixture_covers_every_checked_tensor():
    import oracle
    from tagan_amd import TAGAN, synthetic
    with open(os.path.join(os.path.dirname(__file__), "golden", "bf16_conditioning.json")) as f:
        fx = json.load(f)
    kappa = fx["kappa_rss"]
    assert fx["workload"]["config"] == "c2" and fx["joint_draws"] >= 8
    cfg = synthetic.config_for("c2", dropout=0.0)
    torch.manual_seed(0)
    model = TAGAN(cfg)
    # the parameters the oracle gives a gradient (the ones the GPU test bounds), from a small C2-shaped run
    P = {k: v.detach().double().requires_grad_(v.is_floating_point()) for k, v in model.state_dict().items()}
    seq = synthetic.make_sequence("c2", torch.device("cpu"), seed=1000, nodes=200, edges=2000, snapshots=4)
    seq = [(x.double(), ei, None, ids) for x, ei, _, ids in seq]
    oracle.tagan_forward(P, cfg.to_dict(), seq, torch.tensor([1.0], dtype=torch.float64))["loss"].backward()
    need = ["logits", "loss", "grad x"] + ["grad " + n for n, _ in model.named_parameters()
                                            if P[n].grad is not None]
    missing = [k for k in need if k not in kappa]
    assert not missing, missing
    for k in need:
        assert math.isfinite(kappa[k]) and kappa[k] > 0, k
