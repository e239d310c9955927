"""Seeded synthetic temporal graphs for the benchmark configs.

No datasets are available offline, so the shapes of the reference's inputs are
reproduced instead:
  * ``example``       — example.py:35-48: x~N(0,1), edge_index~U{0..N-1}
                        (duplicates and self-loops allowed), edge_attr~N(0,1).
  * ``social``        — synthetic_social_media_data.py/preprocess_social_media.py
                        shapes: F=27 node features, De=2 edge features, reply
                        edges parent-author -> reply-author with Zipf(1.1) user
                        activity (power-law degrees), same user set every snapshot.
Generated directly on the target device (inputs resident in HBM before timing).
"""
from typing import List, Sequence, Tuple

import torch

CONFIGS = {
    # name: (nodes, edges/snapshot, snapshots, hidden, heads, F, De, generator)
    "c1": (500, 1000, 10, 64, 4, 16, 8, "example"),
    "c2": (10_000, 100_000, 32, 128, 8, 27, 2, "social"),
    "c3": (100_000, 2_000_000, 64, 256, 8, 27, 2, "uniform"),
    "c4": (1_000_000, 20_000_000, 16, 128, 4, 27, 2, "uniform"),
    "c5": (100_000, 2_000_000, 128, 256, 16, 27, 2, "uniform"),
}


def make_sequence(name: str, device, seed: int = 42, snapshots: int = None,
                  nodes: int = None, edges: int = None) -> List[Tuple]:
    N, E, T, _H, _h, F, De, kind = CONFIGS[name]
    N = nodes or N
    E = edges or E
    T = snapshots or T
    g = torch.Generator(device=device).manual_seed(seed)
    seq = []
    if kind == "social":
        ranks = torch.randperm(N, generator=g, device=device).to(torch.float32) + 1.0
        activity = ranks.pow(-1.1)
    for _ in range(T):
        x = torch.randn(N, F, generator=g, device=device)
        if kind == "social":
            src = torch.multinomial(activity, E, replacement=True, generator=g)
            dst = torch.multinomial(activity, E, replacement=True, generator=g)
            ei = torch.stack([src, dst])
        else:
            ei = torch.randint(0, N, (2, E), generator=g, device=device)
        ea = torch.randn(E, De, generator=g, device=device)
        seq.append((x, ei, ea, list(range(N)) if N <= 100_000 else torch.arange(N)))
    return seq


def config_for(name: str, **over):
    from .utils.config import TAGANConfig
    N, E, T, H, h, F, De, _ = CONFIGS[name]
    kw = dict(hidden_dim=H, num_heads=h, node_feature_dim=F, edge_feature_dim=De, use_edge_features=True,
              output_dim=1, loss_type="bce", dropout=0.1, device="cuda")
    kw.update(over)
    return TAGANConfig(**kw)
