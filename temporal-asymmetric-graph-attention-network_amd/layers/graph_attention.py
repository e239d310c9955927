"""TAGANGraphAttention on MI355X (drop-in for src/tagan/layers/graph_attention.py:15-136).

The reference scatters ``edge_index`` into a dense [1,N,N] mask plus ``eye(N)``
(graph_attention.py:96-105).  Here the same set — unique (src,dst) pairs plus
self-loops, src = query row — is built once as a device CSR/CSC by
``tagan_csr_build`` and shared by every layer, by forward and backward, and by
all snapshots of a sequence (``forward_graph``).
"""
from typing import Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from ..kernels import SnapshotGraph, build_graph
from .geometric_attention import GeometricAttention


class TAGANGraphAttention(nn.Module):
    def __init__(self, hidden_dim: int, num_heads: int = 8, dropout: float = 0.1,
                 distance_metric: str = "scaled_dot_product", use_layer_norm: bool = True,
                 learnable_distance: bool = False):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.geometric_attention = GeometricAttention(hidden_dim=hidden_dim, num_heads=num_heads, dropout=dropout,
                                                      distance_metric=distance_metric,
                                                      use_layer_norm=use_layer_norm,
                                                      learnable_distance=learnable_distance)

    def forward_graph(self, x: torch.Tensor, graph: SnapshotGraph, skip_ln=None) -> torch.Tensor:
        return self.geometric_attention.forward_graph(x, graph, skip_ln)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, edge_attr: Optional[torch.Tensor] = None,
                return_attention_weights: bool = False
                ) -> Union[torch.Tensor, Tuple[torch.Tensor, Dict[str, Optional[torch.Tensor]]]]:
        """x [N,H], edge_index [2,E] -> [N,H] (edge_attr is ignored, as in the reference :108-112)."""
        N = x.size(0)
        if edge_index is None:
            # no mask: dense attention over all N nodes (geometric_attention.py mask=None)
            out = self.geometric_attention(x.unsqueeze(0)).squeeze(0)
        else:
            graph = build_graph([edge_index], [N])
            out = self.forward_graph(x, graph)
        if return_attention_weights:
            return out, {"node_attention": None}          # placeholder, as graph_attention.py:121
        return out

    def extra_repr(self) -> str:
        return f"hidden_dim={self.hidden_dim}"
