"""TAGAN host model on MI355X (drop-in for src/tagan/model.py:22-514).

Same constructor, module tree / ``state_dict`` keys, forward signature and
outputs as the reference ``TAGAN``.  The forward restates model.py:158-473
MI355X-first:

* all T snapshots of a sequence are processed as ONE block-diagonal graph:
  node features are concatenated ([ΣN_t, F]), one CSR/CSC is built on the
  device (``tagan_csr_build``) and shared by both geometric layers, forward
  and backward — one kernel launch per op per sequence instead of per snapshot;
* the temporal stage runs time-major ([T, N_max, H]) so neither the
  reference's stack+permute (temporal_attention.py:968-972) nor the pooling
  view (model.py:412) copies anything but the node-major pooling gather;
* the reference's exception-driven semantics are reproduced as explicit
  branches: TemporalPropagation always raises -> identity (model.py:302-309);
  the ones(T,T) temporal mask is causal iff T == num_heads, and a one-head
  T>1 model retries without a mask (model.py:362-375).

Parity against the reference (fp32, dropout=0): tests/test_gpu_parity.py.
"""
import os
from typing import Any, Dict, List, Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from .fused import precision as precision_ctx
from .ingest import SnapshotBatch, unpack as _unpack
from .kernels import build_graph, build_graph_cat, cat_adjacent, embed_linear, layer_norm, pool_time_major
from .layers.classification import ClassificationModule, TemporalLossModule, fused_head
from .layers.graph_attention import TAGANGraphAttention
from .layers.temporal_attention import AsymmetricTemporalAttention, MaskBroadcastError
from .layers.temporal_propagation import TemporalPropagation
from .utils.config import TAGANConfig
from .utils.memory_bank import NodeMemoryBank

# TAGAN_FUSED_HEAD=0: the classification head + loss as torch modules instead of csrc/head.hip (A/B)
FUSED_HEAD = os.environ.get("TAGAN_FUSED_HEAD", "1") != "0"

Snapshot = Union[Dict[str, Any], Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor], List[int]]]


class TAGAN(nn.Module):
    """``precision``: "fp32" (default, the parity mode), "bf16-gemm" (projection GEMM operands in
    bf16) or "bf16" (bf16 activations between kernels, fp32 math; see fused.py).  ``temporal_propagation``: "shipped" (default) reproduces the reference, whose
    TemporalPropagation never returns (identity); "intended" runs its tensor-mask compute
    (TemporalPropagation.forward_intended, pinned by the G6 fixtures) on the padded
    time-major features before the temporal attention."""

    def __init__(self, config: TAGANConfig, temporal_propagation: str = "shipped", precision: str = "fp32"):
        super().__init__()
        if temporal_propagation not in ("shipped", "intended"):
            raise ValueError("temporal_propagation must be 'shipped' or 'intended'")
        precision_ctx(precision)   # validates
        self.temporal_propagation_mode = temporal_propagation
        # index validation of the edge lists: "deferred" (checked after the geometric stage is launched, waiting
        # only for the CSR build), True (immediate device sync), False (off: HIP-graph capture)
        self.validate_edges = "deferred"
        self.precision = precision
        self.config = config
        self.memory_bank = NodeMemoryBank(hidden_dim=config.hidden_dim, decay_factor=0.8,
                                          max_inactivity=config.temporal_window_size)
        self.node_embedding = nn.Linear(config.node_feature_dim, config.hidden_dim)
        self.edge_embedding = (nn.Linear(config.edge_feature_dim, config.hidden_dim)
                               if config.edge_feature_dim > 0 else None)
        self.geometric_attention_layers = nn.ModuleList([
            TAGANGraphAttention(hidden_dim=config.hidden_dim, num_heads=config.num_heads, dropout=config.dropout,
                                distance_metric="scaled_dot_product" if config.learnable_distance else "euclidean",
                                use_layer_norm=config.use_layer_norm, learnable_distance=config.learnable_distance)
            for _ in range(config.num_layers)])
        self.temporal_propagation = TemporalPropagation(
            input_dim=config.hidden_dim, hidden_dim=config.hidden_dim, dropout=config.dropout,
            time_aware=config.time_aware, bidirectional=config.bidirectional, use_layer_norm=config.use_layer_norm,
            use_skip_connection=config.use_skip_connection, use_gating=config.use_gating,
            window_size=config.temporal_window_size, aggregation=config.aggregation_method,
            residual=config.use_residual)
        self.temporal_attention = AsymmetricTemporalAttention(
            hidden_dim=config.hidden_dim, num_heads=config.num_heads, dropout=config.dropout,
            causal=config.causal_attention, time_aware=True, use_layer_norm=config.use_layer_norm,
            asymmetric_window_size=config.window_size, relative_position_bias=config.asymmetric_temporal_bias)
        self.classification_head = ClassificationModule(
            hidden_dim=config.hidden_dim, task_configs={"output_dim": config.output_dim, "task_type": config.loss_type},
            multi_task=False, num_layers=2, dropout=config.dropout, use_layer_norm=config.use_layer_norm)
        self.loss_fn = TemporalLossModule(
            task_configs={"default": {"task_type": config.loss_type, "output_dim": config.output_dim}},
            loss_config={"reduction": "mean", "focal_alpha": config.focal_alpha, "focal_gamma": config.focal_gamma})
        self.skip_layer_norm = nn.LayerNorm(config.hidden_dim) if config.use_layer_norm else None
        nn.init.xavier_uniform_(self.node_embedding.weight)
        nn.init.zeros_(self.node_embedding.bias)
        if self.edge_embedding is not None:
            nn.init.xavier_uniform_(self.edge_embedding.weight)
            nn.init.zeros_(self.edge_embedding.bias)

    # ------------------------------------------------------------------ stages
    def encode_snapshots(self, graph_sequence: List[Snapshot], return_attention_weights: bool = False):
        """Per-snapshot stage (model.py:213-266) for all snapshots at once.

        Returns (x_cat [ΣN_t, H], node_counts, geometric attention placeholders).
        ``edge_embedding`` is not evaluated: its output is dead in the reference
        (model.py:236-239, never consumed) and its parameters get no gradient there either.
        """
        device = next(self.parameters()).device
        if isinstance(graph_sequence, SnapshotBatch):      # pre-ingested (ingest.py): one packed batch
            batch = graph_sequence if graph_sequence.x.device == device else graph_sequence.to(device)
            x_cat, counts = batch.x, list(batch.node_counts)
            graph = build_graph_cat(batch.edge_index, batch.edge_ptr, counts, validate=self.validate_edges)
        else:
            xs, eis, counts = [], [], []
            for snap in graph_sequence:
                x, ei, _ea, _ids = _unpack(snap)
                xs.append(x.to(device))
                eis.append(ei.to(device))
                counts.append(int(x.shape[0]))
            x_cat = cat_adjacent(xs, 0)   # a view when the snapshots share one buffer
            graph = build_graph(eis, counts, validate=self.validate_edges)
        h = embed_linear(x_cat, self.node_embedding.weight, self.node_embedding.bias)
        skip = h
        for i, layer in enumerate(self.geometric_attention_layers):
            if i == 0 and self.skip_layer_norm is not None:
                h = layer.forward_graph(h, graph, skip_ln=self.skip_layer_norm)   # + LN_skip(skip), fused
            else:
                h = layer.forward_graph(h, graph)
                if i == 0:
                    h = h + skip
        graph.check_valid()   # the reference's IndexError for an out-of-range edge (deferred: no stream stall)
        weights = [{"node_attention": None} for _ in range(len(counts))] if return_attention_weights else []
        return h, counts, weights

    @staticmethod
    def _time_major(x_cat: torch.Tensor, counts: List[int], n_max: Optional[int] = None) -> torch.Tensor:
        """Concatenated snapshots -> zero-padded [T, N_max, H] (temporal_attention.py:928-968 minus permute)."""
        T, H = len(counts), x_cat.shape[1]
        n_max = max(counts) if n_max is None else n_max
        if all(c == n_max for c in counts):
            return x_cat.view(T, n_max, H)
        out = x_cat.new_zeros(T, n_max, H)
        row = torch.cat([torch.arange(c, device=x_cat.device) + t * n_max for t, c in enumerate(counts)])
        return out.view(T * n_max, H).index_copy(0, row, x_cat).view(T, n_max, H)

    def _temporal(self, xt: torch.Tensor, return_attention_weights: bool):
        """AsymmetricTemporalAttention with the default ones(T,T) mask (model.py:320-375)."""
        try:
            return self.temporal_attention.forward_time_major(xt, True, return_attention_weights)
        except MaskBroadcastError:
            return self.temporal_attention._run(xt, True, None, None, return_attention_weights)

    @staticmethod
    def _pool(out_tm: torch.Tensor) -> torch.Tensor:
        """Pooling of model.py:377-427 on the time-major output.

        The reference holds out as node-major [N,T,H] and takes
        gf[t] = mean(out.view(T,-1,H)[t]) = mean of node-major flat rows
        [t*N, (t+1)*N) — not a per-snapshot mean.  Flat row r = n*T + t' lives at
        time-major row t'*N + n.
        """
        if out_tm.shape[-1] % 4 == 0 and out_tm.stride(2) == 1:
            return pool_time_major(out_tm)                      # csrc/pool.hip
        T, N, H = out_tm.shape
        node_major = out_tm.transpose(0, 1).reshape(T, N, H)   # == out.view(T, -1, H) of the reference
        return node_major.mean(1)

    def ingest(self, graph_sequence: List[Snapshot]) -> SnapshotBatch:
        """Pack a snapshot sequence (dicts or tuples, host or device tensors) into one device batch
        (ingest.py); ``forward`` accepts the result in place of the list."""
        return SnapshotBatch.from_sequence(graph_sequence, next(self.parameters()).device)

    def forward(self, graph_sequence: List[Snapshot], labels: Optional[torch.Tensor] = None,
                return_attention_weights: bool = False) -> Dict[str, Any]:
        with precision_ctx(self.precision):
            return self._forward(graph_sequence, labels, return_attention_weights)

    def _forward(self, graph_sequence, labels, return_attention_weights):
        if not isinstance(graph_sequence, SnapshotBatch):
            for snap in graph_sequence:
                _unpack(snap)   # format validation of model.py:187-200
        x_cat, counts, geo_w = self.encode_snapshots(graph_sequence, return_attention_weights)
        # TemporalPropagation never returns in the shipped code: identity (model.py:276-309).
        xt = self._time_major(x_cat, counts)
        if self.temporal_propagation_mode == "intended":
            xt = self.temporal_propagation.forward_intended(xt)
        out_tm, temp_w = self._temporal(xt, return_attention_weights)
        if return_attention_weights:
            self.last_temp_attn_weights = temp_w
        outputs = self.head(self._pool(out_tm), labels)
        if return_attention_weights:
            outputs["geometric_attention_weights"] = geo_w
            outputs["temporal_attention_weights"] = temp_w
        return outputs

    def head(self, pooled: torch.Tensor, labels: Optional[torch.Tensor] = None,
             dropout_seed: Optional[int] = None) -> Dict[str, Any]:
        """graph_features -> classification head -> loss / predictions (model.py:377-459); pooled [T, H].
        On the device the whole head + loss is one kernel each way (csrc/head.hip) when its shape and loss form
        are the fused ones; ``dropout_seed`` fixes that kernel's dropout mask (replicated heads)."""
        T = pooled.shape[0]
        batch_size = labels.shape[0] if (labels is not None and labels.dim() > 0) else 1
        if FUSED_HEAD:
            fused = fused_head(self.classification_head, pooled, batch_size, labels, self.config.output_dim,
                               dropout_seed)
            if fused is not None:
                logits, predictions, loss = fused
                # detached (the reference keeps the autograd history): a stored graph would keep the previous
                # step's AccumulateGrad nodes -- and the stream they were created on -- alive into the next
                # backward (a cross-stream join inside a captured HIP graph step)
                self.last_predictions = predictions.detach()
                if self.config.output_dim == 1:
                    self.last_binary_predictions = (predictions > 0.65).float()
                return {"logits": logits, "predictions": predictions, "loss": loss}
        if batch_size > 1:
            graph_features = torch.cat([pooled.unsqueeze(0), pooled.new_zeros(batch_size - 1, T, pooled.shape[1])])
        else:
            graph_features = pooled.unsqueeze(0)
        logits = self.classification_head(graph_features)
        loss = None
        if labels is not None:
            if labels.dtype == torch.bool:
                labels = labels.long()
            if self.config.output_dim > 1 and labels.dim() == 1:
                loss = nn.CrossEntropyLoss()(logits, labels)
            else:
                loss = self.loss_fn(logits, labels)
        if self.config.output_dim == 1:
            predictions = torch.sigmoid(logits)
            self.last_predictions = predictions.detach()
            self.last_binary_predictions = (predictions > 0.65).float()
        else:
            predictions = F.softmax(logits, dim=1)
            self.last_predictions = predictions.detach()
        return {"logits": logits, "predictions": predictions, "loss": loss}

    def infer(self, graph_sequence, return_probs: bool = True) -> Dict[str, Any]:
        self.eval()
        with torch.no_grad():
            outputs = self.forward(graph_sequence, return_attention_weights=False)
        if return_probs:
            preds = outputs["predictions"]
        elif self.config.output_dim == 1:
            preds = (outputs["predictions"] > 0.25).float()
        else:
            preds = torch.argmax(outputs["predictions"], dim=1)
        return {"predictions": preds, "logits": outputs["logits"]}

    @torch.no_grad()
    def infer_with_attention(self, graph_sequence) -> Dict[str, Any]:
        self.eval()
        return self.forward(graph_sequence, return_attention_weights=True)

    @classmethod
    def from_config(cls, config: Union[Dict[str, Any], TAGANConfig]) -> "TAGAN":
        if isinstance(config, dict):
            config = TAGANConfig.from_dict(config)
        return cls(config)

    def extra_repr(self) -> str:
        return f"config={self.config}"
