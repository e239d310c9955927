"""Data parallelism for TAGAN training: one process per GPU, gradients only.

The reference has no distributed code.  Sequences are
independent (one ``TAGAN.forward`` = one sequence, model.py:378-384), so each
rank trains on its own sequences and the only exchange is a gradient all-reduce
(RCCL over xGMI with backend "nccl"; gloo for CPU tests).  Gradients are
packed into ONE flat fp32 bucket (≤ 3.7 MB for every config — latency-bound,
so one collective beats per-tensor calls); parameters whose grad is None on
every rank (edge_embedding, temporal_propagation.*, time_encoding — dead in the
shipped forward) are skipped identically on all ranks.
"""
from typing import Iterable, List

import torch
import torch.distributed as dist


class GradBucket:
    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.flat = None

    def allreduce_mean(self, group=None) -> None:
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
            return
        live = [p for p in self.params if p.grad is not None]
        n = sum(p.numel() for p in live)
        if self.flat is None or self.flat.numel() != n or self.flat.device != live[0].grad.device:
            self.flat = torch.empty(n, dtype=torch.float32, device=live[0].grad.device)
        off = 0
        for p in live:
            k = p.numel()
            self.flat[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.flat.div_(dist.get_world_size(group))
        off = 0
        for p in live:
            k = p.numel()
            p.grad.copy_(self.flat[off:off + k].view_as(p.grad))
            off += k


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank start from rank ``src``'s weights."""
    if not dist.is_available() or not dist.is_initialized():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src=src, group=group)
