"""One TAGAN sequence sharded over P ranks by snapshot (second mode; C5).

The reference runs a sequence in one process (model.py:158-473).  Here rank r owns a
contiguous block of snapshots for the geometric stage — independent per snapshot
(model.py:213-266) — and a contiguous block of node rows for the temporal stage —
independent per node row (temporal_attention.py:904-1205 treats the padded [N_max, T, H]
batch row by row).  The only exchanges:

1. forward: ONE all-to-all from snapshot-major [T/P, N_max, H] to node-row-major
   [T, N_max/P, H] (backward: the reverse all-to-all);
2. the pooling of model.py:377-427, gf[t] = mean of node-major flat rows
   [t*N_max, (t+1)*N_max): each rank sums the flat rows it holds into a [T, H]
   partial, ONE all-reduce(SUM) gives gf on every rank (backward: identity, since the
   head is evaluated redundantly and identically on every rank);
3. the gradient exchange (``ShardGradSync``): sharded-stage parameters hold partial
   gradients (SUM across ranks); head parameters hold the full gradient on every rank
   (SUM / P) — one flat all-reduce that also carries a has-grad flag per parameter, so
   parameters that are dead on every rank keep grad None exactly as in the reference.

The head's dropout must draw the same mask on every rank: the generator it draws from is
reseeded from a per-step counter shared by all ranks.
"""
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .distributed import _phase


def blocks(n: int, parts: int) -> List[Tuple[int, int]]:
    """Contiguous near-equal split of range(n) into ``parts`` blocks (first blocks one longer)."""
    q, r = divmod(n, parts)
    out, a = [], 0
    for i in range(parts):
        b = a + q + (1 if i < r else 0)
        out.append((a, b))
        a = b
    return out


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _host_staged(t: torch.Tensor, group) -> bool:
    # gloo (CPU tests, several ranks sharing one GPU in the GPU tests) moves device tensors via the host
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_to_all(sends: List[torch.Tensor], recv_shapes: List[Tuple[int, ...]], group) -> List[torch.Tensor]:
    """Variable-size all-to-all as ONE all_to_all_single over flat buffers (RCCL over xGMI)."""
    x = torch.cat([s.reshape(-1) for s in sends])
    dev = x.device
    with _phase("all_to_all", x):
        staged = _host_staged(x, group)
        if staged:
            x = x.cpu()
        out_sizes = [int(torch.Size(sh).numel()) for sh in recv_shapes]
        y = x.new_empty(sum(out_sizes))
        dist.all_to_all_single(y, x, output_split_sizes=out_sizes, input_split_sizes=[s.numel() for s in sends],
                               group=group)
        if staged:
            y = y.to(dev)
    return [c.view(sh) for c, sh in zip(y.split(out_sizes), recv_shapes)]


def _all_reduce_sum(t: torch.Tensor, group, phase: str = "pool_allreduce") -> None:
    with _phase(phase, t):
        if _host_staged(t, group):
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)


class _SnapshotsToRows(torch.autograd.Function):
    """[T_r, N, H] (this rank's snapshots, all rows) -> [T, n_r, H] (all snapshots, this rank's rows)."""

    @staticmethod
    def forward(ctx, x_local, t_sizes, n_blocks, group, force=False):
        P, r = _world(group)
        H = x_local.shape[2]
        ctx.t_sizes, ctx.n_blocks, ctx.group, ctx.force = list(t_sizes), list(n_blocks), group, force
        n0, n1 = n_blocks[r]
        if P == 1 and not force:
            return x_local.clone()
        sends = [x_local[:, a:b] for a, b in n_blocks]
        recvs = _all_to_all(sends, [(t_sizes[p], n1 - n0, H) for p in range(P)], group)
        return torch.cat(recvs, 0)

    @staticmethod
    def backward(ctx, g):
        P, r = _world(ctx.group)
        if P == 1 and not ctx.force:
            return g.clone(), None, None, None, None
        H = g.shape[2]
        t_r = ctx.t_sizes[r]
        sends = list(g.split(ctx.t_sizes, 0))
        recvs = _all_to_all(sends, [(t_r, b - a, H) for a, b in ctx.n_blocks], ctx.group)
        return torch.cat(recvs, 1), None, None, None, None


class _SumAcrossRanks(torch.autograd.Function):
    """all-reduce(SUM) whose consumer is replicated on every rank: the backward is the identity."""

    @staticmethod
    def forward(ctx, x, group, force=False):
        y = x.clone()
        P, _ = _world(group)
        if P > 1 or (force and dist.is_available() and dist.is_initialized()):
            _all_reduce_sum(y, group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None, None


def pool_partial(out_rows: torch.Tensor, n0: int, n_max: int) -> torch.Tensor:
    """[T, n_r, H] temporal output of rows [n0, n0+n_r) -> [T, H] partial sums of the reference's
    pooling chunks (chunk t = node-major flat rows [t*N, (t+1)*N), flat row = n*T + t').

    The rank's flat rows meet a contiguous run of chunks, each in one contiguous stretch of them: one fixed-order
    column sum per stretch (static Python bounds: no device-side length table, nothing a captured HIP graph cannot
    replay -- torch.segment_reduce refused stream capture)."""
    T, n_r, H = out_rows.shape
    flat = out_rows.transpose(0, 1).reshape(n_r * T, H)
    f0, f1 = n0 * T, (n0 + n_r) * T
    sums, first = [], None
    for t in range(T):
        a, b = max(t * n_max, f0), min((t + 1) * n_max, f1)
        if b > a:
            first = t if first is None else first
            sums.append(flat[a - f0:b - f0].sum(0))
    if not sums:
        return flat.new_zeros(T, H)
    return torch.cat([flat.new_zeros(first, H), torch.stack(sums), flat.new_zeros(T - first - len(sums), H)])


class SnapshotShardedTAGAN:
    """Forward of one sequence over the ranks of ``group``.

    ``encode(snapshots) -> (x_cat [ΣN_t, H], counts)`` is the per-snapshot stage,
    ``temporal(xt [T, n, H]) -> [T, n, H]`` the temporal stage (time-major, rows independent),
    ``head(pooled [T, H], labels) -> outputs`` the replicated head.  ``for_model`` wires a
    ``tagan_amd.TAGAN``; tests wire the CPU oracle to check the exchange logic.
    """

    def __init__(self, encode: Callable, temporal: Callable, head: Callable, group=None, head_seed: int = 0x7A6A,
                 force_collectives: bool = False):
        self.encode, self.temporal, self.head = encode, temporal, head
        self.group = group
        self.head_seed = head_seed
        self.step = 0
        # run the all-to-all and the pooling all-reduce even at world size 1 (a live process group is required):
        # the one-GPU RCCL tests exercise (and capture) the exchange path this way
        self.force_collectives = force_collectives

    @classmethod
    def for_model(cls, model, group=None, force_collectives: bool = False):
        def encode(snaps):
            x_cat, counts, _ = model.encode_snapshots(snaps)
            return x_cat, counts

        def temporal(xt):   # propagation (intended mode) and attention are both per node row
            if model.temporal_propagation_mode == "intended":
                xt = model.temporal_propagation.forward_intended(xt)
            return model._temporal(xt, False)[0]

        def head(pooled, labels, step_seed):   # the fused head kernel's dropout mask: same on every rank
            return model.head(pooled, labels, dropout_seed=step_seed)

        obj = cls(encode, temporal, head, group, force_collectives=force_collectives)
        obj.head_takes_seed = True
        return obj

    def forward(self, local_snapshots: Sequence, counts_all: Sequence[int], labels: Optional[torch.Tensor] = None):
        P, r = _world(self.group)
        T, n_max = len(counts_all), max(counts_all)
        t_blocks, n_blocks = blocks(T, P), blocks(n_max, P)
        t0, t1 = t_blocks[r]
        if len(local_snapshots) != t1 - t0:
            raise ValueError("rank %d expects snapshots [%d, %d) of %d, got %d" % (r, t0, t1, T, len(local_snapshots)))
        n0, n1 = n_blocks[r]
        if t1 > t0:
            x_cat, counts = self.encode(local_snapshots)
            if list(counts) != list(counts_all[t0:t1]):
                raise ValueError("snapshot node counts differ from counts_all[%d:%d]" % (t0, t1))
            from .model import TAGAN
            x_local = TAGAN._time_major(x_cat, list(counts), n_max)
        else:
            x_local = self._empty(n_max)
        force = self.force_collectives and dist.is_available() and dist.is_initialized()
        xt_rows = _SnapshotsToRows.apply(x_local, [b - a for a, b in t_blocks], n_blocks, self.group, force)
        out_rows = self.temporal(xt_rows) if n1 > n0 else xt_rows
        pooled = _SumAcrossRanks.apply(pool_partial(out_rows, n0, n_max), self.group, force) / n_max
        self.step += 1
        if getattr(self, "head_takes_seed", False):
            # the fused head kernel takes its dropout seed directly (the same on every rank; under a captured
            # HIP graph the device seed counter is mixed in at run time): no torch generator involved
            return self.head(pooled, labels, (self.head_seed * 0x9E3779B1 + self.step) & 0x3FFFFFFFFFFFFFFF)
        # same head-dropout mask on every rank: the head draws from a generator seeded from a per-step
        # counter shared by all ranks, inside fork_rng so the caller's generators are left as they were
        devices = [pooled.device] if pooled.is_cuda else []
        with torch.random.fork_rng(devices=devices):
            if pooled.is_cuda:
                torch.cuda.manual_seed(self.head_seed + self.step)
            else:
                torch.manual_seed(self.head_seed + self.step)
            return self.head(pooled, labels)

    __call__ = forward

    def _empty(self, n_max):
        raise ValueError("every rank needs at least one snapshot (T >= world size)")


REPLICATED_PREFIXES = ("classification_head.", "loss_fn.")


class ShardGradSync:
    """Gradient exchange of the snapshot-sharded mode (see module docstring, item 3)."""

    def __init__(self, named_params, replicated_prefixes=REPLICATED_PREFIXES, group=None):
        self.items = [(n, p) for n, p in named_params if p.requires_grad]
        self.replicated = [any(n.startswith(x) for x in replicated_prefixes) for n, _ in self.items]
        self.group = group
        self.flat = None

    def sync(self, force: bool = False, static: bool = False):
        """``force``: run the collective even at world size 1 (exercises the RCCL path on one GPU).
        ``static``: the capturable form (HIP graph step): no has-grad flags and no host read-back -- the grads
        present locally are packed, summed, the replicated ones scaled by 1/P, and written back; every rank must
        hold the same set of grads (the flagged eager form run during warm-up establishes that)."""
        P, _ = _world(self.group)
        if P == 1 and not (force and dist.is_available() and dist.is_initialized()):
            return
        if static:
            live = [(k, p) for k, (_, p) in enumerate(self.items) if p.grad is not None]
            if not live:
                return
            n = sum(p.numel() for _, p in live)
            if self.flat is None or self.flat.numel() < n or self.flat.device != live[0][1].device:
                self.flat = torch.empty(n, dtype=live[0][1].dtype, device=live[0][1].device)
            flat = self.flat[:n]
            torch.cat([p.grad.reshape(-1) for _, p in live], out=flat)
            _all_reduce_sum(flat, self.group, phase="grad_allreduce")
            off = 0
            for k, p in live:
                m = p.numel()
                g = flat[off:off + m].view_as(p)
                if self.replicated[k]:
                    p.grad.copy_(g).div_(P)
                else:
                    p.grad.copy_(g)
                off += m
            return
        ref = self.items[0][1]
        n = sum(p.numel() for _, p in self.items)
        flat = torch.zeros(n + len(self.items), dtype=ref.dtype, device=ref.device)
        off = 0
        for k, (_, p) in enumerate(self.items):
            m = p.numel()
            if p.grad is not None:
                flat[off:off + m].copy_(p.grad.reshape(-1))
                flat[n + k] = 1.0
            off += m
        _all_reduce_sum(flat, self.group, phase="grad_allreduce")
        has = (flat[n:] > 0).tolist()
        off = 0
        for k, (_, p) in enumerate(self.items):
            m = p.numel()
            if has[k]:
                g = flat[off:off + m].view_as(p)
                if self.replicated[k]:
                    g = g / P
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
            off += m
