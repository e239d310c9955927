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
import os
import time
from contextlib import contextmanager
from typing import Dict, Iterable, List, Optional

import torch
import torch.distributed as dist


# Capturing a collective while a process group is live.  ProcessGroupNCCL's watchdog thread polls the
# end event of every eager collective's Work (``hipEventQuery``) until it has seen it complete and dropped the Work
# from its list -- up to one poll period (100 ms) after the device finished it.  A collective issued with
# async_op=False runs on, and records its end event on, the CALLER's current stream; GraphedStep warms up on the very
# stream it then captures.  HIP answers a query of an event whose recording stream is capturing with
# hipErrorCapturedEvent -- even when the record itself was eager (tools/captured_event_probe.py shows it without any
# process group) -- and the watchdog treats that as fatal.  So an eager Work still on the watchdog's list when the
# capture starts aborts the process whenever a poll lands inside the capture: a timing race (once in ~5 suites).
# ``retire_pending_works`` removes it: it returns only when every RCCL group's watchdog list is empty
# (ProcessGroupNCCL::waitForPendingWorks), so no event the watchdog can poll was recorded on the capturing stream.
#
# The event cache is switched off too (independent of the race): with it on, a retired Work's end event is handed to
# the next collective -- the captured one -- so one event object would be shared between a graph node and later
# eager Works.  The flag is read when a process group is constructed: it must be set before init_process_group.
EVENT_CACHE_ENV = "TORCH_NCCL_CUDA_EVENT_CACHE"
_graph_safe_groups = False   # graph_safe_env() ran (init_process_group calls it before creating the group)
_cache_on_group = False      # graph_safe_env() ran while a group built with the cache ON already existed


def graph_safe_env() -> None:
    """Switch ProcessGroupNCCL's event recycling off for the process groups created from here on.  Called while a
    process group built with the cache on already exists, it records that: that group stays unsafe to capture."""
    global _graph_safe_groups, _cache_on_group
    if dist.is_available() and dist.is_initialized() and os.environ.get(EVENT_CACHE_ENV) != "0":
        _cache_on_group = True
    os.environ[EVENT_CACHE_ENV] = "0"
    _graph_safe_groups = True


def graph_safe_groups() -> bool:
    """True when this process's groups were built with the event cache off: created after ``graph_safe_env()``, or
    with ``TORCH_NCCL_CUDA_EVENT_CACHE=0`` exported by the caller before ``dist.init_process_group``."""
    if _cache_on_group:
        return False
    return _graph_safe_groups or os.environ.get(EVENT_CACHE_ENV) == "0"


def init_process_group(backend: str, **kw) -> None:
    """``torch.distributed.init_process_group`` with ``graph_safe_env()`` applied first (any backend: a later RCCL
    group created with ``new_group`` reads the same flag)."""
    graph_safe_env()
    dist.init_process_group(backend, **kw)


def nccl_groups() -> list:
    """Every live process group whose backend is RCCL ("nccl")."""
    if not (dist.is_available() and dist.is_initialized()):
        return []
    out = []
    for pg in list(dist.distributed_c10d._world.pg_map.keys()):
        try:
            if "nccl" in str(dist.get_backend(pg)).lower():
                out.append(pg)
        except Exception:
            continue
    return out


def retire_pending_works(device=None) -> int:
    """Drain the device, then block until every RCCL group's watchdog has retired all of its eager Works
    (``ProcessGroup._wait_for_pending_works``: returns once the watchdog's work list is empty; the watchdog holds
    the list's mutex while it polls, so after the return it polls no earlier event).  Returns the number of groups
    waited on.  Call it right before capturing a graph on a stream that eager collectives have used."""
    groups = nccl_groups()
    if not groups:
        return 0
    missing = [pg for pg in groups if not callable(getattr(pg, "_wait_for_pending_works", None))]
    if missing:
        raise RuntimeError("retire_pending_works: this torch (%s) has no ProcessGroup._wait_for_pending_works, so the "
                           "RCCL watchdog's eager Works cannot be retired before a capture; capturing now could abort "
                           "the process (DESIGN.md section 6) -- run the step eagerly (GraphedStep off)" % torch.__version__)
    torch.cuda.synchronize(device)
    for pg in groups:
        pg._wait_for_pending_works()
    return len(groups)


def _staged(t: torch.Tensor, group) -> bool:
    # gloo moves device tensors through the host (CPU tests; several ranks sharing one GPU).  PyTorch's gloo backend
    # has no ROCm device-tensor path of its own (ProcessGroupGloo's device collectives are the CUDA-stream ones), so
    # device tensors are always staged here; RCCL ("nccl") takes device tensors directly.
    return t.is_cuda and dist.get_backend(group) == "gloo"


class ExchangeTimer:
    """Per-phase time of the collectives inside a step (``bench.py`` sub-records: gradient all-reduce, all-to-all,
    pooling all-reduce).  Device tensors: HIP events recorded on the current stream around the call, so the time is
    what the collective costs the step (the current stream waits for RCCL's); host tensors: wall clock.
    Events are resolved after the caller's synchronisation (``totals``)."""

    def __init__(self):
        self.marks: Dict[str, list] = {}
        self.host: Dict[str, float] = {}
        self.calls: Dict[str, int] = {}

    @contextmanager
    def phase(self, name: str, t: Optional[torch.Tensor] = None):
        self.calls[name] = self.calls.get(name, 0) + 1
        if t is not None and t.is_cuda and not torch.cuda.is_current_stream_capturing():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            yield
            b.record()
            self.marks.setdefault(name, []).append((a, b))
        else:
            t0 = time.perf_counter()
            yield
            self.host[name] = self.host.get(name, 0.0) + (time.perf_counter() - t0) * 1e3

    def totals(self) -> Dict[str, float]:
        """Milliseconds per phase since the last ``reset`` (device events synchronised here)."""
        out = dict(self.host)
        for name, evs in self.marks.items():
            ms = 0.0
            for a, b in evs:
                b.synchronize()
                ms += a.elapsed_time(b)
            out[name] = out.get(name, 0.0) + ms
        return out

    def reset(self) -> None:
        self.marks.clear()
        self.host.clear()
        self.calls.clear()


TIMER: Optional[ExchangeTimer] = None   # set by bench.py around its sub-record steps


@contextmanager
def _phase(name: str, t: torch.Tensor):
    if TIMER is None:
        yield
    else:
        with TIMER.phase(name, t):
            yield


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None, phase: str = "all_reduce") -> None:
    """In-place all-reduce of ``t`` on any backend (host-staged for gloo with a device tensor)."""
    with _phase(phase, t):
        if _staged(t, group):
            h = t.cpu()
            dist.all_reduce(h, op=op, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op, group=group)


def broadcast_(t: torch.Tensor, src: int = 0, group=None) -> None:
    if _staged(t, group):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src, group=group)


class GradBucket:
    """ONE flat all-reduce of every trainable parameter's gradient plus a has-grad flag per parameter.

    The buffer layout is the same on every rank whatever grads exist locally (a missing grad is packed as
    zeros), so the collective always matches across ranks; after the reduction a parameter whose grad was
    None on EVERY rank keeps grad None (dead in the shipped forward, as in the reference), one that had a
    grad on some rank gets the mean.  The flags ride in the same buffer: no second collective.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.n = sum(p.numel() for p in self.params)
        self.flat = None

    def allreduce_mean(self, group=None, force: bool = False, static: bool = False) -> None:
        """``force``: run the collective even at world size 1 (exercises the RCCL path on one GPU).
        ``static``: the capturable form (HIP graphs): no flags and no host read-back — the grads present
        locally are packed, reduced and written back; every rank must have the same grads present (the
        flagged form, used by the eager warm-up before a capture, establishes that)."""
        if not dist.is_available() or not dist.is_initialized():
            return
        if dist.get_world_size(group) == 1 and not force:
            return
        if not self.params:
            return
        if static:
            live = [p for p in self.params if p.grad is not None]
            if not live:
                return
            n = sum(p.numel() for p in live)
            if self.flat is None or self.flat.device != live[0].device or self.flat.numel() < n:
                self.flat = torch.empty(max(n, self.n + len(self.params)), dtype=torch.float32, device=live[0].device)
            torch.cat([p.grad.reshape(-1) for p in live], out=self.flat[:n])
            all_reduce_(self.flat[:n], dist.ReduceOp.SUM, group, phase="grad_allreduce")
            self.flat[:n].div_(dist.get_world_size(group))
            off = 0
            for p in live:
                m = p.numel()
                p.grad.copy_(self.flat[off:off + m].view_as(p))
                off += m
            return
        dev = self.params[0].device
        k = len(self.params)
        if self.flat is None or self.flat.device != dev:
            self.flat = torch.empty(self.n + k, dtype=torch.float32, device=dev)
        flags = self.flat[self.n:]
        off = 0
        for i, p in enumerate(self.params):
            m = p.numel()
            if p.grad is not None:
                self.flat[off:off + m].copy_(p.grad.reshape(-1))
            else:
                self.flat[off:off + m].zero_()
            off += m
        flags.copy_(torch.tensor([p.grad is not None for p in self.params], dtype=torch.float32), non_blocking=True)
        all_reduce_(self.flat, dist.ReduceOp.SUM, group, phase="grad_allreduce")
        self.flat[:self.n].div_(dist.get_world_size(group))
        has = (flags > 0).tolist()
        off = 0
        for i, p in enumerate(self.params):
            m = p.numel()
            if has[i]:
                g = self.flat[off:off + m].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
            off += m


def broadcast_parameters(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Make every rank start from rank ``src``'s weights."""
    if not dist.is_available() or not dist.is_initialized():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        broadcast_(t.data, src, group)
