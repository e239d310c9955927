"""A whole TAGAN training step as ONE replayable HIP graph.

The reference trainer's step (trainer.py:295-311: forward, loss, backward, clip_grad_norm_, optimizer step)
issues ~300 launches per C2 sequence from Python: at C2 bf16 and at C1 the host, not the GPU, sets the pace
(DESIGN.md §4).  ``GraphedStep`` captures the step once with ``torch.cuda.graph`` and replays it: the CSR
build, both attention stacks, the fused head + loss, their backward passes, the gradient all-reduce (N > 1:
the RCCL collective is captured into the same graph), clipping and Adam all run from one ``hipGraphLaunch``.

What capture needs from the hot path, and how it gets it:
* fresh dropout masks per replay — the seeds drawn at capture time are constants in the graph, so the step
  first advances a device counter (``tagan_seed_counter_step``) that every dropout kernel mixes into its seed
  at run time (``tagan_set_seed_counter``, include/tagan_hip.h);
* no host synchronisation inside the step — the edge-index validation is switched off for the captured step
  (``model.validate_edges = False``; the inputs are static and were validated by the eager warm-up), and the
  gradient bucket runs in its static form (``GradBucket.allreduce_mean(static=True)``);
* static inputs — the replay re-runs the step on the same input tensors (the bench's resident sequence);
  a caller feeding new data copies it into those tensors before ``__call__``;
* device tables the graph reads by address stay alive — the snapshot offset tables cached by
  ``kernels._ptr_table`` are pinned when they are looked up during a capture;
* a capturable optimizer (``torch.optim.Adam(..., capturable=True)``).

There is deliberately no split form (an eager segment between two captured ones): DESIGN.md §6 records how
that form faulted and why the collective lives inside the one graph instead.
"""
import ctypes
from typing import Callable

import torch

from ._lib import check, lib, ptr


def _nccl_live() -> bool:
    """A process group with an RCCL ("nccl") backend is initialised (its watchdog thread polls work events)."""
    from .distributed import nccl_groups
    return bool(nccl_groups())


class GraphedStep:
    """``step_fn()`` (no ``zero_grad`` inside: gradients are written, not accumulated, by the captured backward)
    captured after ``warmup`` eager calls on a side stream; ``__call__`` replays it and returns the static loss."""

    def __init__(self, model: torch.nn.Module, step_fn: Callable[[], torch.Tensor], optimizer=None, warmup: int = 3,
                 **unsupported):
        if unsupported:
            raise TypeError("GraphedStep captures the whole step as one graph; unsupported arguments: %s"
                            % sorted(unsupported))
        dev = next(model.parameters()).device
        self.model, self.dev = model, dev
        self.prev_validate = getattr(model, "validate_edges", None)
        if self.prev_validate is not None:
            model.validate_edges = False
        self.counter = torch.zeros(1, dtype=torch.int64, device=dev)
        lib().tagan_set_seed_counter(ptr(self.counter))
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                if optimizer is not None:
                    optimizer.zero_grad(set_to_none=True)
                step_fn()
        torch.cuda.current_stream(dev).wait_stream(side)
        if optimizer is not None:
            optimizer.zero_grad(set_to_none=True)
        if _nccl_live():
            # the warm-up steps' collectives ran on `side` and recorded their end events there; the RCCL watchdog
            # polls those events until it retires their Works, and a poll of an event whose recording stream is
            # capturing fails (hipErrorCapturedEvent) and aborts the process.  Wait until the watchdog's lists are
            # empty before `side` starts capturing (distributed.py).
            from .distributed import EVENT_CACHE_ENV, graph_safe_groups, retire_pending_works
            if not graph_safe_groups():
                raise RuntimeError("GraphedStep with a live RCCL process group needs the group built with the event "
                                   "cache off: create it through tagan_amd.distributed.init_process_group, or export "
                                   "%s=0 before dist.init_process_group" % EVENT_CACHE_ENV)
            retire_pending_works(dev)
        self.graph = torch.cuda.CUDAGraph()
        # captured on the warm-up stream: autograd nodes that outlive a warm-up step (a loss the caller kept,
        # AccumulateGrad nodes) then belong to the capture stream, so the backward adds no cross-stream join.
        # thread_local capture: another thread's runtime calls during the capture (the RCCL process group's
        # watchdog polling its work events) must not invalidate it -- under the default "global" mode such a
        # poll aborted the process mid-capture when a process group was live
        with torch.cuda.graph(self.graph, stream=side, capture_error_mode="thread_local"):
            s = torch.cuda.current_stream(dev)
            check(lib().tagan_seed_counter_step(ptr(self.counter), ctypes.c_void_p(s.cuda_stream)),
                  "tagan_seed_counter_step")
            self.loss = step_fn()

    def __call__(self) -> torch.Tensor:
        self.graph.replay()
        return self.loss

    def close(self) -> None:
        """Unregister the seed counter (eager launches use their seeds as passed again) and destroy the graph now
        (not at garbage collection): a captured RCCL collective must not outlive its process group."""
        lib().tagan_set_seed_counter(None)
        if self.prev_validate is not None:
            self.model.validate_edges = self.prev_validate
        if self.graph is not None:
            torch.cuda.synchronize(self.dev)
            self.graph.reset()
        self.graph = None
        self.loss = None   # releases the captured step's autograd graph (its AccumulateGrad nodes)
