"""Data-parallel gradient exchange (tagan_amd.distributed) on CPU with gloo, world_size 2.

The GPU path runs the same code over RCCL (backend "nccl"); the collective
pattern — one flat fp32 bucket, SUM then /world — is backend independent.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import tagan_amd  # noqa: F401
    from tagan_amd.distributed import GradBucket, broadcast_parameters
    torch.manual_seed(100 + rank)                         # ranks start different ...
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3), torch.nn.Linear(3, 2))
    broadcast_parameters(model)                           # ... and are synchronised from rank 0
    for p in model.parameters():
        results["w%d" % rank] = torch.cat([q.detach().flatten() for q in model.parameters()])
    x = torch.randn(4, 6, generator=torch.Generator().manual_seed(rank))
    loss = model[:2](x).sum()                            # last layer unused -> grad None on every rank
    loss.backward()
    local = torch.cat([p.grad.flatten() for p in model.parameters() if p.grad is not None])
    results["local%d" % rank] = local.clone()
    GradBucket(model.parameters()).allreduce_mean()
    results["avg%d" % rank] = torch.cat([p.grad.flatten() for p in model.parameters() if p.grad is not None])
    results["none%d" % rank] = [p.grad is None for p in model.parameters()]
    dist.barrier()
    dist.destroy_process_group()


def test_grad_bucket_allreduce_world2():
    port = _free_port()
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(2, port, res), nprocs=2, join=True)
        res = dict(res)
    assert torch.equal(res["w0"], res["w1"])
    want = (res["local0"] + res["local1"]) / 2
    assert torch.allclose(res["avg0"], want, atol=1e-7)
    assert torch.equal(res["avg0"], res["avg1"])
    assert res["none0"] == res["none1"] == [False, False, False, False, True, True]


def _worker_uneven(rank, world, port, results):
    """A parameter with a grad on rank 0 only: same bucket layout on both ranks, mean over ranks."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import tagan_amd  # noqa: F401
    from tagan_amd.distributed import GradBucket
    from tagan_amd.kernels import new_seed
    torch.manual_seed(0)
    a, b = torch.nn.Linear(3, 2), torch.nn.Linear(2, 2)
    x = torch.ones(1, 3) * (rank + 1)
    y = a(x)
    if rank == 0:
        y = b(y)
    y.sum().backward()
    results["b%d" % rank] = b.weight.grad.clone() if b.weight.grad is not None else None
    GradBucket(list(a.parameters()) + list(b.parameters())).allreduce_mean()
    results["a_avg%d" % rank] = a.weight.grad.clone()
    results["b_avg%d" % rank] = b.weight.grad.clone()
    torch.manual_seed(5)                      # identical generators on every rank ...
    results["seed%d" % rank] = new_seed()     # ... still give per-rank dropout seeds
    dist.barrier()
    dist.destroy_process_group()


def test_grad_bucket_grad_on_one_rank_only():
    port = _free_port()
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker_uneven, args=(2, port, res), nprocs=2, join=True)
        res = dict(res)
    assert res["b1"] is None and res["b0"] is not None
    assert torch.allclose(res["b_avg0"], res["b0"] / 2) and torch.equal(res["b_avg0"], res["b_avg1"])
    assert torch.equal(res["a_avg0"], res["a_avg1"])
    assert res["seed0"] != res["seed1"]


def _guard_worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.pop("TORCH_NCCL_CUDA_EVENT_CACHE", None)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import tagan_amd.distributed as D
    dist.init_process_group("gloo", rank=rank, world_size=world)   # built by the caller, cache env not set
    results["before%d" % rank] = D.graph_safe_groups()
    D.graph_safe_env()                                             # too late for the group that exists
    results["late%d" % rank] = D.graph_safe_groups()
    dist.destroy_process_group()


def test_graph_safe_guard_states(monkeypatch):
    """the capture guard accepts a caller-exported TORCH_NCCL_CUDA_EVENT_CACHE=0 and refuses a group that
    existed before graph_safe_env() set it; retire_pending_works names a torch without _wait_for_pending_works."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import tagan_amd.distributed as D
    monkeypatch.setattr(D, "_graph_safe_groups", False)
    monkeypatch.setattr(D, "_cache_on_group", False)
    monkeypatch.setenv(D.EVENT_CACHE_ENV, "0")
    assert D.graph_safe_groups()                 # exported by the caller, no graph_safe_env() call
    monkeypatch.delenv(D.EVENT_CACHE_ENV)
    assert not D.graph_safe_groups()
    monkeypatch.setattr(D, "nccl_groups", lambda: [object()])
    with pytest.raises(RuntimeError, match="_wait_for_pending_works"):
        D.retire_pending_works()
    results = mp.Manager().dict()
    mp.spawn(_guard_worker, args=(2, _free_port(), results), nprocs=2, join=True)
    for r in range(2):
        assert results["before%d" % r] is False
        assert results["late%d" % r] is False
