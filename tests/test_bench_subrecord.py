"""bench.py's multi-GPU sub-record code path (``sub_record``) on CPU with gloo, world size 2.

The driver's N = 2/4/8 runs put the c3_dp / c5_shard sub-records beside the C2 headline; this drives the same
measurement function with a step made of the same collectives (the gradient bucket, the snapshot-shard all-to-all
and the pooling all-reduce, all on host tensors) and checks the JSON schema, the MAX-over-ranks timing and the
per-phase exchange accounting.  Also checks ``sub_records_for`` (which sub-records each N gets).
"""
import json
import os
import socket

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
    import bench
    from tagan_amd.distributed import GradBucket
    from tagan_amd.sharded import ShardGradSync, _all_reduce_sum, _all_to_all
    torch.manual_seed(rank)
    model = torch.nn.Sequential(torch.nn.Linear(8, 8), torch.nn.Linear(8, 2))
    bucket = GradBucket(model.parameters())
    sync = ShardGradSync(list(model.named_parameters()), replicated_prefixes=("1.",))
    calls = {"n": 0}

    def step():
        calls["n"] += 1
        x = torch.randn(4, 8)
        model.zero_grad(set_to_none=True)
        model(x).sum().backward()
        bucket.allreduce_mean()                       # phase grad_allreduce
        _all_to_all(list(x.split([2, 2])), [(2, 8), (2, 8)], None)   # phase all_to_all
        _all_reduce_sum(torch.ones(3), None)          # phase pool_allreduce
        if rank == 1:
            import time
            time.sleep(0.02)                          # the slower rank sets the wall time
        sync.sync(static=True)                        # phase grad_allreduce again (capturable form)

    rec = bench.sub_record("toy", step, world, None, steps=4, warmup=2, snapshots_per_step=10,
                           extra={"parallelism": "dp%d" % world, "n_ranks_rccl": 0})
    results[rank] = json.dumps(rec)
    results["calls%d" % rank] = calls["n"]
    dist.barrier()
    dist.destroy_process_group()


def test_sub_record_gloo_world2():
    port = _free_port()
    with mp.Manager() as m:
        res = m.dict()
        mp.spawn(_worker, args=(2, port, res), nprocs=2, join=True)
        res = dict(res)
    r0, r1 = json.loads(res[0]), json.loads(res[1])
    assert res["calls0"] == res["calls1"] == 6                # 2 warm-up + 4 timed
    assert r0["ms_per_step"] == r1["ms_per_step"]             # MAX over ranks: the same on every rank
    assert r0["ms_per_step"] >= 20.0                          # at least rank 1's sleep per step
    assert abs(r0["value"] - 10 * 4 / (r0["ms_per_step"] * 4 / 1e3)) / r0["value"] < 1e-2
    for k in ("workload", "value", "unit", "ms_per_step", "steps", "warmup", "n_ranks", "exchange_ms_per_step",
              "parallelism", "n_ranks_rccl"):
        assert k in r0, k
    ex = r0["exchange_ms_per_step"]
    assert set(ex) == {"grad_allreduce", "all_to_all", "pool_allreduce"}, ex
    assert all(v >= 0.0 for v in ex.values())
    assert r0["steps"] == 4 and r0["warmup"] == 2 and r0["n_ranks"] == 2


def test_sub_records_for():
    import bench
    assert bench.sub_records_for("auto", 1) == []
    assert bench.sub_records_for("auto", 2) == ["c3_dp"]
    assert bench.sub_records_for("auto", 4) == ["c3_dp"]
    assert bench.sub_records_for("auto", 8) == ["c5_shard"]
    assert bench.sub_records_for("none", 8) == []
    assert bench.sub_records_for("c3_dp,c5_shard", 1) == ["c3_dp", "c5_shard"]
