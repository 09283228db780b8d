"""world_size = 2 gloo rehearsal of the data-parallel path (shard -> per-rank records ->
all-gather), on CPU."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pose_estimation_amd import distributed as kd


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    kd.init_from_env("gloo")
    mine = kd.bucket_shard(sizes, world, rank)
    ids = [i for v in mine.values() for i in v]
    B = 4
    R = torch.eye(3).repeat(B, 1, 1) * (rank + 1)
    t = torch.full((B, 3), float(rank))
    rec = kd.pack_records(R, t, t + 0.5, torch.full((B,), 7.0 + rank))
    allrec = kd.gather_records(rec)
    mx = kd.allreduce_max(float(rank), "cpu")
    q.put((rank, ids, allrec.tolist(), mx))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shard_and_gather():
    sizes = [80, 120, 120, 160, 80, 120, 200, 160, 120, 80, 240]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    ids = res[0][1] + res[1][1]
    assert sorted(ids) == list(range(len(sizes)))  # every crop exactly once
    for rank, _, allrec, mx in res:
        allrec = torch.tensor(allrec)
        assert allrec.shape == (world * 4, kd.RECORD)
        for r in range(world):
            blk = allrec[4 * r:4 * (r + 1)]
            assert torch.all(blk[:, 0] == r + 1) and torch.all(blk[:, 9] == r) and torch.all(blk[:, 15] == 7 + r)
        assert mx == world - 1


def test_bucket_shard_single_size_per_batch():
    sizes = [120] * 10 + [160] * 5
    a = kd.bucket_shard(sizes, 4, 0)
    assert a == {120: [0, 1, 2], 160: [10, 11]}
    assert kd.shard_range(10, 4, 3) == (8, 10)
