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


class _FakeSet:
    """Stands in for PoseDataset in the sharded-epoch rehearsal: crop sizes, objects, diameters."""
    objlist = [1, 2, 4, 5, 6, 8, 9, 10, 11, 12, 13, 14, 15]
    sym_obj = [7, 8]

    def __init__(self, n):
        g = torch.Generator().manual_seed(0)
        self.sizes = [int(s) for s in (torch.randint(1, 6, (n,), generator=g) * 40)]
        self.diameter = [0.1 + 0.01 * i for i in range(len(self.objlist))]

    def __len__(self):
        return len(self.sizes)

    def crop_size(self, i):
        return self.sizes[i]


def _fake_records(model, dataset, indices, bs, device, opt_pose=True, with_loss=True):
    """Deterministic per-crop records (a function of the crop id only), in evaluation order."""
    from pose_estimation_amd import evaluate as ev
    rows = []
    for S, idx in ev._batches(indices, bs):
        for i in idx:
            g = torch.Generator().manual_seed(1000 + i)
            r = torch.rand(len(ev.REC), generator=g, dtype=torch.float64)
            r[ev._R["crop"]] = i
            r[ev._R["cls"]] = i % len(dataset.objlist)
            r[ev._R["add_b"]] *= 0.03
            r[ev._R["add_f"]] *= 0.03
            r[ev._R["r_b"]] *= 10
            r[ev._R["r_f"]] *= 10
            r[ev._R["t_b"]] *= 0.1
            r[ev._R["t_f"]] *= 0.1
            r[ev._R["valid"]] = 1.0
            rows.append(r)
    return torch.stack(rows) if rows else torch.zeros((0, len(ev.REC)), dtype=torch.float64)


def _epoch_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from pose_estimation_amd import evaluate as ev
    ev.eval_records = _fake_records
    kd.init_from_env("gloo")
    out = ev.test_epoch(None, _FakeSet(n), bs=4, device="cpu")
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_epoch_matches_single():
    """The sharded test_epoch (bucket_shard -> per-rank records -> all-gather -> fold in global
    crop order, plus the all_reduce tally check) gives the world-1 result exactly."""
    from pose_estimation_amd import evaluate as ev
    n = 37
    saved = ev.eval_records
    ev.eval_records = _fake_records
    try:
        ref = ev.test_epoch(None, _FakeSet(n), bs=4, device="cpu", world=1, rank=0)
    finally:
        ev.eval_records = saved
    assert ref["test_count"] == n
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_epoch_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, out in res:
        assert out == ref
