"""The multi-GPU path of bench.py on CPU: the pair sharding of the 256-frame sequence for
N in {1, 2, 4, 8}, and a world-size-2 gloo run of the same record gather / max-over-ranks / trajectory
composition the driver's N>1 runs do with RCCL."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402
from rgbd360_amd import odometry as OD  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("streams,min_run", [(16, 4), (16, 1), (3, 4)])
def test_pair_partition_covers_each_pair_once(world, streams, min_run):
    seen = []
    prev_end = 0
    for r in range(world):
        p0, p1 = OD.shard_pairs(r, world)
        assert p0 == prev_end and p1 > p0                   # contiguous, non-empty, in rank order
        prev_end = p1
        P = OD.pipelines_for(p1 - p0, streams, min_run)
        runs = OD.split_range(p0, p1, P)
        assert 1 <= len(runs) <= streams
        assert runs[0][0] == p0 and runs[-1][1] == p1
        for (a, b), (c, d) in zip(runs, runs[1:]):
            assert b == c                                    # a pipeline's run starts where the previous ends
        for a, b in runs:
            assert b - a >= min(min_run, p1 - p0)            # no run shorter than asked (unless the shard is)
            seen.extend(range(a, b))
    assert prev_end == 255
    assert seen == list(range(255))                          # every pair exactly once, in order
    sizes = [OD.shard_pairs(r, world)[1] - OD.shard_pairs(r, world)[0] for r in range(world)]
    assert max(sizes) - min(sizes) <= 1


def test_compose_is_the_prefix_product():
    rng = np.random.default_rng(1)
    rec = np.zeros((5, OD.REC), np.float32)
    mats = []
    for k in range(5):
        m = np.eye(4)
        m[:3, :3] = np.linalg.qr(rng.normal(size=(3, 3)))[0]
        m[:3, 3] = rng.normal(size=3)
        mats.append(m.astype(np.float32))
        rec[k, :16] = mats[-1].T.reshape(16)
    T = OD.compose(rec)
    ref = np.eye(4)
    for k in range(5):
        ref = ref @ mats[k].astype(np.float64)
        assert np.allclose(T[k + 1], ref, atol=1e-6)
    gt = np.stack([np.eye(4)] + [T[k + 1] for k in range(5)])
    e = OD.trajectory_error(T, gt)
    assert e["max_rot_err_deg"] < 1e-4 and e["max_trans_err_m"] < 1e-9


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p0, p1 = OD.shard_pairs(rank, world)
    steps = 2
    rec = np.zeros((steps, p1 - p0, OD.REC), np.float32)
    for i in range(p0, p1):                      # each pair's record: a translation of (i + 1) mm in y
        rec[:, i - p0, :16] = np.eye(4, dtype=np.float32).T.reshape(16)
        rec[:, i - p0, 13] = 0.001 * (i + 1)
        rec[:, i - p0, OD.R_STATUS] = rank
    def allgather(a):   # the gloo transport of bench.RankGroup's rehearsal mode (RCCL on the GPU)
        t = torch.from_numpy(np.ascontiguousarray(a))
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return np.stack([o.numpy() for o in out])
    allrec, sizes = bench.gather_records(allgather, rec, -(-255 // world))
    m = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    t = float(m.item())
    if rank == 0:
        np.savez(os.path.join(out_dir, "r0.npz"), allrec=allrec, t=t, sizes=np.array(sizes),
                 traj=OD.compose(allrec[-1]))
    dist.destroy_process_group()


def test_two_rank_gather_and_trajectory(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = np.load(tmp_path / "r0.npz")
    allrec, sizes, traj = d["allrec"], d["sizes"], d["traj"]
    assert float(d["t"]) == 2.0                                   # max over ranks
    assert list(sizes) == [128, 127] and allrec.shape == (2, 255, OD.REC)
    # every pair arrived exactly once, in sequence order, from the rank that owns it
    assert np.allclose(allrec[1, :, 13], 0.001 * np.arange(1, 256))
    assert list(allrec[1, :, OD.R_STATUS]) == [0] * 128 + [1] * 127
    # rank 0's prefix product: y translations add up
    assert np.allclose(traj[-1][1, 3], 0.001 * 255 * 256 / 2, rtol=1e-6)
