"""The multi-GPU path of bench.py on CPU: world-size-2 gloo run of the same shard / pose-gather /
max-over-ranks logic the driver's N>1 runs use with RCCL."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import bench  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wins = bench.shard_windows(rank, world, pipelines=3, window=8)
    poses = np.zeros((2, 3, 16), np.float32)
    for p, w in enumerate(wins):
        poses[:, p, 0] = w[0]           # tag each pose with its window's first frame
        poses[:, p, 1] = rank
    allp = bench.gather_poses(dist, poses, "cpu")
    t = bench.max_over_ranks(dist, 1.0 + rank, "cpu")
    if rank == 0:
        np.savez(os.path.join(out_dir, "r0.npz"), allp=allp, t=t,
                 wins=np.array([bench.shard_windows(r, world, 3, 8) for r in range(world)]))
    dist.destroy_process_group()


def test_two_rank_shard_gather(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = np.load(tmp_path / "r0.npz")
    allp, wins = d["allp"], d["wins"]
    assert float(d["t"]) == 2.0                                   # max over ranks
    assert allp.shape == (world * 2 * 3, 16)
    assert set(allp[:, 1].astype(int)) == {0, 1}                  # every rank's poses arrived
    # shards are disjoint, consecutive and inside the 256-frame sequence
    for r in range(world):
        for w in wins[r]:
            assert list(w) == list(range(w[0], w[0] + 8))
            assert r * 128 <= w[0] and w[-1] < (r + 1) * 128
