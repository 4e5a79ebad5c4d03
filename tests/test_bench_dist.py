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


@pytest.mark.parametrize("world", [1, 8])
@pytest.mark.parametrize("steps,P", [(10, 10), (3, 10), (1, 16), (10, 7)])
def test_stream_pieces_cover_every_step_pair_once(world, steps, P):
    """The runner's default work split (r360_sequence_run, odometry.stream_pieces): the steps x shard pairs, repeat-
    major, cut into at most P contiguous pieces of near-equal size; every (step, pair) exactly once, in order."""
    for r in range(world):
        p0, p1 = OD.shard_pairs(r, world)
        pieces = OD.stream_pieces(p0, p1, steps, P)
        assert 1 <= len(pieces) <= P
        flat = [(rep, i) for segs in pieces for rep, a, b in segs for i in range(a, b)]
        assert flat == [(rep, i) for rep in range(steps) for i in range(p0, p1)]
        sizes = [sum(b - a for _, a, b in segs) for segs in pieces]
        assert max(sizes) - min(sizes) <= 1
        for segs in pieces:
            assert all(p0 <= a < b <= p1 for _, a, b in segs)


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


class _StubCtx:
    """Context stand-in: the timing / sync calls bench.main makes on the pipelines' contexts."""

    def sync(self): pass
    def timing(self, on): pass
    def timing_reset(self): pass
    def kernel_time_reset(self): pass
    def timing_read(self, name): return 0.0, 0
    def kernel_stats(self, level): return 0.0, 0, 0
    def host_times(self, reset=False): return np.zeros(6)
    def match_stats(self): return 0, 0, 0


class _StubRunner:
    """odometry.SequenceRunner stand-in for the CPU: each pair's record is the ground-truth relative motion of the
    synthetic path (so the composed trajectory is exact), its status the rank that registered it; every pair's raw
    frames are fetched through frames_of, as the pipelines do."""

    def __init__(self, device, rows, cols, P, params, **kw):
        import rgbd360_amd as R
        self.R, self.rows, self.cols = R, rows, cols
        self.ctxs, self.queue, self.cals, self.frames = [_StubCtx() for _ in range(P)], None, [], []
        self.host_s = np.zeros((P, 4))
        self.native_ids = set()
        self.rank = int(os.environ["RANK"])

    def run(self, p0, p1, frames_of, out, repeats=1, runs=None, device_inputs=False):
        assert runs is None or (runs[0][0] == p0 and runs[-1][1] == p1)
        for i in range(p0, p1):
            for f in (i, i + 1):
                b, d = frames_of(f)
                assert b.shape == (8, self.rows, self.cols, 3) and d.shape == (8, self.rows, self.cols)
            rel = np.linalg.inv(self.R.synth_path_pose(bench.SEED, i).astype(np.float64)) @ \
                self.R.synth_path_pose(bench.SEED, i + 1).astype(np.float64)
            out[:repeats, i - p0, OD.R_POSE:OD.R_POSE + 16] = rel.T.reshape(16)
            out[:repeats, i - p0, OD.R_STATUS] = self.rank
            out[:repeats, i - p0, OD.R_SSO] = 0.8
        self.host_s[0, 3] += repeats * (p1 - p0)

    def close(self): pass


def _main_worker(rank, world, port, out_dir):
    import contextlib
    import io
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), R360_BENCH_REHEARSAL="1", R360_NO_PIN="1")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--frames", "24", "--rows", "24",
                    "--cols", "32", "--streams", "3", "--min-run", "2", "--no-cpu-baseline", "--no-resident",
                    "--no-config5", "--no-isolated"], runner_factory=_StubRunner)
    with open(os.path.join(out_dir, f"out{rank}.txt"), "w") as f:
        f.write(buf.getvalue())


@pytest.mark.parametrize("world", [2, 8])
def test_bench_main_multi_rank(tmp_path, world):
    """bench.main itself at world size 2 and 8 over gloo (R360_BENCH_REHEARSAL: records gathered by gloo instead of the
    library's RCCL communicator), with a CPU stand-in for the GPU pipelines: each rank registers only its shard,
    rank 0 gathers every rank's records, composes the whole trajectory and prints the one JSON line with the
    whole-job pair count; the other ranks print nothing.  World size 8 is the driver's 8-GPU node (one process per
    GPU, 8 shards of the 23 pairs of the 24-frame test sequence)."""
    import json
    mp.spawn(_main_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(1, world):
        assert (tmp_path / f"out{r}.txt").read_text() == ""
    lines = (tmp_path / "out0.txt").read_text().strip().splitlines()
    assert len(lines) == 1
    out = json.loads(lines[0])
    sizes = [OD.shard_pairs(r, world, 24)[1] - OD.shard_pairs(r, world, 24)[0] for r in range(world)]
    assert sum(sizes) == 23 and max(sizes) - min(sizes) <= 1
    assert out["n_gpus"] == world and out["steps"] == 2 and out["scaling"] == "strong"
    assert out["config"]["parallelism"] == f"pair-shard dp{world}"
    assert out["config"]["pairs_per_step"] == 23 and out["config"]["pairs_per_step_this_rank"] == sizes[0]
    assert out["records_identical"] is True
    tr = out["trajectory"]
    assert tr["pairs"] == 23 and tr["frames"] == 24
    # every pair composed once, in order (the floor: f32 records, arccos of a trace within 1e-7 of 3)
    assert tr["max_rot_err_deg"] < 0.05 and tr["max_trans_err_m"] < 1e-5
    # status = rank: rank 1's pairs count as PbMap failures, rank 2's as ill-posed
    assert tr["pbmap_failed"] == sizes[1] and tr["illposed"] == (sizes[2] if world > 2 else 0)
    assert out["value"] > 0 and abs(out["value"] - 46 / (out["ms_per_step"] * 2e-3)) < 1e-6 * out["value"]
    # per-rank diagnostics of the N > 1 line: shard sizes, rates, the gather's time, halo frames
    pr = out["per_rank"]
    assert [r["rank"] for r in pr] == list(range(world)) and [r["pairs_per_step"] for r in pr] == sizes
    assert all(r["pairs_per_s"] > 0 and r["gather_ms"] >= 0 and r["halo_frames_per_step"] >= 1 for r in pr)
    assert max(r["timed_s"] for r in pr) == pytest.approx(out["ms_per_step"] * 2e-3, rel=1e-5)
