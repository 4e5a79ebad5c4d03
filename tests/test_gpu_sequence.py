"""BASELINE config 4 on one GPU: OdometryRGBD360 over the synthetic 256-frame sequence, sharded by pair
(rgbd360_amd/odometry.py, the bench's default workload).

* the first 16 pairs of the pipelined run equal the oracle chain (PbMap -> RegisterPbMap -> rotOffset
  conjugation -> alignFrames360 with the bench's 20 level-0 iterations) to the north-star tolerance;
* the records of all 255 pairs do not depend on how the pairs are sharded (ranks x pipelines): the N = 2 and
  N = 8 rank shards, each run alone, reproduce the single-GPU run bit for bit;
* the composed trajectory follows the synthetic ground truth (synth_path_pose)."""
import numpy as np
import pytest

import rgbd360_amd as R
from rgbd360_amd import odometry as OD

pytestmark = pytest.mark.gpu

SEED = 360 << 16


@pytest.fixture(scope="module")
def seq():
    rt8 = np.stack([np.loadtxt(f"{R.EXTRINSICS_DIR}/Rt_0{k + 1}.txt", dtype=np.float32) for k in range(8)])
    bgr = np.zeros((256, 8, 480, 640, 3), np.uint8)
    dep = np.zeros((256, 8, 480, 640), np.uint16)
    for i in range(256):
        bgr[i], dep[i] = R.synth_frame_rt(480, 640, rt8, SEED, R.synth_path_pose(SEED, i))
    pin = R.HostPinned(bgr, dep)
    p = R.IcpParams.default()
    p.n_pyr = 5
    p.std_dev_photo = np.float32(3.0 / 255)
    p.fixed_iters_level0 = 20
    # dense stages batched on a dense queue, plane stages on the pipelines' own streams
    runner = OD.SequenceRunner(0, 480, 640, 16, p, queue=16, plane_batch=0)
    rec = np.zeros((1, 255, OD.REC), np.float32)
    runner.run(0, 255, lambda i: (bgr[i], dep[i]), rec)
    yield dict(bgr=bgr, dep=dep, runner=runner, rec=rec[0], params=p, rt8=rt8)
    runner.close()
    pin.close()


def test_first_pairs_match_oracle_chain(seq):
    from oracle import oracle360 as O
    bgr, dep, rec = seq["bgr"], seq["dep"], seq["rec"]
    cal = seq["runner"].cals[0]
    rt, rti, K = cal.extrinsics()
    Km = K.reshape(3, 3).T
    rt8 = np.stack([rt[16 * k:16 * k + 16].reshape(4, 4).T for k in range(8)])
    prm = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255), fixed_iters_level0=20)
    Ro = OD.ROT_OFFSET.astype(np.float32)
    Ri = OD.ROT_OFFSET_INV.astype(np.float32)

    def build(i):
        sb, sd = O.stitch(bgr[i], dep[i], rti, Km)
        return sb, sd, O.PbMap(dep[i].astype(np.float32) * np.float32(0.001), bgr[i], rt8)

    prev = build(0)
    for i in range(16):
        cur = build(i + 1)
        r = O.register_pbmap(prev[2], cur[2], 25, O.PLANAR_3DoF)
        assert r["good"] == (rec[i, OD.R_STATUS] == 0), i
        init = Ro @ (r["pose"] if r["good"] else np.eye(4, dtype=np.float32)) @ Ri
        _, dense, _, _, _ = O.align360(prev[0], prev[1], cur[0], cur[1], init, O.PHOTO_DEPTH, prm)
        ref = Ri.astype(np.float64) @ dense.astype(np.float64) @ Ro.astype(np.float64)
        pose = rec[i, :16].reshape(4, 4).T
        assert O.rot_angle(pose[:3, :3], ref[:3, :3]) <= 1e-4, i
        assert np.linalg.norm(pose[:3, 3] - ref[:3, 3]) <= 1e-3, i
        prev = cur


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_runs_reproduce_the_single_gpu_records(seq, world):
    bgr, dep = seq["bgr"], seq["dep"]
    runner = seq["runner"]
    parts = []
    for r in range(world):
        p0, p1 = OD.shard_pairs(r, world)
        runs = OD.split_range(p0, p1, OD.pipelines_for(p1 - p0, 16, 4))
        out = np.zeros((1, p1 - p0, OD.REC), np.float32)
        runner.run(p0, p1, lambda i: (bgr[i], dep[i]), out, runs=runs)
        parts.append(out[0])
    assert np.array_equal(np.concatenate(parts), seq["rec"])


def test_device_resident_inputs_give_the_same_records(seq):
    bgr, dep = seq["bgr"], seq["dep"]
    dB, dD = R.DeviceArray(0, bgr[:33]), R.DeviceArray(0, dep[:33])
    out = np.zeros((1, 32, OD.REC), np.float32)
    seq["runner"].run(0, 32, lambda i: (dB.ptr(i), dD.ptr(i)), out, device_inputs=True)
    dB.close()
    dD.close()
    assert np.array_equal(out[0], seq["rec"][:32])


def test_rccl_comm_single_rank():
    """The record gather's RCCL path (r360_comm) with one rank: all_gather returns the rank's own buffer,
    the max is the value (multi-rank RCCL needs one GPU per rank: exercised by the driver's N > 1 runs)."""
    c = R.Comm(0, 1, 0, R.Comm.unique_id())
    a = np.arange(3 * 5 * 56, dtype=np.float32).reshape(3, 5, 56)
    assert np.array_equal(c.allgather(a), a[None])
    assert c.allreduce_max(2.5) == 2.5
    c.close()


def test_trajectory_follows_ground_truth(seq):
    rec = seq["rec"]
    assert (rec[:, OD.R_STATUS] == 0).all()                   # every PbMap stage succeeded, none ill-posed
    gt = np.stack([R.synth_path_pose(SEED, k).astype(np.float64) for k in range(256)])
    # every pair: the relative pose of the synthetic path
    for i in range(255):
        rel = np.linalg.inv(gt[i]) @ gt[i + 1]
        pose = rec[i, :16].reshape(4, 4).T.astype(np.float64)
        D = np.linalg.inv(rel) @ pose
        assert np.degrees(np.arccos(np.clip((np.trace(D[:3, :3]) - 1) / 2, -1, 1))) < 0.2, i
        assert np.linalg.norm(pose[:3, 3] - rel[:3, 3]) < 0.02, i
    e = OD.trajectory_error(OD.compose(rec), gt)
    print(e)
    # drift of the composed odometry over the closed 256-frame loop
    assert e["max_rot_err_deg"] < 2.0 and e["max_trans_err_m"] < 0.02 * e["path_length_m"], e


def test_plane_queue_reproduces_the_records(seq):
    """The same 255 pairs with the plane stages batched on a plane queue (up to 8 frames per launch, two streams):
    every record is bit-identical to the run with plane stages on the pipelines' own streams."""
    bgr, dep = seq["bgr"], seq["dep"]
    runner = OD.SequenceRunner(0, 480, 640, 16, seq["params"], queue=16)
    try:
        rec = np.zeros((1, 255, OD.REC), np.float32)
        runner.run(0, 255, lambda i: (bgr[i], dep[i]), rec)
        st = runner.queue.stats()
        pst = runner.plane_stats()
    finally:
        runner.close()
    assert st["jobs"] == 255 and st["batches"] < 255
    assert pst["frames"] >= 256 and pst["batches"] < pst["frames"]
    assert np.array_equal(rec[0], seq["rec"])


def test_unqueued_lone_alignments_match_the_records(seq):
    """Without the dense queue every pair is a lone alignFrames360 (r360_register_async, the sequential callers'
    path: two workgroups per CU against the batched grid's one, PF 5 over compacted points against the batched image
    streams), so the records equal the queued run's to rounding: the same PbMap stages, and poses within 2e-5 rad /
    2e-4 m where every Gauss-Newton decision is the same.  A decision at a rounding edge can flip (one iteration more
    or less at a level): such pairs are rare (at most 5 %) and stay within the north-star bar (1e-4 rad / 1e-3 m)."""
    import json
    import os
    from oracle import oracle360 as O
    bgr, dep = seq["bgr"], seq["dep"]
    runner = OD.SequenceRunner(0, 480, 640, 16, seq["params"], plane_batch=0)
    try:
        rec = np.zeros((1, 255, OD.REC), np.float32)
        runner.run(0, 255, lambda i: (bgr[i], dep[i]), rec)
    finally:
        runner.close()
    ref = seq["rec"]
    assert np.array_equal(rec[0][:, OD.R_STATUS], ref[:, OD.R_STATUS])
    assert np.array_equal(rec[0][:, 16:52], ref[:, 16:52])          # the PbMap information matrices
    dr, dt = [], []
    for i in range(255):
        a, b = rec[0][i, :16].reshape(4, 4).T, ref[i, :16].reshape(4, 4).T
        dr.append(O.rot_angle(a[:3, :3], b[:3, :3]))
        dt.append(float(np.linalg.norm(a[:3, 3] - b[:3, 3])))
    dr, dt = np.array(dr), np.array(dt)
    out = os.environ.get("R360_TEST_DRIFT_OUT")
    if out:
        with open(f"{out}_sequence.json", "w") as fo:
            json.dump({"max_rot_rad": float(dr.max()), "max_trans_m": float(dt.max()),
                       "beyond_rounding": int(((dr > 2e-5) | (dt > 2e-4)).sum()), "pairs": 255}, fo)
    assert dr.max() <= 1e-4 and dt.max() <= 1e-3, (dr.max(), dt.max())
    assert ((dr > 2e-5) | (dt > 2e-4)).sum() <= 13, np.flatnonzero((dr > 2e-5) | (dt > 2e-4))


def test_single_pipeline_latency_path_equals_the_pipelined_lone_path(seq):
    """One pipeline without a dense queue is the sequential caller's configuration (bench.sequential_leg): its context
    waits for each new frame's PbMap by assembling it itself (join_help), uploads the depth images before the BGR
    images on a second stream (split_upload) and replays the plane stage as two graphs around the BGR wait.  None of
    that may change a record: the registrations equal those of 16 pipelines doing the same lone Register() calls with
    the plane stage launched kernel by kernel, bit for bit."""
    bgr, dep = seq["bgr"], seq["dep"]
    recs = []
    for P in (1, 16):
        runner = OD.SequenceRunner(0, 480, 640, P, seq["params"], queue=0, plane_batch=0)
        try:
            rec = np.zeros((1, 48, OD.REC), np.float32)
            runner.run(0, 48, lambda i: (bgr[i], dep[i]), rec)
            recs.append(rec[0])
        finally:
            runner.close()
    assert np.array_equal(recs[0], recs[1])


def test_bench_runner_mode_reproduces_the_records(seq):
    """The mode the headline bench line runs in (bench.py defaults: 12 pipelines, dense queue batches of 16, 3
    alignments in flight per pipeline, 1 frame built ahead, plane stages batched 8 frames per launch, runs=None: the
    repeats x 255 registrations cut into 12 contiguous pieces that cross repeat boundaries): every repeat's records
    equal the single-run records bit for bit, so no pair at a piece's repeat boundary takes a wrong frame buffer."""
    bgr, dep = seq["bgr"], seq["dep"]
    runner = OD.SequenceRunner(0, 480, 640, 12, seq["params"], queue=16, depth=3, lookahead=1, plane_batch=8)
    try:
        rec = np.zeros((3, 255, OD.REC), np.float32)
        runner.run(0, 255, lambda i: (bgr[i], dep[i]), rec, repeats=3)
        pieces = OD.stream_pieces(0, 255, 3, 12)
    finally:
        runner.close()
    # the cut really crosses repeat boundaries (pieces with segments of two repeats)
    assert sum(len(p) > 1 for p in pieces) >= 2
    for r in range(3):
        bad = np.nonzero((rec[r] != seq["rec"]).any(axis=1))[0]
        assert len(bad) == 0, (r, bad[:16].tolist())


def test_failed_pipeline_drains_its_tickets(seq):
    """A pipeline step that fails (here: a frame with null image pointers) collects every alignment it still had in
    flight before the run returns its error, so the dense queue holds no job over the pipeline's frames: the next run
    on the same runner reproduces the records and destroying the runner afterwards is clean."""
    bgr, dep = seq["bgr"], seq["dep"]
    runner = OD.SequenceRunner(0, 480, 640, 4, seq["params"], queue=16, depth=3, lookahead=1)
    try:
        out = np.zeros((1, 40, OD.REC), np.float32)
        with pytest.raises(RuntimeError, match="null arg"):
            runner.run(0, 40, lambda i: (None, None) if i == 27 else (bgr[i], dep[i]), out)
        q = runner.queue.stats()
        rec = np.zeros((1, 40, OD.REC), np.float32)
        runner.run(0, 40, lambda i: (bgr[i], dep[i]), rec)
        assert runner.queue.stats()["jobs"] == q["jobs"] + 40
        assert np.array_equal(rec[0], seq["rec"][:40])
    finally:
        runner.close()


@pytest.mark.parametrize("depth,lookahead", [(3, 1), (2, 2)])
def test_queued_repeats_as_one_stream(seq, depth, lookahead):
    """Queued pipelines run their repeats as one stream of frames (a repeat's first frame is built while the
    previous repeat's last alignments are in flight; buffers are refilled only after every pair that used them is
    collected): short runs (the 1/8-shard shape, 6-7 pairs per pipeline) repeated three times give every repeat's
    records bit-identical to the single-GPU run's."""
    bgr, dep = seq["bgr"], seq["dep"]
    p0, p1 = OD.shard_pairs(7, 8)
    runs = OD.split_range(p0, p1, 5)
    runner = OD.SequenceRunner(0, 480, 640, 5, seq["params"], queue=16, depth=depth, lookahead=lookahead)
    try:
        rec = np.zeros((3, p1 - p0, OD.REC), np.float32)
        runner.run(p0, p1, lambda i: (bgr[i], dep[i]), rec, repeats=3, runs=runs)
    finally:
        runner.close()
    ref = seq["rec"][p0:p1]
    for r in range(3):
        bad = []
        for i in range(p1 - p0):
            d = np.nonzero(rec[r, i] != ref[i])[0]
            if len(d):
                bad.append((i, int((d < 16).sum()), int(((d >= 16) & (d < 52)).sum()), [int(k) for k in d[d >= 52]]))
        assert not bad, (r, "pair, pose fields, info fields, other fields", bad[:8])


@pytest.mark.parametrize("run_len", [1, 2])
def test_short_runs_sharing_edges_do_not_deadlock(seq, run_len):
    """Runs of at most `depth` pairs sharing their edge frames, repeated: a pipeline collects its previous repeat's
    pairs (whose last releases its right neighbour's edge frame) before it waits for that neighbour's rebuild of the
    edge, so neither waits on the other; every repeat reproduces the single-GPU records."""
    bgr, dep = seq["bgr"], seq["dep"]
    p0 = 40
    runs = [(p0 + k * run_len, p0 + (k + 1) * run_len) for k in range(4)]
    p1 = runs[-1][1]
    runner = OD.SequenceRunner(0, 480, 640, 4, seq["params"], queue=16, depth=3)
    try:
        rec = np.zeros((3, p1 - p0, OD.REC), np.float32)
        runner.run(p0, p1, lambda i: (bgr[i], dep[i]), rec, repeats=3, runs=runs)
    finally:
        runner.close()
    for r in range(3):
        assert np.array_equal(rec[r], seq["rec"][p0:p1]), r
