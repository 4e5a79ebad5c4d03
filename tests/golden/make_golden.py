"""Generate the oracle regression fixtures under tests/golden/ (run from the repo root):

    python tests/golden/make_golden.py

The reference ships no golden outputs; these fixtures are the CPU oracle's
own outputs on the reference's sample pair (data/samples/sphere_images_{1,10}.bin, real QVGA
captures + the reference rig's Rt_0k.txt and CLAMS models), so any change to the restatement is
diffable.  They pin the oracle against itself, not against the (unbuildable) reference.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle360 as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def sample_inputs():
    d = os.path.join(ROOT, "data")
    b1, d1 = O.load_bin(os.path.join(d, "samples", "sphere_images_1.bin"))
    b2, d2 = O.load_bin(os.path.join(d, "samples", "sphere_images_10.bin"))
    rt = O.read_extrinsics(os.path.join(d, "calib", "Extrinsics"))
    rti = np.concatenate([O.mat16(np.linalg.inv(r.astype(np.float64))) for r in rt]).astype(np.float32)
    K = O.camera_matrix(240, 320)
    return b1, d1, b2, d2, rt, rti, K


POSES = [np.eye(4, dtype=np.float32),
         O.exp_se3([0.02, -0.03, 0.05, 0.01, -0.015, 0.02]),
         O.exp_se3([-0.05, 0.04, -0.02, -0.03, 0.02, 0.01])]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    b1, d1, b2, d2, rt, rti, K = sample_inputs()
    s1b, s1d = O.stitch(b1, d1, rti, K)
    s2b, s2d = O.stitch(b2, d2, rti, K)
    clams = [O.Clams(os.path.join(ROOT, "data", "calib", "Intrinsics", f"distortion_model{k + 1}.r360"))
             for k in range(8)]
    und = np.stack([clams[k].undistort(O.depth_to_m(d1[k])) for k in range(8)])
    lt = O.sphere_pyramid(s1b, s1d, 5)
    ls = O.sphere_pyramid(s2b, s2d, 5)
    out = dict(rti=rti, K=K,
               sph1_sha=sha(s1b) + sha(s1d), sph2_sha=sha(s2b) + sha(s2d),
               und1_sha=sha(und), und1_sample=und[:, ::17, ::13])
    for l in (3, 4):
        for k in ("gray", "depth", "gx", "gy", "dgx", "dgy"):
            out[f"t{l}_{k}"] = lt[l][k]
            out[f"s{l}_{k}"] = ls[l][k]
        for m in (0, 1, 2):
            for i, P in enumerate(POSES):
                e, e2, nv = O.error_sphere(ls[l], lt[l], P, m)
                H, g, nvis = O.hessgrad_sphere(ls[l], lt[l], P, m)
                out[f"icp{l}_{m}_{i}"] = np.concatenate([[e, e2, nv, nvis], g, H.ravel()])
    p = O.IcpParams.default(n_pyr=5, std_dev_photo=np.float32(3.0 / 255))
    rc, pose, H, g, st = O.align360(s1b, s1d, s2b, s2d, None, O.PHOTO_DEPTH, p)
    out["align_pose"] = pose
    out["align_iters"] = np.array(list(st.iters)[:5])
    out["align_H"] = H
    out["poses"] = np.stack(POSES)
    np.savez_compressed(os.path.join(OUT, "oracle_samples.npz"), **out)
    print("wrote", os.path.join(OUT, "oracle_samples.npz"), "iters", out["align_iters"])


if __name__ == "__main__":
    main()
