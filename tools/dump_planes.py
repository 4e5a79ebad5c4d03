"""Dump the GPU plane-half intermediates of the sample frames (debug aid): gpurun_out/planes_dump.npz"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rgbd360_amd as R

ctx = R.Context(0)
cal = R.Calib360(ctx, 240, 320)
cal.loadExtrinsicCalibration(R.EXTRINSICS_DIR)
cal.loadIntrinsicCalibration(R.INTRINSICS_DIR)
f = R.Frame360(cal)
f.loadFrame(os.path.join(R.SAMPLES_DIR, "sphere_images_1.bin"))
f.build(R.BUILD_UNDISTORT | R.BUILD_PLANES)
xyz, rgb, nrm, dist = f.cloud()
lab, labf = f.labels()
regs = [f.regions(k) for k in range(8)]
np.savez_compressed("gpurun_out/planes_dump.npz", xyz=xyz, nrm=nrm, lab=lab, labf=labf,
                    models=np.array([[r["model"] for r in rr] + [np.zeros(4)] * (64 - len(rr)) for rr in regs]),
                    nreg=np.array([len(rr) for rr in regs]))
print("ok", [len(r) for r in regs])
