"""The C++ drivers over the façade (apps/, built by __graft_entry__.build() into build/bin) run end to end on
the GPU: OdometryRGBD360 (Registration/OdometryRGBD360.cpp loop) and SphereGraphTracking (the tracking +
loop-closure front end of SLAM/SphereGraphSLAM.cpp over BatchRegistration), on the synthetic sequence."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")


def _run(name, *args):
    exe = os.path.join(BIN, name)
    assert os.path.exists(exe), f"{exe} missing: run __graft_entry__.build()"
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr + p.stdout[-2000:]
    return p.stdout


def test_sphere_graph_tracking_synthetic():
    out = _run("SphereGraphTracking", "--synthetic", "10")
    m = re.search(r"(\d+) keyframes, (\d+) loop-closure edges", out)
    assert m, out
    assert int(m.group(1)) == 10                     # every frame of the smooth path tracks
    assert out.count("Good TRACKING") == 9


def test_odometry_synthetic():
    out = _run("OdometryRGBD360", "--synthetic", "4")     # frames 1..3 of the path (first = 1)
    assert "3 keyframes" in out and out.count("PbMap ok") == 2, out
