"""examples/triangle.c: the reference's triangle frame driven from plain C through
include/zenith_raster.h (no Python in the loop).  CPU: it compiles and links
against libzenith_raster.  GPU: its frame equals the oracle's."""
import os
import subprocess

import numpy as np
import pytest

from zenith_amd import zr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(tmp_path):
    exe = str(tmp_path / "triangle_c")
    libdir = os.path.dirname(zr.LIB_PATH)
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "triangle.c"), "-L", libdir, "-lzenith_raster",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe


def test_c_example_builds(tmp_path):
    assert os.access(build(tmp_path), os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("t", [0.0, 1.25])
def test_c_example_frame(tmp_path, t):
    from oracle import oracle
    from zenith_amd import scenes
    out = str(tmp_path / "frame.bgra")
    r = subprocess.run([build(tmp_path), out, str(t)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "38400 covered pixels" in r.stdout
    img = np.fromfile(out, dtype=np.uint8).reshape(480, 640, 4)
    ref, _ = oracle.render(scenes.triangle_scene(time=t))
    assert np.array_equal(img, ref)
