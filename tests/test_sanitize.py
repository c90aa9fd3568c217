"""Host AddressSanitizer + UndefinedBehaviorSanitizer builds.

CPU only (no GPU code is sanitized: the device side stays as built):
- the oracle (oracle/zr_oracle.c) with gcc, driven by oracle/san_driver.c over
  scenes that cover every program, indexed / non-indexed / u16 draws,
  instancing, out-of-range indices, clipping and tile-row shards; each frame
  must equal the unsanitized oracle's;
- the runtime's host code (zenith_amd/csrc/zr_runtime.cpp, zr_rccl.cpp) built
  with hipcc -Xarch_host -fsanitize=..., exercised through the device-free paths
  of the C ABI (tests/sanitize/abi_host.c) and by examples/triangle.c, which on
  a machine without a GPU must fail cleanly at zr_device_create.
Every build uses -fno-sanitize-recover=all, so any report ends the run non-zero.
"""
import ctypes as C
import glob
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle
from zenith_amd import scenes, zr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


@pytest.fixture(scope="module")
def oracle_san(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("san") / "oracle_san")
    subprocess.run(["gcc", *SAN, "-std=c11", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-Wall",
                    "-I", os.path.join(ROOT, "oracle"), os.path.join(ROOT, "oracle", "zr_oracle.c"),
                    os.path.join(ROOT, "oracle", "san_driver.c"), "-lm", "-o", exe], check=True)
    return exe


def write_scene(path, s, shard=(0, 1), nthreads=1):
    """The scene file san_driver.c reads: the same structures oracle.render passes."""
    W, H = s.width, s.height
    vb = np.ascontiguousarray(s.vertices, dtype=np.float32)
    ib = None if s.indices is None else np.ascontiguousarray(s.indices)
    nat = len(s.layout)
    offs = [4 * sum(s.layout[:a]) for a in range(nat)] + [0] * (4 - nat)
    sizes = [4 * n for n in s.layout] + [0] * (4 - nat)
    st = oracle._DrawState(s.program, s.time, (C.c_float * 6)(0.0, 0.0, float(W), float(H), 0.0, 1.0),
                           (C.c_int32 * 4)(0, 0, W, H), (C.c_int32 * 4)(0, 0, W, H), s.cull_mode, s.front_face,
                           1 if s.depth_test else 0, 1 if s.depth_write else 0, s.depth_op, s.write_mask, 32,
                           shard[0], shard[1], (C.c_float * 16)(*(s.view_proj or (0.0,) * 16)))
    cmd = oracle._DrawCmd(s.draw_count, s.instance_count, s.first, s.vertex_offset, 0, 1 if ib is not None else 0)
    head = np.array([0x4253525A, nthreads], dtype=np.uint32).tobytes() + bytes(st) + bytes(cmd)
    tail = (np.array([W, H], dtype=np.uint32).tobytes() + np.array([s.color_format], dtype=np.int32).tobytes()
            + np.array([1 if s.depth else 0], dtype=np.uint32).tobytes()
            + np.array([0, 0, W, H], dtype=np.int32).tobytes() + np.array(s.clear_color, dtype=np.float32).tobytes()
            + np.array([s.depth_clear], dtype=np.float32).tobytes()
            + np.array([32, vb.shape[1] * 4, nat, *offs, *sizes], dtype=np.uint32).tobytes()
            + np.array([s.index_type], dtype=np.int32).tobytes()
            + np.array([vb.nbytes, ib.nbytes if ib is not None else 0], dtype=np.uint64).tobytes())
    with open(path, "wb") as f:
        f.write(head + tail + vb.tobytes() + (ib.tobytes() if ib is not None else b""))


def _scenes():
    out = [("triangle_t1p25", scenes.triangle_scene(time=1.25)), ("cube", scenes.cube_scene()),
           ("soup_flat", scenes.soup_scene(5, 3000, 256, 192, 10.0, scenes.PROGRAM_FLAT_COLOR)),
           ("soup_blinn", scenes.soup_scene(6, 3000, 256, 192, 12.0, scenes.PROGRAM_BLINN_PHONG)),
           ("mesh_clip", scenes.mesh_soup_scene(7, 1500, 256, 192))]
    s = scenes.soup_scene(8, 2000, 200, 160, 20.0, scenes.PROGRAM_FLAT_COLOR)
    s.indices = s.indices.copy()
    s.indices[::7] = 10_000_000  # out-of-range vertex ids: the draw drops those primitives
    out.append(("oob_indices", s))
    s = scenes.soup_scene(9, 800, 200, 160, 30.0, scenes.PROGRAM_BLINN_PHONG)
    s.instance_count, s.first, s.vertex_offset = 3, 6, 3
    out.append(("instanced_offsets", s))
    s = scenes.soup_scene(10, 1200, 200, 160, 9.0, scenes.PROGRAM_FLAT_COLOR)
    s.indices = None  # non-indexed
    out.append(("non_indexed", s))
    return out


@pytest.mark.parametrize("name,scene", _scenes(), ids=[n for n, _ in _scenes()])
@pytest.mark.parametrize("shard,nthreads", [((0, 1), 1), ((1, 3), 2)], ids=["whole", "shard1of3"])
def test_oracle_sanitized(oracle_san, tmp_path, name, scene, shard, nthreads):
    path, out = str(tmp_path / "scene.bin"), str(tmp_path / "out.bin")
    write_scene(path, scene, shard, nthreads)
    r = subprocess.run([oracle_san, path, out], capture_output=True, text=True, timeout=120, env=ENV)
    assert r.returncode == 0, r.stderr[-4000:]
    color, depth = oracle.render(scene, shard=shard)
    raw = np.fromfile(out, dtype=np.uint8)
    assert np.array_equal(raw[:color.size], color.reshape(-1))
    if depth is not None:
        got = raw[color.size:].view(np.uint32)
        assert np.array_equal(got, depth.reshape(-1).view(np.uint32))


def _clang_asan_rt():
    libs = glob.glob("/opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    if not libs:
        pytest.skip("no clang ASan runtime in this image")
    return os.path.dirname(libs[0])


@pytest.fixture(scope="module")
def runtime_san(tmp_path_factory):
    """libzenith_raster with the host code sanitized (the kernels' object as built)."""
    d = tmp_path_factory.mktemp("rtsan")
    kernels = os.path.join(ROOT, "zenith_amd", "build", "zr_kernels.o")
    if not os.path.exists(kernels):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "zenith_amd"), "ARCH=gfx950"], check=True)
    hip = ["/opt/rocm/bin/hipcc", "-O1", "-g", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
           "-fvisibility=hidden", "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "zenith_amd", "csrc"),
           "--offload-arch=gfx950"]
    host_san = [x for f in ("-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=all",
                            "-fno-omit-frame-pointer") for x in ("-Xarch_host", f)]
    objs = []
    for src in ("zr_runtime.cpp", "zr_rccl.cpp"):
        o = str(d / (src + ".o"))
        subprocess.run(hip + host_san + ["-x", "hip", "-c", os.path.join(ROOT, "zenith_amd", "csrc", src), "-o", o],
                       check=True)
        objs.append(o)
    lib = str(d / "libzenith_raster_san.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-Xarch_host",
                    "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-shared-libasan", "-o", lib,
                    *objs, kernels, "-ldl", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return str(d)


def _build_c(runtime_san, src, exe):
    rt = _clang_asan_rt()
    subprocess.run(["/opt/rocm/llvm/bin/clang", *SAN, "-shared-libasan", "-Wall", "-I", os.path.join(ROOT, "include"),
                    src, "-L", runtime_san, "-lzenith_raster_san", f"-Wl,-rpath,{runtime_san}", f"-Wl,-rpath,{rt}",
                    "-o", exe], check=True)
    return exe


def test_runtime_abi_sanitized(runtime_san, tmp_path):
    exe = _build_c(runtime_san, os.path.join(ROOT, "tests", "sanitize", "abi_host.c"), str(tmp_path / "abi_host"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=ENV, cwd=ROOT)
    assert r.returncode == 0 and "abi_host ok" in r.stdout, r.stderr[-4000:]


def test_c_example_sanitized(runtime_san, tmp_path):
    """examples/triangle.c under ASan/UBSan: without a GPU it must stop at
    zr_device_create with the error message and exit 1, with no sanitizer report."""
    h = C.c_void_p()
    if zr.lib().zr_device_create(0, C.byref(h)) == zr.SUCCESS:
        zr.lib().zr_device_destroy(h)
        pytest.skip("a GPU is present (tests/test_c_example.py runs the frame there)")
    exe = _build_c(runtime_san, os.path.join(ROOT, "examples", "triangle.c"), str(tmp_path / "triangle_san"))
    r = subprocess.run([exe, str(tmp_path / "frame.bgra")], capture_output=True, text=True, timeout=120, env=ENV)
    assert r.returncode == 1, r.stderr[-4000:]
    assert "zr_device_create" in r.stderr and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr
