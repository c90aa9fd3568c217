"""Baked-mesh files (zenith_amd.assets): zenith-asset's ``Mesh<Vertex>`` in
bincode 2.0.1's standard encoding (zenith-asset/src/lib.rs:256-279,
render.rs:10-36) and the glTF bake (gltf_loader.rs:62-148).  The reference holds
no baked ``.mesh`` file, so the byte layout is pinned by known-answer vectors
written from bincode's published format (varint boundaries 250 / 251 / 2^16 /
2^32 - 1, Option tags); parity against a reference-written file is unpinned."""
import json
import os
import struct

import numpy as np
import pytest

from zenith_amd import assets, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mesh_bytes_known_answer():
    v = np.arange(16, dtype=np.float32).reshape(2, 8)
    idx = np.array([0, 250, 251, 65535, 65536, 0xFFFFFFFF], np.uint32)
    b = assets.encode_mesh(v, idx)
    expect = (b"\x02" + struct.pack("<16f", *range(16)) + b"\x06" + b"\x00" + b"\xfa" + b"\xfb\xfb\x00" +
              b"\xfb\xff\xff" + b"\xfc\x00\x00\x01\x00" + b"\xfc\xff\xff\xff\xff" + b"\x00")
    assert b == expect
    dv, di, mat = assets.decode_mesh(b)
    assert np.array_equal(dv, v) and np.array_equal(di, idx) and mat is None


@pytest.mark.parametrize("material,tail", [(None, b"\x00"), (3, b"\x01\x03"), (300, b"\x01\xfb\x2c\x01"),
                                           (1 << 40, b"\x01\xfd" + (1 << 40).to_bytes(8, "little"))])
def test_mesh_material_option(material, tail):
    b = assets.encode_mesh(np.zeros((0, 8), np.float32), np.zeros(0, np.uint32), material)
    assert b == b"\x00\x00" + tail
    assert assets.decode_mesh(b)[2] == material


def test_mesh_vertex_count_varint():
    v = np.zeros((251, 8), np.float32)
    b = assets.encode_mesh(v, np.zeros(0, np.uint32))
    assert b[:3] == b"\xfb\xfb\x00" and len(b) == 3 + 251 * 32 + 2


@pytest.mark.parametrize("data", [b"", b"\x01", b"\x00\x02\x05", b"\x00\x00", b"\x00\x00\x02", b"\x00\x01\xfe",
                                  b"\x00\x01\xfb\x01"])
def test_mesh_decode_errors(data):
    with pytest.raises(ValueError):
        assets.decode_mesh(data)


def test_cerberus_round_trip(tmp_path):
    with np.load(os.path.join(ROOT, scenes.CERBERUS_NPZ), allow_pickle=False) as z:
        v, i = z["vertices"], z["indices"]
    path = str(tmp_path / "mesh" / "cerberus" / "scene.mesh")
    assets.save_mesh(path, v, i)
    dv, di, mat = assets.load_mesh(path)
    assert dv.shape == (len(v), 8) and np.array_equal(dv.view(np.uint32), v.astype(np.float32).view(np.uint32))
    assert np.array_equal(di, i) and mat is None and len(di) == 3 * 33543
    a = scenes.cerberus_scene(160, 120)
    b = scenes.cerberus_scene(160, 120, npz=path)
    assert np.array_equal(a.vertices, b.vertices) and np.array_equal(a.indices, b.indices)
    assert np.array_equal(a.view_proj, b.view_proj)


def _write_gltf(tmp_path, with_normals: bool) -> str:
    pos = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 0], [0, 0, 1], [1, 0, 0]], np.float32)
    nrm = np.tile(np.array([[0, 0, 1]], np.float32), (6, 1))
    idx = np.array([0, 1, 2, 3, 4, 5], np.uint16)
    blob = pos.tobytes() + (nrm.tobytes() if with_normals else b"") + idx.tobytes()
    (tmp_path / "scene.bin").write_bytes(blob)
    views = [{"buffer": 0, "byteOffset": 0, "byteLength": 72}]
    accessors = [{"bufferView": 0, "componentType": 5126, "count": 6, "type": "VEC3"}]
    attrs = {"POSITION": 0}
    off = 72
    if with_normals:
        views.append({"buffer": 0, "byteOffset": off, "byteLength": 72})
        accessors.append({"bufferView": 1, "componentType": 5126, "count": 6, "type": "VEC3"})
        attrs["NORMAL"] = 1
        off += 72
    views.append({"buffer": 0, "byteOffset": off, "byteLength": 12})
    accessors.append({"bufferView": len(views) - 1, "componentType": 5123, "count": 6, "type": "SCALAR"})
    gltf = {"asset": {"version": "2.0"}, "scene": 0, "scenes": [{"nodes": [0]}],
            "nodes": [{"children": [1]}, {"mesh": 0}],
            "meshes": [{"primitives": [{"attributes": attrs, "indices": len(accessors) - 1}]}],
            "buffers": [{"uri": "scene.bin", "byteLength": len(blob)}], "bufferViews": views, "accessors": accessors}
    path = tmp_path / "scene.gltf"
    path.write_text(json.dumps(gltf))
    return str(path)


@pytest.mark.parametrize("with_normals", [True, False])
def test_bake_gltf(tmp_path, with_normals):
    src = _write_gltf(tmp_path, with_normals)
    out = tmp_path / "baked"
    urls = assets.bake_gltf(src, str(out), "mesh/toy/scene.gltf")
    assert urls == ["mesh/toy/scene.mesh"]
    v, i, mat = assets.load_mesh(str(out / "mesh/toy/scene.mesh"))
    assert mat is None and list(i) == [0, 1, 2, 3, 4, 5]
    assert np.array_equal(v[:, 6:], np.zeros((6, 2), np.float32))  # TEXCOORD_0 missing -> zeros
    # flat normals when NORMAL is missing: (v1 - v0) x (v2 - v0), normalized
    want = [[0, 0, 1]] * 6 if with_normals else [[0, 0, 1]] * 3 + [[0, 1, 0]] * 3
    assert np.array_equal(v[:, 3:6], np.array(want, np.float32))
