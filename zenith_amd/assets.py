"""Real-mesh ingestion: a glTF primitive baked into
zenith-asset's ``Mesh<Vertex>`` as ``RawGltfProcessor::bake_mesh`` does
(zenith-asset/src/gltf_loader.rs:94-148): positions, normals (flat normals when
missing), TEXCOORD_0 (zeros when missing) zipped into ``Vertex {position, normal,
tex_coord}`` (zenith-asset/src/render.rs:12-16, 32 B), indices widened to u32.
Node transforms are ignored, as in the reference (gltf_loader.rs:64-91 only walks
the node tree for meshes).  Host-side data loading only: JSON + raw buffers,
nothing executed from the file.
"""
from __future__ import annotations

import json
import os

import numpy as np

_COMPONENT = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16, 5125: np.uint32, 5126: np.float32}
_WIDTH = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4}


def _accessor(gltf: dict, buffers: list, index: int) -> np.ndarray:
    acc = gltf["accessors"][index]
    view = gltf["bufferViews"][acc["bufferView"]]
    dtype = np.dtype(_COMPONENT[acc["componentType"]])
    width = _WIDTH[acc["type"]]
    count = acc["count"]
    base = view.get("byteOffset", 0) + acc.get("byteOffset", 0)
    stride = view.get("byteStride", dtype.itemsize * width)
    raw = buffers[view["buffer"]]
    out = np.empty((count, width), dtype)
    for i in range(width):  # strided gather, one component at a time
        out[:, i] = np.ndarray((count,), dtype, raw, base + i * dtype.itemsize, (stride,))
    return out


def _flat_normals(pos: np.ndarray) -> np.ndarray:
    """generate_flat_normals: each vertex of triangle t gets t's face normal."""
    p = pos.reshape(-1, 3, 3).astype(np.float32)
    n = np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0])
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), np.float32(1e-20))
    return np.repeat(n, 3, axis=0).astype(np.float32)


def load_gltf_meshes(path: str) -> list:
    """Every mesh primitive reachable from the scene's nodes, depth-first
    (process_node order), as (vertices float32 [V, 8], indices uint32 [I])."""
    with open(path) as fh:
        gltf = json.load(fh)
    base = os.path.dirname(path)
    buffers = []
    for b in gltf["buffers"]:
        with open(os.path.join(base, b["uri"]), "rb") as fh:
            buffers.append(fh.read())
    out = []

    def visit(n):
        node = gltf["nodes"][n]
        if "mesh" in node:
            for prim in gltf["meshes"][node["mesh"]]["primitives"]:
                attrs = prim["attributes"]
                pos = _accessor(gltf, buffers, attrs["POSITION"]).astype(np.float32)
                nrm = (_accessor(gltf, buffers, attrs["NORMAL"]).astype(np.float32) if "NORMAL" in attrs
                       else _flat_normals(pos))
                uv = (_accessor(gltf, buffers, attrs["TEXCOORD_0"]).astype(np.float32) if "TEXCOORD_0" in attrs
                      else np.zeros((len(pos), 2), np.float32))
                if "indices" not in prim:
                    raise ValueError("Missing indices")
                idx = _accessor(gltf, buffers, prim["indices"]).reshape(-1).astype(np.uint32)
                if not (len(pos) == len(nrm) == len(uv)):
                    raise ValueError("Vertex attribute count mismatch")
                out.append((np.concatenate([pos, nrm, uv], axis=1), idx))
        for c in node.get("children", []):
            visit(c)

    for root in gltf["scenes"][gltf.get("scene", 0)]["nodes"]:
        visit(root)
    return out


# ------------------------------------------------------------ baked .mesh files
#
# zenith-asset stores a baked ``Mesh<Vertex>`` (render.rs:29-36) with
# ``bincode::encode_to_vec(asset, config::standard())`` (lib.rs:256-270) and reads
# it back with ``bincode::serde::decode_from_slice`` (lib.rs:272-279).  bincode
# 2.0.1's standard configuration (Cargo.toml:31; third-party, restated from its
# published format): little endian, variable-width unsigned integers (< 251 one
# byte; 251 / 252 / 253 + u16 / u32 / u64 LE), sequence lengths as varint u64,
# fixed-size arrays without a length, f32 as 4 LE bytes, Option as a 0 / 1 tag
# byte (+ value).  So a mesh file is
#   varint(V) + V * 32 B of Vertex {position[3], normal[3], tex_coord[2]}
#   + varint(I) + I * varint(u32 index) + (0 | 1 varint(material)).

_VERTEX_FLOATS = 8  # render.rs:12-16


def _varint(v: int) -> bytes:
    if v < 0:
        raise ValueError("bincode varint: negative value")
    if v < 251:
        return bytes([v])
    if v < 1 << 16:
        return b"\xfb" + v.to_bytes(2, "little")
    if v < 1 << 32:
        return b"\xfc" + v.to_bytes(4, "little")
    if v < 1 << 64:
        return b"\xfd" + v.to_bytes(8, "little")
    raise ValueError("bincode varint: value exceeds u64")


def _read_varint(buf: memoryview, pos: int) -> tuple:
    if pos >= len(buf):
        raise ValueError("bincode: unexpected end of data")
    b = buf[pos]
    if b < 251:
        return b, pos + 1
    width = {251: 2, 252: 4, 253: 8}.get(b)
    if width is None:
        raise ValueError(f"bincode: invalid varint tag {b} at byte {pos}")
    if pos + 1 + width > len(buf):
        raise ValueError("bincode: unexpected end of data")
    return int.from_bytes(buf[pos + 1:pos + 1 + width], "little"), pos + 1 + width


def _encode_u32_varints(values: np.ndarray) -> bytes:
    """Vectorized varint encoding of a u32 array (one, three or five bytes each)."""
    v = values.astype(np.uint64)
    size = np.where(v < 251, 1, np.where(v < 1 << 16, 3, 5)).astype(np.int64)
    start = np.concatenate([[0], np.cumsum(size)[:-1]]) if len(v) else np.zeros(0, np.int64)
    out = np.zeros(int(size.sum()), np.uint8)
    one, two, four = size == 1, size == 3, size == 5
    out[start[one]] = v[one].astype(np.uint8)
    out[start[two]] = 251
    for k in range(2):
        out[start[two] + 1 + k] = ((v[two] >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    out[start[four]] = 252
    for k in range(4):
        out[start[four] + 1 + k] = ((v[four] >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    return out.tobytes()


def encode_mesh(vertices: np.ndarray, indices: np.ndarray, material: int | None = None) -> bytes:
    """The bytes ``serialize_asset`` writes for ``Mesh {vertices, indices,
    material}`` (zenith-asset/src/lib.rs:256-270)."""
    vtx = np.ascontiguousarray(vertices, dtype="<f4").reshape(-1, _VERTEX_FLOATS)
    idx = np.asarray(indices).reshape(-1)
    if idx.size and (idx.min() < 0 or idx.max() > 0xFFFFFFFF):
        raise ValueError("indices must fit u32")
    parts = [_varint(len(vtx)), vtx.tobytes(), _varint(len(idx)), _encode_u32_varints(idx)]
    parts.append(b"\x00" if material is None else b"\x01" + _varint(int(material)))
    return b"".join(parts)


def decode_mesh(data: bytes) -> tuple:
    """``deserialize_asset::<Mesh>`` (lib.rs:272-279): (vertices float32 [V, 8],
    indices uint32 [I], material or None).  Trailing bytes are ignored, as
    ``decode_from_slice`` returns the consumed length without checking it."""
    buf = memoryview(data)
    nv, pos = _read_varint(buf, 0)
    end = pos + nv * _VERTEX_FLOATS * 4
    if end > len(buf):
        raise ValueError("bincode: unexpected end of data")
    vertices = np.frombuffer(data, "<f4", nv * _VERTEX_FLOATS, pos).reshape(nv, _VERTEX_FLOATS).astype(np.float32)
    ni, pos = _read_varint(buf, end)
    indices = np.empty(ni, np.uint32)
    for i in range(ni):
        v, pos = _read_varint(buf, pos)
        if v > 0xFFFFFFFF:
            raise ValueError("bincode: index exceeds u32")
        indices[i] = v
    if pos >= len(buf):
        raise ValueError("bincode: unexpected end of data")
    tag = buf[pos]
    if tag == 0:
        material = None
    elif tag == 1:
        material, pos = _read_varint(buf, pos + 1)
    else:
        raise ValueError(f"bincode: invalid Option tag {tag}")
    return vertices, indices, material


def save_mesh(path: str, vertices: np.ndarray, indices: np.ndarray, material: int | None = None) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as fh:
        fh.write(encode_mesh(vertices, indices, material))


def load_mesh(path: str) -> tuple:
    with open(path, "rb") as fh:
        return decode_mesh(fh.read())


def mesh_url(main_url: str) -> str:
    """``Mesh::url`` (render.rs:61-66): the main url with extension ``mesh``
    ("mesh/cerberus/scene.gltf" -> "mesh/cerberus/scene.mesh")."""
    root, _ = os.path.splitext(main_url)
    return root + ".mesh"


def bake_gltf(gltf_path: str, base_directory: str, main_url: str) -> list:
    """``RawGltfProcessor::process_node``'s mesh half (gltf_loader.rs:62-91): every
    primitive is baked and serialized to ``base_directory / mesh_url(main_url)``.
    Every primitive gets that same url, so with several primitives the file holds
    the last one, as in the reference; the returned list has one url per primitive."""
    urls = []
    for vertices, indices in load_gltf_meshes(gltf_path):
        url = mesh_url(main_url)
        save_mesh(os.path.join(base_directory, url), vertices, indices, None)
        urls.append(url)
    return urls
