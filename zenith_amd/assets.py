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
