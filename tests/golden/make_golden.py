"""Generates the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference ships no tests, fixtures or golden images and
cannot be built or run here (no Rust / Vulkan / slangc), so the
fixtures are the oracle's output on the reference's own scene (triangle.rs at
T=0) and on synthetic scenes, pinned by analytic known-answer tests in
tests/test_oracle.py.  Each fixture is raw data: the rendered attachment bytes
(gzip) plus a JSON manifest with shape, format and the SHA-256 of the raw bytes.

    python tests/golden/make_golden.py
"""
import gzip
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from zenith_amd import scenes  # noqa: E402


def golden_scenes():
    """name -> scene; small enough that the fixtures stay a few hundred KB."""
    tie = tie_scene()
    return {
        "triangle_640x480_t0": scenes.triangle_scene(),
        "triangle_640x480_t1p25": scenes.triangle_scene(time=1.25),
        "cube_640x480": scenes.cube_scene(),
        "soup_flat_256x192": scenes.soup_scene(21, 1000, 256, 192, 12.0, scenes.PROGRAM_FLAT_COLOR),
        "soup_blinn_256x192": scenes.soup_scene(22, 1000, 256, 192, 8.0, scenes.PROGRAM_BLINN_PHONG),
        "ties_64x64": tie,
        # mesh.slang through a camera: near-plane crossings, behind-camera and
        # off-screen primitives, and the cerberus asset
        "mesh_soup_160x120": scenes.mesh_soup_scene(31, 600, 160, 120),
        "cerberus_320x240": scenes.cerberus_scene(320, 240),
    }


def tie_scene():
    """64 triangles over a 64x64 target with shared edges and vertices placed
    exactly on pixel centres (pins the tie rule and submission order)."""
    W = H = 64
    verts = []
    rng = np.random.default_rng(5)
    # an 8x8 grid of quads whose corners sit on pixel centres, split along both diagonals
    g = [(4 + 8 * i) + 0.5 for i in range(8)]
    k = 0
    for yi in range(7):
        for xi in range(7):
            if k >= 64:
                break
            x0, x1, y0, y1 = g[xi], g[xi + 1], g[yi], g[yi + 1]
            c = rng.random(3)
            if (xi + yi) % 2:
                tris = [((x0, y0), (x1, y0), (x1, y1)), ((x0, y0), (x1, y1), (x0, y1))]
            else:
                tris = [((x0, y0), (x1, y0), (x0, y1)), ((x1, y0), (x1, y1), (x0, y1))]
            for tri in tris:
                z = 0.25 + 0.5 * rng.random()
                for (x, y) in tri:
                    verts.append([2 * x / W - 1, 2 * y / H - 1, z, *c])
                k += 1
    v = np.array(verts[:64 * 3], dtype=np.float32)
    idx = np.arange(v.shape[0], dtype=np.uint32)
    s = scenes.Scene("ties", W, H, scenes.PROGRAM_FLAT_COLOR, v, idx, depth=True)
    return s


def render_bytes(scene):
    col, dep = oracle.render(scene)
    blobs = {"color": col.tobytes()}
    if dep is not None:
        blobs["depth"] = dep.tobytes()
    return blobs


def bake_cerberus():
    """tests/golden/cerberus.mesh.npz: /root/reference/content/mesh/cerberus/scene.gltf
    baked as zenith-asset's gltf_loader does (zenith_amd.assets).  Only where the
    reference is mounted; the GPU box and later rounds use the committed file."""
    from zenith_amd import assets
    src = "/root/reference/content/mesh/cerberus/scene.gltf"
    if not os.path.exists(src):
        return
    v, i = assets.load_gltf_meshes(src)[0]
    np.savez_compressed(os.path.join(HERE, "cerberus.mesh.npz"), vertices=v, indices=i)


def main():
    if "--mesh" in sys.argv:
        bake_cerberus()
    manifest = {}
    for name, scene in golden_scenes().items():
        blobs = render_bytes(scene)
        entry = {"width": scene.width, "height": scene.height, "color_format": scene.color_format,
                 "program": scene.program, "triangles": scene.triangles}
        for kind, data in blobs.items():
            fn = f"{name}.{kind}.bin.gz"
            with gzip.GzipFile(os.path.join(HERE, fn), "wb", mtime=0) as fh:
                fh.write(data)
            entry[kind] = {"file": fn, "sha256": hashlib.sha256(data).hexdigest(), "bytes": len(data)}
        manifest[name] = entry
    with open(os.path.join(HERE, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print(json.dumps({k: v["color"]["sha256"][:16] for k, v in manifest.items()}, indent=1))


if __name__ == "__main__":
    main()
