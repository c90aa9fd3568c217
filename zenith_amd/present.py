"""Headless present: the swapchain's role without a window.

- ``write_png``: a rendered BGRA8/RGBA8 frame (sRGB codes as stored) to an
  8-bit RGBA PNG, zlib only (frames can be inspected off the GPU box).
- ``FrameRateCounter``: the frame-rate line of the reference's main loop
  (zenith/src/main_loop.rs:141-170): frames counted per window of more than one
  second, fps = ceil(frames / elapsed).
"""
from __future__ import annotations

import math
import struct
import time
import zlib

import numpy as np

_BGRA = (50, 44)  # B8G8R8A8_SRGB, B8G8R8A8_UNORM


def png_bytes(image: np.ndarray, vk_format: int) -> bytes:
    """image: [H, W, 4] uint8 as the texture stores it."""
    img = np.ascontiguousarray(image, dtype=np.uint8)
    if img.ndim != 3 or img.shape[2] != 4:
        raise ValueError("expected an [H, W, 4] 8-bit colour image")
    if vk_format in _BGRA:
        img = img[:, :, [2, 1, 0, 3]]
    h, w = img.shape[:2]
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))  # filter 0 per row

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0)  # 8-bit RGBA
    return b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")


def write_png(path: str, image: np.ndarray, vk_format: int) -> None:
    with open(path, "wb") as fh:
        fh.write(png_bytes(image, vk_format))


def read_png_rgba(data: bytes) -> np.ndarray:
    """Decoder for this module's own files (filter 0, 8-bit RGBA, one IDAT)."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, w, h, idat = 8, 0, 0, b""
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if tag == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    return raw[:, 1:].reshape(h, w, 4)


class FrameRateCounter:
    """main_loop.rs:141-170: tick() once per frame; returns the fps of the last
    window when more than one second has passed since the last report, else None."""

    def __init__(self, clock=time.monotonic):
        self.clock = clock
        self.last_printed = clock()
        self.frames = 0

    def tick(self):
        now = self.clock()
        elapsed = now - self.last_printed
        report = None
        if elapsed > 1.0:
            report = int(math.ceil(self.frames / elapsed))
            self.last_printed = now
            self.frames = 0
        self.frames += 1
        return report
