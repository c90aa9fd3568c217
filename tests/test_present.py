"""Headless present: PNG dump and the main loop's frame-rate
line (zenith/src/main_loop.rs:141-170).  CPU only."""
import numpy as np

from zenith_amd import present


def test_png_round_trip_bgra():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    data = present.png_bytes(img, 50)  # B8G8R8A8_SRGB
    back = present.read_png_rgba(data)
    assert np.array_equal(back, img[:, :, [2, 1, 0, 3]])
    rgba = present.read_png_rgba(present.png_bytes(img, 37))  # R8G8B8A8_UNORM: as stored
    assert np.array_equal(rgba, img)


def test_frame_rate_counter_matches_main_loop():
    """frames counted since the last line; a line when > 1 s passed:
    fps = ceil(frames / elapsed), then the count restarts at this frame."""
    t = [0.0]
    c = present.FrameRateCounter(clock=lambda: t[0])
    reports = []
    for _ in range(200):          # 200 frames at 7 ms
        t[0] += 0.007
        r = c.tick()
        if r is not None:
            reports.append((round(t[0], 3), r))
    # the 143rd tick (t = 1.001 s) reports the 142 frames counted before it:
    # ceil(142 / 1.001) = 142
    assert reports == [(1.001, 142)]
