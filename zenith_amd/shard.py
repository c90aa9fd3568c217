"""Screen-tile sharding across ranks and the tile gather.

Ownership (zr_internal.h ShardGeom, restated here): of a target's
tiles_y rows of 32x32 tiles, the first F = floor(tiles_y / G) * G go round robin
(row t to rank t % G, interleaved for load balance); the n tiles of the last
tiles_y - F rows, in row-major order, are cut into G runs, tile i of them
belonging to rank floor(i * G / n).  Every rank owns the floor or the ceiling of
the tiles / G.  The gather: each rank packs its owned pixels into one
contiguous buffer, sends it point-to-point to rank 0 (RCCL over xGMI on the GPU
box: each peer uses its own link, no ring), and rank 0 scatters them into place.
Works on any torch device, so the same code is exercised with gloo on CPU in
tests/test_dist.py.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import zr

TILE = zr.tile_size()  # the library's tile edge (zr::kTile, zr_tile_size): the unit of ownership


def tile_owner(tiles_x: int, tiles_y: int, world: int) -> np.ndarray:
    """[tiles_y, tiles_x] owner rank of every tile."""
    full = (tiles_y // world) * world
    own = np.empty((tiles_y, tiles_x), dtype=np.int64)
    own[:full] = (np.arange(full) % world)[:, None]
    n = (tiles_y - full) * tiles_x
    if n:
        own[full:] = (np.arange(n) * world // n).reshape(tiles_y - full, tiles_x)
    return own


def owned_mask(width: int, height: int, rank: int, world: int, tile: int = TILE) -> np.ndarray:
    """[height, width] bool: the pixels of the tiles rank `rank` of `world` owns."""
    own = tile_owner(-(-width // tile), -(-height // tile), world) == rank
    return np.repeat(np.repeat(own, tile, axis=0), tile, axis=1)[:height, :width]


def owned_pixels(width: int, height: int, rank: int, world: int, tile: int = TILE) -> int:
    return int(owned_mask(width, height, rank, world, tile).sum())


class TileGather:
    """Pre-plans the owned-pixel index lists and receive buffers for one image
    shape (torch.distributed point-to-point; the runtime's own RCCL gather is
    zr_device_gather_tile_rows)."""

    def __init__(self, width: int, height: int, bytes_per_pixel: int, rank: int, world: int, device,
                 tile: int = TILE, group=None):
        self.rank, self.world, self.group = rank, world, group
        self.shape = (height * width, bytes_per_pixel)
        flat = [torch.from_numpy(np.flatnonzero(owned_mask(width, height, r, world, tile))).to(device)
                for r in range(world)]
        self.pix = flat
        self.send_buf = torch.empty((len(flat[rank]), bytes_per_pixel), dtype=torch.uint8, device=device)
        self.recv_bufs = None
        if rank == 0:
            self.recv_bufs = [torch.empty((len(flat[r]), bytes_per_pixel), dtype=torch.uint8, device=device)
                              for r in range(world)]

    def gather(self, image: torch.Tensor) -> None:
        """image: [H, W * bytes_per_pixel] uint8, fully valid on rank 0 afterwards."""
        if self.world == 1:
            return
        img = image.view(self.shape)
        peer = (lambda r: dist.get_global_rank(self.group, r)) if self.group is not None else (lambda r: r)
        if self.rank == 0:
            ops = [dist.P2POp(dist.irecv, self.recv_bufs[r], peer(r), group=self.group) for r in range(1, self.world)]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            for r in range(1, self.world):
                img.index_copy_(0, self.pix[r], self.recv_bufs[r])
        else:
            torch.index_select(img, 0, self.pix[self.rank], out=self.send_buf)
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, self.send_buf, peer(0), group=self.group)]):
                req.wait()


# ------------------------------------------------ partitioned setup exchange
#
# zr_cmd_set_tile_shard_exchange (include/zenith_raster.h): each
# rank sets up 1/G of a draw's primitives and ships each set-up primitive to the
# ranks owning the tile rows it touches; the blocks travel in one all-to-all per
# draw.  Host model of the device layout (zr_internal.h RouteEntry / RouteHeader,
# zr_runtime.cpp exec_draw): rank r routes primitives [r * span, (r + 1) * span)
# with span = ceil(ceil(N / G) / ROUTE_CHUNK) * ROUTE_CHUNK; its block for one
# destination is a 16-B header (u32 pad, u32 total, 2 pad) then `cap` 48-B
# entries (32-B compact record, u32 bb0, u32 bb1, u32 draw id, pad).  The device
# appends a workgroup's run of entries at an atomically reserved offset, so their
# order in a block is unspecified: the receiver keys records by the draw id.  The
# block holds min(total, cap) entries; total > cap tells the receiver it overflowed.

ROUTE_CHUNK = 512   # zr::kRouteChunk (primitives per k_route workgroup)
HEADER_BYTES = 16   # sizeof(zr::RouteHeader)
ENTRY_BYTES = 48    # sizeof(zr::RouteEntry)
_ENTRY = np.dtype([("rec", "<i4", 8), ("bb0", "<u4"), ("bb1", "<u4"), ("gid", "<u4"), ("pad", "<u4")])
_HEADER = np.dtype([("pad0", "<u4"), ("total", "<u4"), ("pad", "<u4", 2)])
assert _ENTRY.itemsize == ENTRY_BYTES and _HEADER.itemsize == HEADER_BYTES


def capacity_default(span: int, world: int) -> int:
    """zr_runtime.cpp route_capacity_default: entries per block when the caller sets none."""
    return span if world <= 2 else min(span, -(-2 * span // world) + 4096)


def route_geometry(n_prims: int, world: int, cap: int = 0):
    """(chunks, span, cap, block_bytes) of a G-way partitioned draw of n primitives
    with `cap` entries per block (0: the runtime's default)."""
    per_rank = -(-n_prims // world)
    chunks = max(1, -(-per_rank // ROUTE_CHUNK))
    span = chunks * ROUTE_CHUNK
    cap = max(1, min(span, cap if cap else capacity_default(span, world)))
    return chunks, span, cap, HEADER_BYTES + cap * ENTRY_BYTES


def route_range(n_prims: int, rank: int, world: int):
    """[lo, hi) of the primitives rank `rank` routes."""
    _, span, _, _ = route_geometry(n_prims, world)
    lo = min(n_prims, rank * span)
    return lo, min(n_prims, lo + span)


def route_dests(row_lo: int, row_hi: int, world: int, tiles_x: int, tiles_y: int):
    """Ranks owning a tile of rows [row_lo, row_hi] (every column): k_route's
    dest_mask for a bbox spanning the target's width."""
    own = tile_owner(tiles_x, tiles_y, world)
    return sorted(set(own[row_lo:row_hi + 1].reshape(-1).tolist()))


def route_blocks(row_lo, row_hi, rank: int, world: int, cap: int = 0, tiles_x: int = 1, tiles_y: int = 0) -> torch.Tensor:
    """Host model of k_route for rank `rank`: row_lo/row_hi are each primitive's
    first/last tile row (row_lo < 0: no sample) of a tiles_x x tiles_y target
    (default: one column, rows up to the largest row_hi), the primitive spanning
    every column; the entries' bbox words carry the rows (bb0 = row_lo, bb1 =
    row_hi) in place of a pixel bbox.  Returns the send buffer,
    [world][block_bytes] uint8, entries in primitive order (one of the orders the
    device may produce)."""
    n = len(row_lo)
    tiles_y = tiles_y or int(max(row_hi)) + 1
    own = tile_owner(tiles_x, tiles_y, world)
    _, span, cap, bb = route_geometry(n, world, cap)
    hdr = np.zeros(world, dtype=_HEADER)
    ent = np.zeros((world, cap), dtype=_ENTRY)
    lo, hi = route_range(n, rank, world)
    for p in range(lo, hi):
        a, b = int(row_lo[p]), int(row_hi[p])
        if a < 0:
            continue
        dests = sorted(set(own[a:b + 1].reshape(-1).tolist()))
        for d in dests:
            k = int(hdr[d]["total"])
            if k < cap:
                ent[d][k]["bb0"], ent[d][k]["bb1"], ent[d][k]["gid"] = a, b, p
            hdr[d]["total"] = k + 1
    out = np.zeros((world, bb), dtype=np.uint8)
    for d in range(world):
        out[d, :HEADER_BYTES] = np.frombuffer(hdr[d:d + 1].tobytes(), dtype=np.uint8)
        out[d, HEADER_BYTES:] = np.frombuffer(ent[d].tobytes(), dtype=np.uint8)
    return torch.from_numpy(out)


def received_primitives(recv: torch.Tensor, n_prims: int, world: int, cap: int = 0):
    """(draw ids of a rank's received entries in block-position order -- the
    device's dense setup positions --, True if a block overflowed: the device then
    sets up every primitive instead)."""
    _, _, cap, bb = route_geometry(n_prims, world, cap)
    raw = recv.reshape(world, bb).numpy()
    out, over = [], False
    for s in range(world):
        h = np.frombuffer(raw[s, :HEADER_BYTES].tobytes(), dtype=_HEADER)[0]
        e = np.frombuffer(raw[s, HEADER_BYTES:].tobytes(), dtype=_ENTRY)
        out += e["gid"][:min(int(h["total"]), cap)].tolist()
        over |= int(h["total"]) > cap
    return out, over


class _DeviceBytes:
    """A raw device pointer as a uint8 array (__cuda_array_interface__), so the
    runtime's exchange blocks can be handed to torch without a copy."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


def device_bytes(ptr: int, nbytes: int, device) -> torch.Tensor:
    return torch.as_tensor(_DeviceBytes(ptr, nbytes), device=device)


class Exchange:
    """An all-to-all the runtime calls once per partitioned draw (zr_exchange_fn).
    Subclasses implement ``exchange(stream, send_ptr, recv_ptr, bytes_per_rank)``
    and must order it on ``stream``."""

    def __init__(self):
        self._cb = None
        self.calls = 0

    def exchange(self, stream: int, send: int, recv: int, nbytes: int) -> None:
        raise NotImplementedError

    def c_callback(self):
        if self._cb is None:
            from . import zr

            def call(user, stream, send, recv, nbytes):
                try:
                    self.exchange(stream or 0, send or 0, recv or 0, int(nbytes))
                    self.calls += 1
                    return zr.SUCCESS
                except Exception as e:  # never unwind into the C runtime
                    import traceback
                    traceback.print_exc()
                    self.error = e
                    return zr.ERROR_UNKNOWN
            self._cb = zr.EXCHANGE_FN(call)
        return self._cb


class RcclExchange(Exchange):
    """The exchange over torch.distributed (RCCL over xGMI with the "nccl"
    backend): one all_to_all_single per draw, ordered on the runtime's stream
    without a host wait."""

    def __init__(self, device, group=None):
        super().__init__()
        self.device = torch.device(device)
        self.group = group
        self.world = dist.get_world_size(group)
        self._views = {}

    def _view(self, ptr, nbytes):
        key = (ptr, nbytes)
        t = self._views.get(key)
        if t is None:
            t = self._views[key] = device_bytes(ptr, nbytes, self.device)
        return t

    def exchange(self, stream, send, recv, nbytes):
        s = self._view(send, nbytes * self.world)
        r = self._view(recv, nbytes * self.world)
        cur = torch.cuda.current_stream(self.device)
        if stream and stream != cur.cuda_stream:
            with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=self.device)):
                dist.all_to_all_single(r, s, group=self.group)
        else:
            dist.all_to_all_single(r, s, group=self.group)


class ThreadGroupExchange(Exchange):
    """G ranks emulated by G threads of one process on one GPU (tests): each
    rank's runtime calls its own instance from its submitting thread; the
    instances meet at a barrier and copy blocks device-to-device."""

    class Group:
        def __init__(self, world: int, device):
            import threading
            self.world = world
            self.device = torch.device(device)
            self.barrier = threading.Barrier(world, timeout=120)
            self.sends = [None] * world

    def __init__(self, group: "ThreadGroupExchange.Group", rank: int):
        super().__init__()
        self.group, self.rank = group, rank

    def exchange(self, stream, send, recv, nbytes):
        g = self.group
        torch.cuda.ExternalStream(stream, device=g.device).synchronize()  # k_route done
        g.sends[self.rank] = send
        g.barrier.wait()
        r = device_bytes(recv, nbytes * g.world, g.device)
        for s in range(g.world):
            src = device_bytes(g.sends[s] + self.rank * nbytes, nbytes, g.device)
            r[s * nbytes:(s + 1) * nbytes].copy_(src)
        torch.cuda.synchronize(g.device)
        g.barrier.wait()  # every rank copied before any send buffer is rewritten


def runtime_rccl_available() -> bool:
    """True if libzenith_raster can load RCCL in this process."""
    from . import zr
    return zr.lib().zr_rccl_available() == 1


def init_runtime_rccl(device, rank: int, world: int, group=None) -> None:
    """Gives ``device`` (rhi.RenderDevice) the runtime's own RCCL communicators:
    rank 0 makes the two ids, torch.distributed carries them to every rank, and
    every rank joins (zr_device_init_rccl).  After this, tile-row shards can use
    exchange="rccl" and RenderDevice.gather_tile_rows."""
    import ctypes as C
    from . import zr
    ids = [None]
    if rank == 0:
        a = C.create_string_buffer(zr.RCCL_ID_BYTES)
        b = C.create_string_buffer(zr.RCCL_ID_BYTES)
        zr.check(zr.lib().zr_rccl_get_unique_id(a), "zr_rccl_get_unique_id")
        zr.check(zr.lib().zr_rccl_get_unique_id(b), "zr_rccl_get_unique_id")
        ids = [(a.raw, b.raw)]
    if world > 1:
        dist.broadcast_object_list(ids, src=0, group=group)
    device.init_rccl(ids[0][0], ids[0][1], world, rank)
