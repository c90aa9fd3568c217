"""Screen-tile sharding across ranks and the tile-row gather.

Rank r of G renders the tile rows t with t % G == r (interleaved for load
balance).  Its rows of the final image are contiguous row spans, so the gather
is: pack the owned rows into one contiguous buffer, point-to-point send it to
rank 0 (RCCL over xGMI on the GPU box: each peer uses its own link, no ring),
and rank 0 scatters the received rows into place.  Works on any torch device,
so the same code is exercised with gloo on CPU in tests/test_dist.py.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

TILE = 32  # must match zr::kTile (zenith_amd/csrc/zr_internal.h)


def owned_rows(height: int, rank: int, world: int, tile: int = TILE, device=None) -> torch.Tensor:
    rows = torch.arange(height, device=device)
    return rows[((rows // tile) % world) == rank]


class TileRowGather:
    """Pre-plans the row index lists and receive buffers for one image shape."""

    def __init__(self, height: int, row_bytes: int, rank: int, world: int, device, tile: int = TILE):
        self.rank, self.world = rank, world
        self.rows = [owned_rows(height, r, world, tile, device) for r in range(world)]
        self.send_buf = torch.empty((len(self.rows[rank]), row_bytes), dtype=torch.uint8, device=device)
        self.recv_bufs = None
        if rank == 0:
            self.recv_bufs = [torch.empty((len(self.rows[r]), row_bytes), dtype=torch.uint8, device=device)
                              for r in range(world)]

    def gather(self, image: torch.Tensor) -> None:
        """image: [H, row_bytes] uint8, fully valid on rank 0 afterwards."""
        if self.world == 1:
            return
        if self.rank == 0:
            ops = [dist.P2POp(dist.irecv, self.recv_bufs[r], r) for r in range(1, self.world)]
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            for r in range(1, self.world):
                image.index_copy_(0, self.rows[r], self.recv_bufs[r])
        else:
            torch.index_select(image, 0, self.rows[self.rank], out=self.send_buf)
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, self.send_buf, 0)]):
                req.wait()
