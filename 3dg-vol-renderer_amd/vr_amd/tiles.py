"""Pixel-tile sharding of one frame over R ranks (one process per GPU) and its reassembly.

The reference parallelises the pixel loop with OpenMP only (test_integrators.h:164); pixels are
independent, so the frame is the data-parallel axis. The frame is cut into 16x16 tiles numbered
row-major; rank r renders tiles r, r + R, r + 2R, ... (interleaved, which balances dense and empty
regions of the image) into a packed slab, slabs are gathered to rank 0 with one RCCL collective
and scattered back into the row-major frame by the device unshuffle kernel. `unshuffle_reference`
is the host mirror of that kernel used by the CPU tests.
"""
import numpy as np

TILE = 16


def num_tiles(W, H):
    return ((W + TILE - 1) // TILE) * ((H + TILE - 1) // TILE)


def rank_tiles(W, H, rank, world):
    """(first_tile, tile_stride, count) of `rank`'s share, and the padded per-rank slab size."""
    nt = num_tiles(W, H)
    per = (nt + world - 1) // world
    count = len(range(rank, nt, world))
    return rank, world, count, per


def tile_pixels(W, H, first, stride, count):
    """Global (x, y) of every slab pixel (tile-major, row-major inside a tile); -1 outside the frame."""
    tx = (W + TILE - 1) // TILE
    tiles = first + stride * np.arange(count, dtype=np.int64)
    ly, lx = np.divmod(np.arange(TILE * TILE), TILE)
    x = (tiles[:, None] % tx) * TILE + lx[None, :]
    y = (tiles[:, None] // tx) * TILE + ly[None, :]
    inside = (x < W) & (y < H)
    return np.where(inside, x, -1).reshape(-1), np.where(inside, y, -1).reshape(-1)


def unshuffle_reference(slabs, W, H):
    """slabs: (R, per * 256, 3) -> (H, W, 3) frame (host mirror of vr_unshuffle_tiles_device)."""
    R = slabs.shape[0]
    per = slabs.shape[1] // (TILE * TILE)
    img = np.zeros((H, W, 3), slabs.dtype)
    for r in range(R):
        x, y = tile_pixels(W, H, r, R, per)
        m = x >= 0
        img[y[m], x[m]] = slabs[r][m]
    return img


def render_local(dev, camera, params, W, H, rank, world, slab, frame, stream_ptr):
    """This rank's share of one frame (device buffers are torch tensors). World 1 renders straight
    into `frame`; otherwise the rank's interleaved tiles go into its packed `slab`. Asynchronous on
    the stream; the frame's outcome is checked by `finish_local`."""
    first, stride, count, per = rank_tiles(W, H, rank, world)
    if world == 1:
        dev.render_tiles_device(camera, params, W, H, 0, 1, count, False, frame.data_ptr(), stream_ptr)
    else:
        dev.render_tiles_device(camera, params, W, H, first, stride, count, True, slab.data_ptr(), stream_ptr)


def finish_local(dev, camera, params, W, H, rank, world, slab, frame, stream_ptr, retries=2):
    """Waits for this rank's share and surfaces its outcome (vr_synchronize): a share that outgrew
    the record buffers sized from earlier frames is rendered again (they have been grown); pixels
    over every per-ray capacity raise VRError (VR_ERR_OVERFLOW), never a silent NaN frame."""
    from . import _lib as L
    for attempt in range(retries + 1):
        try:
            dev.synchronize()
            return
        except L.VRError as e:
            if attempt == retries or e.status != L.VR_ERR_RETRY:
                raise
        render_local(dev, camera, params, W, H, rank, world, slab, frame, stream_ptr)


def gather_frame(dev, W, H, rank, world, slab, slabs, frame, stream_ptr, dist, via_host=False):
    """Gather every rank's slab to rank 0 (one RCCL gather over xGMI) and unshuffle there.
    via_host: gather CPU copies instead (gloo rehearsal of the N > 1 path on one GPU)."""
    if world == 1:
        return
    per = slab.numel() // (TILE * TILE * 3)
    if via_host:
        import torch
        torch.cuda.synchronize()
        host = [torch.empty_like(slab, device="cpu") for _ in range(world)] if rank == 0 else None
        dist.gather(slab.cpu(), host, dst=0)
        if rank == 0:
            slabs.copy_(torch.stack(host).to(slabs.device))
    else:
        dist.gather(slab, list(slabs.unbind(0)) if rank == 0 else None, dst=0)
    if rank == 0:
        dev.unshuffle_tiles_device(slabs.data_ptr(), world, per, W, H, frame.data_ptr(), stream_ptr)
