"""Pixel-tile sharding of one frame over R ranks (one process per GPU) and its reassembly.

The reference parallelises the pixel loop with OpenMP only (test_integrators.h:164); pixels are
independent, so the frame is the data-parallel axis. The frame is cut into 16x16 tiles numbered
row-major; rank r renders tiles r, r + R, r + 2R, ... (interleaved, which balances dense and empty
regions of the image). Rank 0 renders its tiles straight into the row-major frame; every other rank
renders into a packed slab, sends it to rank 0 (point-to-point RCCL sends in one batch, so the links
run concurrently and nothing is sent to the root itself) and the device unshuffle kernel scatters
those slabs into the frame. `unshuffle_reference` is the host mirror of that kernel used by the CPU
tests.
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


def unshuffle_reference(slabs, W, H, first=0, stride=None):
    """slabs: (n, per * 256, 3), slab k = rank first + k of a stride-way split (stride defaults to n)
    -> (H, W, 3) frame holding those ranks' tiles (host mirror of vr_unshuffle_tiles_part_device)."""
    n = slabs.shape[0]
    stride = n if stride is None else stride
    per = slabs.shape[1] // (TILE * TILE)
    img = np.zeros((H, W, 3), slabs.dtype)
    for k in range(n):
        x, y = tile_pixels(W, H, first + k, stride, per)
        m = x >= 0
        img[y[m], x[m]] = slabs[k][m]
    return img


def render_local(dev, camera, params, W, H, rank, world, slab, frame, stream_ptr):
    """This rank's share of one frame (device buffers are torch tensors). Rank 0 renders its tiles
    straight into `frame` (world 1: the whole frame); every other rank into its packed `slab`.
    Asynchronous on the stream; the frame's outcome is checked by `finish_local`."""
    first, stride, count, per = rank_tiles(W, H, rank, world)
    if count == 0:
        return
    if rank == 0:
        dev.render_tiles_device(camera, params, W, H, first, stride, count, False, frame.data_ptr(), stream_ptr)
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
    """Ranks 1 .. world-1 send their slabs to rank 0 (one batch of point-to-point RCCL sends over xGMI:
    the links run concurrently, the root sends nothing to itself) and rank 0 unshuffles them into the
    frame it already holds its own tiles in. slabs (rank 0): (world - 1, per * 256 * 3).
    via_host: the same exchange through CPU copies (gloo rehearsal of the N > 1 path on one GPU)."""
    if world == 1:
        return
    per = (slab if rank else slabs[0]).numel() // (TILE * TILE * 3)
    if via_host:
        import torch
        torch.cuda.synchronize()
        if rank == 0:
            for r in range(1, world):
                host = torch.empty(slabs[r - 1].shape, dtype=slabs.dtype)
                dist.recv(host, src=r)
                slabs[r - 1].copy_(host.to(slabs.device))
        else:
            dist.send(slab.cpu(), dst=0)
    else:
        if rank == 0:
            ops = [dist.P2POp(dist.irecv, slabs[r - 1], r) for r in range(1, world)]
        else:
            ops = [dist.P2POp(dist.isend, slab, 0)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if rank == 0:
        dev.unshuffle_tiles_part_device(slabs.data_ptr(), 1, world - 1, world, per, W, H, frame.data_ptr(), stream_ptr)
