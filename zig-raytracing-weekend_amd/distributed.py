"""Multi-GPU image sharding (one process per GPU, torch.distributed over RCCL).

The reference splits one image over 8 CPU threads in contiguous chunks
(src/main.zig:314-326), which is load-imbalanced (sky rows are cheap, ground
rows expensive).  Here rank r of N renders the row blocks b (of
``rows_per_block`` rows) with b % N == r -- interleaved, so every rank gets
the same mix of sky and ground -- into a compact float4 tile, and the tiles
meet on rank 0 in ONE gather (the only data-path collective: there is no other
exchange in the algorithm).  The counter-based RNG keys every sample by
(seed, pixel, sample), so the gathered image is bit-identical to a 1-GPU
render for any N.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Tuple

from . import _abi


def shard_row(height: int, rows_per_block: int, n_shards: int, shard: int, r: int) -> int:
    """Image row of tile row r of `shard` (>= height: padding): rtw_shard_row (rtw_layout.h) restated.  Plain
    layout: row block b of rpb rows goes to shard b % n_shards.  rows_per_block | RTW_ROWS_BALANCED: rounds of
    n_shards blocks dealt in alternating order (round k: shard s takes block position s if k is even, else
    n_shards - 1 - s), then the left-over rows split evenly (`sub` consecutive rows each, in one more block slot
    of the tile)."""
    rpb = rows_per_block & ~_abi.RTW_ROWS_BALANCED
    if not rows_per_block & _abi.RTW_ROWS_BALANCED:
        return ((r // rpb) * n_shards + shard) * rpb + r % rpb
    full = height // (rpb * n_shards)
    k = r // rpb
    pos = n_shards - 1 - shard if k % 2 else shard  # rounds dealt in alternating order
    if r < full * rpb:
        return (k * n_shards + pos) * rpb + r % rpb
    y0 = full * rpb * n_shards
    sub = (height - y0 + n_shards - 1) // n_shards
    i = r - full * rpb
    return y0 + pos * sub + i if i < sub else 0xFFFFFFFF


def shard_tile_rows(height: int, rows_per_block: int, n_shards: int, shard: int) -> int:
    """Tile rows (whole blocks, padding included) of `shard` (rtw_shard_tile_rows)."""
    rpb = rows_per_block & ~_abi.RTW_ROWS_BALANCED
    if rows_per_block & _abi.RTW_ROWS_BALANCED:
        full = height // (rpb * n_shards)
        y0 = full * rpb * n_shards
        sub = (height - y0 + n_shards - 1) // n_shards
        pos = n_shards - 1 - shard if full % 2 else shard
        return full * rpb + (rpb if pos * sub < height - y0 else 0)
    n_blk = (height + rpb - 1) // rpb
    return ((n_blk - shard + n_shards - 1) // n_shards) * rpb if n_blk > shard else 0


def shard_rows(height: int, rows_per_block: int, n_shards: int, shard: int) -> List[int]:
    """Image rows owned by `shard`, in tile order (rtw_shard_rows / map_row)."""
    rows = []
    for r in range(shard_tile_rows(height, rows_per_block, n_shards, shard)):
        y = shard_row(height, rows_per_block, n_shards, shard, r)
        if y < height:
            rows.append(y)
    return rows


def tile_rows_capacity(height: int, rows_per_block: int, n_shards: int) -> int:
    """Rows of the (padded) per-rank tile: equal on every rank so the gather is uniform (rtw_shard_capacity)."""
    return max(shard_tile_rows(height, rows_per_block, n_shards, s) for s in range(n_shards))


def reassembly_index(height: int, rows_per_block: int, n_shards: int) -> Tuple[List[int], List[int]]:
    """(src, dst): row src of the stacked [n_shards * cap] tile buffer -> image row dst."""
    cap = tile_rows_capacity(height, rows_per_block, n_shards)
    src, dst = [], []
    for s in range(n_shards):
        for r in range(cap):
            y = shard_row(height, rows_per_block, n_shards, s, r)
            if y < height:
                src.append(s * cap + r)
                dst.append(y)
    return src, dst


def render_rows_host(world, cam, rows_per_block: int, n_shards: int, shard: int, spp_begin: int, spp_end: int,
                     tile, seed: int = 0, running=None, progress=None, spp_batch: int = 0) -> None:
    """rtw_render_rows: this shard's rows x samples [spp_begin, spp_end) onto a HOST float32 tile
    [rows_in_shard * W, 4] (blocking), on a GPU context or a host context (RTW_DEVICE_CPU) -- one process
    per rank renders its shard without a GPU (the gloo tests), bit-identical to the device path."""
    assert tile.dtype.name == "float32" and tile.flags.c_contiguous
    rows = _abi.lib().rtw_shard_rows(cam.derived.image_height, rows_per_block, n_shards, shard)
    assert tile.size >= rows * cam.derived.image_width * 4
    opts = _abi.render_opts(spp_batch=spp_batch, running=running, progress=progress)
    rc = _abi.lib().rtw_render_rows(world.handle, C.byref(cam.derived), rows_per_block, n_shards, shard, spp_begin,
                                    spp_end, seed, tile.ctypes.data, C.byref(opts))
    _abi.check(rc, "rtw_render_rows")


class ShardedRender:
    """Per-rank state of a row-interleaved render + gather (used by bench.py)."""

    def __init__(self, world, cam, rank: int, world_size: int, rows_per_block: int = 16, device=None):
        import torch

        self.world, self.cam = world, cam
        self.rank, self.world_size, self.rpb = rank, world_size, rows_per_block
        self.W, self.H = cam.derived.image_width, cam.derived.image_height
        self.cap = tile_rows_capacity(self.H, rows_per_block, world_size)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.tile = torch.zeros((self.cap * self.W, 4), dtype=torch.float32, device=dev)
        src, dst = reassembly_index(self.H, rows_per_block, world_size)
        self.src = torch.tensor(src, device=dev)
        self.dst = torch.tensor(dst, device=dev)
        self.gather_list = ([torch.empty_like(self.tile) for _ in range(world_size)]
                            if (world_size > 1 and rank == 0) else None)
        self.image = torch.zeros((self.H, self.W, 4), dtype=torch.float32, device=dev) if rank == 0 else None
        self.rows = len(shard_rows(self.H, rows_per_block, world_size, rank))

    def render(self, spp_begin: int, spp_end: int, seed: int = 0, stream=None, spp_batch: int = 0,
               counters: Optional[int] = None, sync: bool = False, timing=None) -> None:
        """Enqueue this rank's rows x samples [spp_begin, spp_end) on `stream`.
        timing: optional _abi.RtwKernelTiming filled with per-kernel device time
        (the call then synchronises the stream).  A CPU tile (a host context, RTW_DEVICE_CPU: bench.py
        --host-backend) renders through rtw_render_rows, blocking."""
        import torch
        self.tile.zero_()
        if self.tile.device.type == "cpu":
            render_rows_host(self.world, self.cam, self.rpb, self.world_size, self.rank, spp_begin, spp_end,
                             self.tile.numpy(), seed=seed, spp_batch=spp_batch)
            return
        if stream is not None and stream != torch.cuda.current_stream(self.tile.device):
            stream.wait_stream(torch.cuda.current_stream(self.tile.device))  # the zeroing precedes the render
        flags = 0 if sync else _abi.RTW_RENDER_NO_SYNC
        opts = _abi.RtwRenderOpts(spp_batch, flags, counters, C.pointer(timing) if timing is not None else None)
        rc = _abi.lib().rtw_render_rows_device(self.world.handle, C.byref(self.cam.derived), self.rpb,
                                               self.world_size, self.rank, spp_begin, spp_end, seed,
                                               self.tile.data_ptr(),
                                               C.c_void_p(stream.cuda_stream if stream is not None else 0),
                                               C.byref(opts))
        _abi.check(rc, "rtw_render_rows_device")

    def gather(self) -> None:
        """Tiles -> rank 0 (one RCCL gather), then scatter rows into the image."""
        gather_tiles(self.tile, self.image, self.gather_list, self.src, self.dst, self.W, self.world_size,
                     self.rank)


def gather_tiles(tile, image, gather_list, src, dst, W: int, world_size: int, rank: int) -> None:
    import torch
    import torch.distributed as dist

    if world_size > 1:
        dist.gather(tile, gather_list=gather_list, dst=0)
        if rank == 0:
            allt = torch.stack(gather_list).view(-1, W, 4)
            image.index_copy_(0, dst, allt.index_select(0, src))
    else:
        image.index_copy_(0, dst, tile.view(-1, W, 4).index_select(0, src))


class MultiDeviceRender:
    """One process driving N devices through the C ABI (rtw_multi_*, csrc/rtw_multi.hip):
    the same row-interleaved shards as ShardedRender, rendered concurrently on each
    device's context, then ONE grouped RCCL send/recv of the tiles to device 0 and a
    row scatter into the frame there.  worlds[k] is a World on device k (same scene);
    worlds[0]'s device holds the frame.  Bit-identical to a 1-GPU render for any N."""

    def __init__(self, worlds, rows_per_block: int = 8):
        self.worlds = list(worlds)
        self.rpb = rows_per_block
        n = len(self.worlds)
        handles = (C.c_void_p * n)(*[w.handle.value for w in self.worlds])
        h = C.c_void_p()
        _abi.check(_abi.lib().rtw_multi_create(handles, n, C.byref(h)), "rtw_multi_create")
        self.handle = h

    def render_device(self, cam, spp_begin: int, spp_end: int, d_accum: int, seed: int = 0, stream=None,
                      fresh: bool = False, sync: bool = True, spp_batch: int = 0, running=None,
                      progress=None) -> None:
        """Frame float4[W*H] at device pointer d_accum (worlds[0]'s device): rgb += samples
        [spp_begin, spp_end), w = spp_end (fresh: the range starts from zero).  running (a ctypes
        c_uint8, 0 = stop) and progress(done, total) -> True are polled between spp batches; a stop
        raises RtwError(RTW_E_CANCELLED) with the finished batches gathered into the frame."""
        flags = (0 if sync else _abi.RTW_RENDER_NO_SYNC) | (_abi.RTW_RENDER_FRESH if fresh else 0)
        opts = _abi.render_opts(spp_batch=spp_batch, flags=flags, running=running, progress=progress)
        rc = _abi.lib().rtw_render_multi_device(self.handle, C.byref(cam.derived), self.rpb, spp_begin, spp_end,
                                                seed, d_accum,
                                                C.c_void_p(stream.cuda_stream if stream is not None else 0),
                                                C.byref(opts))
        _abi.check(rc, "rtw_render_multi_device")

    def render_host(self, cam, spp_begin: int, spp_end: int, accum, seed: int = 0, spp_batch: int = 0,
                    running=None, progress=None) -> None:
        """Same on a host numpy float32 [W*H, 4] buffer (blocking, rtw_render_multi_ex)."""
        assert accum.dtype.name == "float32" and accum.flags.c_contiguous and accum.size == cam.size * 4
        opts = _abi.render_opts(spp_batch=spp_batch, running=running, progress=progress)
        rc = _abi.lib().rtw_render_multi_ex(self.handle, C.byref(cam.derived), self.rpb, spp_begin, spp_end, seed,
                                            accum.ctypes.data, C.byref(opts))
        _abi.check(rc, "rtw_render_multi_ex")

    def info(self) -> Tuple[int, int]:
        """(devices, ranks of the RCCL communicator as ncclCommCount reports them)."""
        n, r = C.c_uint32(), C.c_int()
        _abi.check(_abi.lib().rtw_multi_info(self.handle, C.byref(n), C.byref(r)), "rtw_multi_info")
        return int(n.value), int(r.value)

    def close(self) -> None:
        if getattr(self, "handle", None) and self.handle.value:
            _abi.lib().rtw_multi_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
