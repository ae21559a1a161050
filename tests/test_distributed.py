"""Multi-GPU path on CPU: row sharding covers the image exactly once, and the
gather + reassembly of bench.py/distributed.py rebuilds the image over real
world_size-2/3 gloo process groups -- from synthetic (y, x) tiles, and from
shards each rank RENDERS on a host context (rtw_render_rows, the GPU path's
per-sample code on host threads), bit-identical to a one-process render."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_pkg


def test_shard_rows_match_library(rtw):
    L = rtw.lib()
    d = rtw.distributed
    for H in (1, 15, 16, 17, 800, 2160):
        for rpb in (1, 8, 16):
            for n in (1, 2, 3, 4, 8):
                allrows = []
                for s in range(n):
                    rows = d.shard_rows(H, rpb, n, s)
                    assert len(rows) == L.rtw_shard_rows(H, rpb, n, s)
                    assert len(rows) <= d.tile_rows_capacity(H, rpb, n)
                    allrows += rows
                assert sorted(allrows) == list(range(H))
                src, dst = d.reassembly_index(H, rpb, n)
                assert sorted(dst) == list(range(H))


def test_shard_image_row_matches_reassembly(rtw):
    """The library's one row map (rtw_shard_image_row: render kernels and the multi-GPU
    pack/unpack) equals the reassembly index of the gather, and places every image row
    exactly once across the shards' tiles."""
    L = rtw.lib()
    d = rtw.distributed
    for H in (1, 15, 17, 800, 2160):
        for rpb in (1, 8, 16):
            for n in (1, 2, 3, 8):
                cap = d.tile_rows_capacity(H, rpb, n)
                src, dst = d.reassembly_index(H, rpb, n)
                got = {}
                for s in range(n):
                    for r in range(cap):
                        y = L.rtw_shard_image_row(rpb, n, s, r)
                        if y < H:
                            assert y not in got.values()
                            got[s * cap + r] = y
                assert got == dict(zip(src, dst))
                assert sorted(got.values()) == list(range(H))
    assert L.rtw_shard_image_row(8, 2, 2, 0) == 0xFFFFFFFF


BAL = 0x80000000  # RTW_ROWS_BALANCED


def test_balanced_shards_split_the_rest_evenly(rtw):
    """rows_per_block | RTW_ROWS_BALANCED: the library's row map (rtw_shard_image_row_h, rtw_shard_rows -- the
    render kernels' and the multi-GPU pack/unpack's rtw_shard_row) equals the Python restatement and the
    reassembly index, places every image row exactly once, and the shards' row counts differ by at most the
    left-over share `sub` (C2 at 8 ranks, 8-row blocks: 100 rows each instead of 104 / 96)."""
    L = rtw.lib()
    d = rtw.distributed
    for H in (1, 7, 15, 17, 225, 800, 1080, 2160):
        for rpb in (1, 4, 8, 16):
            for n in (1, 2, 3, 4, 8):
                f = rpb | BAL
                cap = d.tile_rows_capacity(H, f, n)
                src, dst = d.reassembly_index(H, f, n)
                got, counts = {}, []
                for sh in range(n):
                    rows = d.shard_rows(H, f, n, sh)
                    assert len(rows) == L.rtw_shard_rows(H, f, n, sh)
                    counts.append(len(rows))
                    assert d.shard_tile_rows(H, f, n, sh) <= cap and cap % rpb == 0
                    for r in range(cap):
                        y = L.rtw_shard_image_row_h(H, f, n, sh, r)
                        assert y == (d.shard_row(H, f, n, sh, r) if r < d.shard_tile_rows(H, f, n, sh) or y >= H else y)
                        if y < H and r < d.shard_tile_rows(H, f, n, sh):
                            assert y not in got.values()
                            got[sh * cap + r] = y
                assert got == dict(zip(src, dst))
                assert sorted(got.values()) == list(range(H))
                full = H // (rpb * n)
                sub = -(-(H - full * rpb * n) // n)
                assert max(counts) - min(counts) <= sub
                # plain layout: the same rows as rtw_shard_image_row
                for sh in range(n):
                    for r in range(d.tile_rows_capacity(H, rpb, n)):
                        assert L.rtw_shard_image_row_h(H, rpb, n, sh, r) == L.rtw_shard_image_row(rpb, n, sh, r)
    assert [len(d.shard_rows(800, 8 | BAL, 8, sh)) for sh in range(8)] == [100] * 8
    assert L.rtw_shard_image_row(8 | BAL, 2, 0, 0) == 0xFFFFFFFF  # the plain map has no height: refused


def test_multi_create_rejects_bad_args(rtw):
    import ctypes as C
    h = C.c_void_p()
    assert rtw.lib().rtw_multi_create(None, 0, C.byref(h)) == rtw._abi.RTW_E_INVALID
    assert rtw.lib().rtw_multi_create(None, 1, None) == rtw._abi.RTW_E_INVALID


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world_size, port, H, W, rpb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    pkg = load_pkg()
    d = pkg.distributed
    cap = d.tile_rows_capacity(H, rpb, world_size)
    rows = d.shard_rows(H, rpb, world_size, rank)
    tile = torch.zeros((cap * W, 4), dtype=torch.float32)
    t = tile.view(cap, W, 4)
    for r, y in enumerate(rows):          # "render": pixel value encodes (y, x)
        t[r, :, 0] = y
        t[r, :, 1] = torch.arange(W, dtype=torch.float32)
        t[r, :, 3] = 7
    src, dst = d.reassembly_index(H, rpb, world_size)
    image = torch.zeros((H, W, 4)) if rank == 0 else None
    glist = [torch.empty_like(tile) for _ in range(world_size)] if rank == 0 else None
    d.gather_tiles(tile, image, glist, torch.tensor(src), torch.tensor(dst), W, world_size, rank)
    if rank == 0:
        q.put(image.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size,H,rpb", [(2, 45, 16), (2, 37, 8), (3, 20, 4)])
def test_gather_reassembles_image_gloo(world_size, H, rpb):
    W = 11
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world_size, port, H, W, rpb, q)) for r in range(world_size)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(img[:, :, 0], np.repeat(np.arange(H, dtype=np.float32)[:, None], W, 1))
    assert np.array_equal(img[:, :, 1], np.repeat(np.arange(W, dtype=np.float32)[None, :], H, 0))
    assert (img[:, :, 3] == 7).all()


def _render_worker(rank, world_size, port, W, spp, rpb, q):
    """One rank: its shard of Book-1 rendered on a host context (rtw_render_rows), gathered to rank 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    pkg = load_pkg()
    d = pkg.distributed
    arr = pkg.flatten(pkg.worlds.generate_world(0, "book1"))
    world = pkg.World(arr, device=pkg._abi.RTW_DEVICE_CPU, tuning={"cpu_threads": 2})
    cam = pkg.book1_camera(image_width=W, aspect_ratio=1.5, spp=spp).init()
    H = cam.derived.image_height
    cap = d.tile_rows_capacity(H, rpb, world_size)
    tile = np.zeros((cap * W, 4), np.float32)
    d.render_rows_host(world, cam, rpb, world_size, rank, 0, spp, tile, seed=13)
    src, dst = d.reassembly_index(H, rpb, world_size)
    image = torch.zeros((H, W, 4)) if rank == 0 else None
    glist = [torch.empty((cap * W, 4)) for _ in range(world_size)] if rank == 0 else None
    d.gather_tiles(torch.from_numpy(tile), image, glist, torch.tensor(src), torch.tensor(dst), W, world_size, rank)
    if rank == 0:
        q.put(image.numpy().reshape(-1, 4))
    dist.barrier()
    world.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size,rpb", [(2, 8), (3, 4), (3, 8 | BAL)])
def test_gather_of_rendered_shards_gloo(rtw, world_size, rpb):
    """Each rank renders its row-interleaved shard (main.zig:314-326's split, made shardable) and rank 0
    gathers and reassembles: the image equals a single-process host render of the whole frame bit for bit
    (the counter-based RNG keys every sample by (seed, pixel, sample))."""
    W, spp = 60, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_render_worker, args=(r, world_size, port, W, spp, rpb, q))
             for r in range(world_size)]
    for p in procs:
        p.start()
    img = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    world = rtw.World(arr, device=rtw._abi.RTW_DEVICE_CPU)
    cam = rtw.book1_camera(image_width=W, aspect_ratio=1.5, spp=spp).init()
    ref = np.zeros((cam.size, 4), np.float32)
    o = rtw._abi.render_opts()
    rtw._abi.check(rtw.lib().rtw_render_ex(world.handle, C.byref(cam.derived), 0, cam.size, 0, spp, 13,
                                           ref.ctypes.data, C.byref(o)), "rtw_render_ex")
    world.close()
    assert (ref[:, 3] == spp).all()
    assert np.array_equal(img, ref)


def _bench_line(out):
    import json
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("world_size", [2, 3])
def test_bench_torchrun_flow_on_host_backend(tmp_path, world_size):
    """bench.py's own N > 1 code path, end to end without a GPU: torchrun starts one process per rank,
    each renders its row-interleaved shard (--host-backend: a host context, rtw_render_rows), the tiles
    meet on rank 0 in one dist.gather (gloo), rank 0 reassembles the frame, the ranks' times are maxed and
    one JSON line is printed.  The frame equals bench.py's one-process frame bit for bit."""
    import subprocess
    import sys

    from conftest import REPO
    common = ["--host-backend", "--config", "c1", "--spp", "2", "--steps", "1", "--warmup", "0",
              "--no-cpu-baseline"]
    one = tmp_path / "one.npy"
    r1 = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *common, "--dump-image", str(one)],
                        capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r1.returncode == 0, r1.stderr[-2000:]
    many = tmp_path / "many.npy"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    rn = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world_size}",
                         "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                         os.path.join(REPO, "bench.py"), "--gpus", str(world_size), *common,
                         "--dump-image", str(many)], capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    assert rn.returncode == 0, rn.stderr[-2000:]
    d = _bench_line(rn.stdout)
    assert d["n_gpus"] == world_size and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["exchange"] == {"mode": "torchrun", "rccl_ranks": world_size, "backend": "gloo"}
    assert (d["config"]["width"], d["config"]["height"]) == (400, 225)
    assert abs(d["value"] - 400 * 225 * 2 / (d["ms_per_step"] / 1e3) / 1e6) <= 0.01 * d["value"]
    a, b = np.load(one), np.load(many)
    assert a.shape == (225, 400, 4) and (a[..., 3] == 2).all()
    assert np.array_equal(a, b)
