"""Camera / SharedStateImageWriter / Task mirror of src/camera.zig, with
``Camera.render`` routed through the C ABI to the gfx950 kernels.

Reference call stack being replaced (src/main.zig:49-69, 314-326)::

    startRender -> 8 x RenderThread.start(Task{thread_idx, chunk_size = size/8})
        -> renderFn -> Camera.render(raytrace, task)        (src/camera.zig:93-116)

Here ``Camera.render(state, task)`` issues ONE ``rtw_render`` for the task's
pixel chunk and the whole sample range; the per-sample loop runs on the GPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from . import _abi
from .scene import World


@dataclass
class Task:
    """camera.zig:19"""
    thread_idx: int
    chunk_size: int


class SharedStateImageWriter:
    """camera.zig:22-67: float4 ColorAndSamples buffer + u8 RGBA texture."""

    def __init__(self, image_width: int, image_height: int):
        self.width, self.height = int(image_width), int(image_height)
        n = self.width * self.height
        self.buffer = np.zeros((n, 4), np.float32)
        self.buffer[:, 3] = 1.0                      # init / scrub: {0,0,0,1} (camera.zig:34-45)
        self.texture_buffer = np.zeros((n, 4), np.uint8)

    def scrub(self):
        self.buffer[:] = 0.0
        self.buffer[:, 3] = 1.0

    def update_texture(self, begin: int = 0, end: Optional[int] = None):
        """toGamma2 texel update of writeColor (camera.zig:58-65) for [begin, end)."""
        end = self.buffer.shape[0] if end is None else end
        if end <= begin:
            return
        src = np.ascontiguousarray(self.buffer[begin:end])
        dst = np.zeros((end - begin, 4), np.uint8)
        _abi.check(_abi.lib().rtw_texture_from_accum(src.ctypes.data, end - begin, dst.ctypes.data),
                   "rtw_texture_from_accum")
        self.texture_buffer[begin:end] = dst

    def image(self) -> np.ndarray:
        return self.texture_buffer.reshape(self.height, self.width, 4)

    def save_ppm(self, path: str, style: int = _abi.RTW_PPM_WRITECOLOR) -> None:
        """P3 PPM of the accumulator (color.zig writeColor / stdout.zig formats)."""
        from .output import write_ppm
        write_ppm(path, self.buffer, self.width, self.height, style)

    def save_png(self, path: str) -> None:
        """RGBA8 PNG of the texture buffer (update_texture first)."""
        from .output import write_png
        write_png(path, self.texture_buffer, self.width, self.height)


@dataclass
class Camera:
    """camera.zig:69-91 (defaults are the reference's), plus the two knobs the
    reference hard-codes: background_mode (gradient = the commented Book-1 sky,
    camera.zig:204-206) and pixel_offset (the +1 of camera.zig:100-101)."""
    aspect_ratio: float = 16.0 / 9.0
    image_width: int = 800
    image_height: int = 0
    samples_per_pixel: int = 100
    max_depth: int = 16
    background: tuple = (0.0, 0.0, 0.0)
    background_mode: int = _abi.RTW_BG_CONSTANT
    vfov: float = 20.0
    lookfrom: tuple = (13.0, 2.0, 3.0)
    lookat: tuple = (0.0, 0.0, 0.0)
    vup: tuple = (0.0, 1.0, 0.0)
    defocus_angle: float = 0.6
    focus_dist: float = 10.0
    pixel_offset: int = 1
    derived: Optional[_abi.RtwCamera] = field(default=None, repr=False)

    def params(self) -> _abi.RtwCameraParams:
        p = _abi.RtwCameraParams()
        p.aspect_ratio = self.aspect_ratio
        p.image_width = self.image_width
        p.image_height = self.image_height
        p.samples_per_pixel = self.samples_per_pixel
        p.max_depth = self.max_depth
        p.background_mode = self.background_mode
        p.background[:] = list(self.background)
        p.vfov = self.vfov
        p.lookfrom[:] = list(self.lookfrom)
        p.lookat[:] = list(self.lookat)
        p.vup[:] = list(self.vup)
        p.defocus_angle = self.defocus_angle
        p.focus_dist = self.focus_dist
        p.pixel_offset = self.pixel_offset
        return p

    def init(self) -> "Camera":
        """Camera.init (camera.zig:118-154) via rtw_camera_init."""
        c = _abi.RtwCamera()
        _abi.check(_abi.lib().rtw_camera_init(C.byref(self.params()), C.byref(c)), "rtw_camera_init")
        self.derived = c
        if self.image_height == 0:
            self.image_height = c.image_height
        return self

    @property
    def size(self) -> int:
        return int(self.derived.size)

    def render(self, state: "RayTraceState", task: Task) -> None:
        """Camera.render (camera.zig:93-116) for one Task, all samples."""
        if self.derived is None:
            self.init()
        start = task.thread_idx * task.chunk_size
        end = start + task.chunk_size
        self.render_range(state, start, end, 0, self.samples_per_pixel)

    def render_range(self, state: "RayTraceState", pix_begin: int, pix_end: int, spp_begin: int, spp_end: int,
                     progress: Optional[Callable[[int, int], bool]] = None, spp_batch: int = 0) -> None:
        """Samples [spp_begin, spp_end) of pixels [pix_begin, pix_end) through rtw_render_ex, polling the
        state's RenderThread.running flag (camera.zig:107) between sample batches (spp_batch, 0 = auto);
        progress(done, total) -> True stops.  A stop raises RtwError(RTW_E_CANCELLED) with the finished
        batches in the buffer (and the texture updated from them): every pixel's .w is the end of the last
        finished batch, so a resume from it adds no sample twice.  Exception: a host context (RTW_DEVICE_CPU)
        given spp_batch = 0 polls per pixel as camera.zig:107 does, so a stop there leaves each pixel at its
        own .w -- resume each pixel from its own .w, or pass a spp_batch."""
        w = state.writer
        buf = w.buffer
        assert buf.flags["C_CONTIGUOUS"] and buf.dtype == np.float32 and buf.shape == (self.size, 4)
        opts = _abi.render_opts(spp_batch=spp_batch, running=state.running, progress=progress)
        rc = _abi.lib().rtw_render_ex(state.world.handle, C.byref(self.derived), pix_begin, pix_end, spp_begin,
                                      spp_end, state.seed, buf.ctypes.data, C.byref(opts))
        w.update_texture(pix_begin, pix_end)
        _abi.check(rc, "rtw_render_ex")


@dataclass
class RayTraceState:
    """The parts of RayTraceState (src/main.zig:71-86) the render path reads."""
    camera: Camera
    writer: SharedStateImageWriter
    world: World
    seed: int = 0
    # RenderThread.running (src/main.zig:50, a Zig bool; true from RenderThread.start, main.zig:55): the
    # render polls it between sample batches (camera.zig:107), through rtw_render_opts.running
    running: C.c_uint8 = field(default_factory=lambda: C.c_uint8(1))

    def stop(self):
        """RenderThread.stop (src/main.zig:58-60): running = false."""
        self.running.value = 0

    def count_samples(self) -> float:
        """countSamples (src/main.zig:470-477): f32 sum of buffer[i][3] (progress / POWER)."""
        b = self.writer.buffer
        return float(_abi.lib().rtw_count_samples(b.ctypes.data, b.shape[0]))

    def samples_done(self) -> int:
        """Samples per pixel already in the buffer (writeColor stores the count in .w)."""
        return int(self.writer.buffer[:, 3].max()) if self.writer.buffer.size else 0

    def checkpoint(self, path: str, spp_done: int) -> None:
        """Write the accumulator + camera/seed/scene hash (rtw_checkpoint_write)."""
        h = C.c_uint64()
        _abi.check(_abi.lib().rtw_scene_hash(self.world.handle, C.byref(h)), "rtw_scene_hash")
        b = self.writer.buffer
        _abi.check(_abi.lib().rtw_checkpoint_write(path.encode(), C.byref(self.camera.derived), self.seed, h.value,
                                                   spp_done, b.ctypes.data), "rtw_checkpoint_write")

    def resume(self, path: str) -> int:
        """Load a checkpoint into the writer; refuses another scene, camera or seed.
        Returns the samples already done (render [done, spp) next)."""
        cam = _abi.RtwCamera()
        seed, h, done = C.c_uint64(), C.c_uint64(), C.c_uint32()
        b = self.writer.buffer
        # read into a scratch buffer: a refused checkpoint leaves the caller's accumulator untouched
        tmp = np.empty_like(b)
        _abi.check(_abi.lib().rtw_checkpoint_read(path.encode(), C.byref(cam), C.byref(seed), C.byref(h),
                                                  C.byref(done), tmp.ctypes.data, tmp.shape[0]),
                   "rtw_checkpoint_read")
        mine = C.c_uint64()
        _abi.check(_abi.lib().rtw_scene_hash(self.world.handle, C.byref(mine)), "rtw_scene_hash")
        if h.value != mine.value or seed.value != self.seed or bytes(cam) != bytes(self.camera.derived):
            raise _abi.RtwError(_abi.RTW_E_INVALID, "resume", "checkpoint is for another scene/camera/seed")
        b[...] = tmp
        self.writer.update_texture()
        return int(done.value)


def progressive_render(state: RayTraceState, spp_begin: int = 0, batch: int = 1,
                       on_batch: Optional[Callable[[int, float], bool]] = None) -> int:
    """Interactive-style render: samples [spp_begin, spp) in batches of `batch` over the
    whole image, refreshing the texture after each (what the UI shows) and calling
    on_batch(samples_done_per_pixel, count_samples()) -- return True to stop (the
    reference's Stop button, main.zig:58-60).  Consecutive batches are bit-identical to
    one render.  Returns the samples per pixel done."""
    cam = state.camera
    if cam.derived is None:
        cam.init()
    s = spp_begin
    spp = cam.samples_per_pixel
    while s < spp and state.running.value:
        e = min(spp, s + batch)
        cam.render_range(state, 0, cam.size, s, e)
        s = e
        if on_batch is not None and on_batch(s, state.count_samples()):
            break
    return s


def start_render(state: RayTraceState, number_of_threads: int = 8) -> None:
    """startRender (src/main.zig:314-326): scrub, Camera.init, 8 Tasks of size/8.

    The Tasks are issued back to back on the GPU (each one is a whole-chunk,
    all-samples launch sequence); the trailing size % 8 pixels are left
    unrendered exactly like the reference."""
    state.writer.scrub()
    state.camera.init()
    chunk = state.camera.size // number_of_threads
    for t in range(number_of_threads):
        state.camera.render(state, Task(t, chunk))


# ------------------------------------------------------------------ presets
def book1_camera(image_width: int = 1200, aspect_ratio: float = 1.5, spp: int = 500, max_depth: int = 50,
                 image_height: int = 0) -> Camera:
    """Book-1 cover camera (camera.zig defaults + gradient sky), BASELINE config 2 by default."""
    return Camera(aspect_ratio=aspect_ratio, image_width=image_width, image_height=image_height,
                  samples_per_pixel=spp, max_depth=max_depth, background_mode=_abi.RTW_BG_GRADIENT,
                  vfov=20.0, lookfrom=(13.0, 2.0, 3.0), lookat=(0.0, 0.0, 0.0), defocus_angle=0.6, focus_dist=10.0)


def earth_perlin_camera(image_width: int = 1920, spp: int = 512, max_depth: int = 50) -> Camera:
    """BASELINE config 5: constant (0.7,0.8,1.0) sky as RTNW, no defocus."""
    return Camera(aspect_ratio=16.0 / 9.0, image_width=image_width, samples_per_pixel=spp, max_depth=max_depth,
                  background=(0.7, 0.8, 1.0), background_mode=_abi.RTW_BG_CONSTANT, vfov=30.0,
                  lookfrom=(13.0, 2.0, 3.0), lookat=(0.0, 1.0, 0.0), defocus_angle=0.0, focus_dist=10.0)


def simple_light_camera(image_width: int = 800, spp: int = 100) -> Camera:
    """Camera{} defaults as modified by simpleLightWorld (src/main.zig:157-162)."""
    return Camera(image_width=image_width, samples_per_pixel=spp, max_depth=50, lookfrom=(26.0, 3.0, 6.0),
                  lookat=(0.0, 2.0, 0.0), vup=(0.0, 1.0, 0.0), defocus_angle=0.0)


def cornell_camera(image_width: int = 600, spp: int = 200, max_depth: int = 200) -> Camera:
    """cornellBox's camera (src/main.zig:194-202): 600x600, 200 spp, depth 200, black background."""
    return Camera(aspect_ratio=1.0, image_width=image_width, samples_per_pixel=spp, max_depth=max_depth, vfov=40.0,
                  lookfrom=(278.0, 278.0, -800.0), lookat=(278.0, 278.0, 0.0), vup=(0.0, 1.0, 0.0),
                  defocus_angle=0.0)


def cornell_smoke_camera(image_width: int = 600, spp: int = 200, max_depth: int = 50) -> Camera:
    """cornellBoxSmoke's camera (src/main.zig:238-246)."""
    return cornell_camera(image_width, spp, max_depth)

