"""BASELINE config 1 (Book-1, 400x225, 10 spp, depth 50: the reference's CPU path) on the
product's HOST backend (rtw_scene_create(desc, RTW_DEVICE_CPU), csrc/rtw_cpu.hip) next to the
oracle (the reference restated in C), both with the reference's 8 threads (main.zig:41) and
with the CPUs this process may use.  One JSON line.  No GPU involved."""
import ctypes as C
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402


def main():
    rtw = importlib.import_module("zig-raytracing-weekend_amd")
    import bench
    import oracle as O
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"))
    cam = rtw.book1_camera(image_width=400, aspect_ratio=16 / 9, spp=10, max_depth=50).init()
    ow = O.World(arr.spheres, arr.materials, arr.textures)
    ocam = O.camera(image_width=400, aspect_ratio=16 / 9, samples_per_pixel=10, max_depth=50, background_mode=1)
    quota = bench.cpu_quota_cores()
    out = {"config": "c1: Book-1 400x225 x 10 spp, depth 50", "unit": "Msamples/s", "cpu_quota_cores": quota,
           "cores_all": os.cpu_count()}
    for th in sorted({8, quota}):
        world = rtw.World(arr, device=rtw._abi.RTW_DEVICE_CPU, tuning={"cpu_threads": th})
        buf = np.zeros((cam.size, 4), np.float32)
        best = 1e9
        for _ in range(3):
            buf[:] = 0
            t = time.perf_counter()
            rtw._abi.check(rtw.lib().rtw_render(world.handle, C.byref(cam.derived), 0, cam.size, 0, 10, 0,
                                                buf.ctypes.data, None, rtw._abi.PROGRESS_FN(0), None), "render")
            best = min(best, time.perf_counter() - t)
        world.close()
        t = time.perf_counter()
        ref = ow.render_pixels(ocam, 0, np.arange(cam.size, dtype=np.uint32), 0, 10, threads=th)
        to = time.perf_counter() - t
        err = float((np.abs(buf[:, :3] - ref[:, :3]) / np.maximum(1.0, np.abs(ref[:, :3]))).max())
        out[f"threads_{th}"] = {"host_backend": round(cam.size * 10 / best / 1e6, 3),
                                "oracle": round(cam.size * 10 / to / 1e6, 3), "max_rel_err": err}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
