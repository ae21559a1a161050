"""Host-core probe for the CPU baseline (bench.py cpu_baseline): what the box
reports (os.cpu_count, affinity, cgroup quota) and how the oracle's render rate
scales with threads on a fixed C2 row sample.  Test infrastructure only."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import importlib  # noqa: E402

import numpy as np  # noqa: E402


def main():
    print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        if os.path.exists(p):
            print(p, open(p).read().strip())
    pkg = importlib.import_module("zig-raytracing-weekend_amd")
    import oracle as O
    cfg = pkg.configs.CONFIGS["c2"]
    arr = pkg.flatten(cfg.objects())
    ow = O.World.from_arrays(arr)
    cam = cfg.camera().init()
    d = cam.derived
    ocam = O.camera(aspect_ratio=cam.aspect_ratio, image_width=d.image_width, image_height=d.image_height,
                    samples_per_pixel=d.samples_per_pixel, max_depth=d.max_depth, background=tuple(d.background),
                    background_mode=d.background_mode, vfov=cam.vfov, lookfrom=cam.lookfrom, lookat=cam.lookat,
                    vup=cam.vup, defocus_angle=cam.defocus_angle, focus_dist=cam.focus_dist,
                    pixel_offset=d.pixel_offset)
    W, H = d.image_width, d.image_height
    rows = np.arange(0, H, 8)
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    for th in [int(x) for x in (sys.argv[1:] or ["8", "16", "32", "64", "128", "256"])]:
        spp = 2 * th
        t = time.perf_counter()
        ow.render_pixels(ocam, 0, pix, 0, spp, threads=th)
        dt = time.perf_counter() - t
        print(f"threads {th:4d}  spp {spp:4d}  {dt:7.2f} s  {len(pix) * spp / dt / 1e6:8.3f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
