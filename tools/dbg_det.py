"""DIAGNOSTIC: run-to-run determinism of the wavefront path on a BASELINE config
(counters + image hash per repetition, fresh and reused worlds)."""
import ctypes as C
import hashlib
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

rtw = importlib.import_module("zig-raytracing-weekend_amd")
name = sys.argv[1] if len(sys.argv) > 1 else "c4"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 4
cfg = rtw.configs.CONFIGS[name]
arr = rtw.flatten(cfg.objects())
cam = cfg.camera()
cam.samples_per_pixel = 2
cam.init()
acc = torch.zeros((cam.size, 4), dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()
w = rtw.World(arr)
for r in range(reps):
    if r == reps // 2:
        w.close()
        w = rtw.World(arr)
    acc.zero_()
    cnt = torch.zeros(8, dtype=torch.int64, device="cuda")
    opts = rtw._abi.RtwRenderOpts(batch, 0, cnt.data_ptr())
    torch.cuda.synchronize()
    rtw._abi.check(rtw.lib().rtw_render_device(w.handle, C.byref(cam.derived), 0, cam.size, 0, 2, 0, acc.data_ptr(),
                                               C.c_void_p(stream.cuda_stream), C.byref(opts)), "render")
    torch.cuda.synchronize()
    h = hashlib.sha1(acc.cpu().numpy().tobytes()).hexdigest()[:12]
    print(r, cnt.cpu().tolist()[:4], h, flush=True)
