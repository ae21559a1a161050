import sys, os, ctypes as C, numpy as np, importlib
sys.path.insert(0,'.'); sys.path.insert(0,'oracle')
rtw = importlib.import_module('zig-raytracing-weekend_amd'); import oracle as O
arr = rtw.flatten(rtw.worlds.generate_world(0,'book1'))
cam = rtw.book1_camera().init()
ow = O.World(arr.spheres, arr.materials, arr.textures)
ocam = O.camera(image_width=1200, aspect_ratio=1.5, samples_per_pixel=500, max_depth=50, background_mode=1)
for fr in ("0","1"):
    os.environ["RTW_FAST_REJECT"]=fr
    w = rtw.World(arr)
    out = np.zeros(3,np.float32)
    for pix,s in ((329008,250),):
        rtw._abi.check(rtw.lib().rtw_debug_sample(w.handle, C.byref(cam.derived), 0, pix, s, out.ctypes.data),"dbg")
        print(fr, pix, s, out, ow.sample(ocam,0,pix,s))
    w.close()
