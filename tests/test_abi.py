"""C-ABI boundary checks that need no GPU: the library loads, exports every
symbol include/rtw_gpu.h declares, its records have the header's sizes, and its
host-side halves (Camera.init, BVH build + flatten, toGamma2) agree bit-exactly
with the oracle."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "rtw_gpu.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(rtw_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_exports_every_header_symbol(rtw):
    lib = rtw.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(rtw._abi.SIGNATURES), set(names) ^ set(rtw._abi.SIGNATURES)
    assert lib.rtw_version() == 8


def test_struct_sizes_match_header(rtw, tmp_path):
    prog = tmp_path / "sizes.c"
    structs = ["rtw_sphere", "rtw_material", "rtw_texture", "rtw_image", "rtw_perlin", "rtw_scene_desc",
               "rtw_camera_params", "rtw_camera", "rtw_render_opts", "rtw_scene_stats", "rtw_tuning"]
    prog.write_text('#include <stdio.h>\n#include "rtw_gpu.h"\nint main(){' +
                    "".join(f'printf("%zu\\n", sizeof({s}));' for s in structs) + "return 0;}\n")
    exe = tmp_path / "sizes"
    subprocess.check_call(["gcc", "-I", os.path.join(REPO, "include"), str(prog), "-o", str(exe)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    A = rtw._abi
    mine = [A.SPHERE_DT.itemsize, A.MATERIAL_DT.itemsize, A.TEXTURE_DT.itemsize, C.sizeof(A.RtwImage),
            A.PERLIN_DT.itemsize, C.sizeof(A.RtwSceneDesc), C.sizeof(A.RtwCameraParams), C.sizeof(A.RtwCamera),
            C.sizeof(A.RtwRenderOpts), C.sizeof(A.RtwSceneStats), C.sizeof(A.RtwTuning)]
    assert sizes == mine


def test_tuning_defaults_and_no_environment_knobs(rtw):
    """The library is configured only through rtw_tuning (no getenv in the product .so);
    rtw_tuning_defaults() is the product configuration."""
    t = rtw._abi.tuning()
    A = rtw._abi
    assert (t.kernel, t.bvh_orders, t.sah_max_leaf, t.compact_nodes, t.fast_box, t.fast_reject) == (0, 0, 1, 1, 1, 1)
    assert t.lds == A.RTW_LDS_ALL and t.fuse == A.RTW_FUSE_STEP | A.RTW_FUSE_TAIL_LDS and t.wf_iters == 0
    assert t.wf_paths == 0 and (t.hoist, t.sort_iters, t.sort_bits, t.sort_iters_split) == (1, 3, 4, 1)
    assert t.object_tree == 90 and (t.clds_shape, t.deal) == (0, 59)
    syms = subprocess.check_output(["nm", "-D", "--undefined-only", rtw._abi.LIB_PATH], text=True)
    assert "getenv" not in syms, "the product library reads the environment"


@pytest.mark.parametrize("kw", [dict(image_width=1200, aspect_ratio=1.5, spp=500),
                                dict(image_width=400, aspect_ratio=16 / 9, spp=10),
                                dict(image_width=3840, aspect_ratio=16 / 9, spp=1024)])
def test_camera_init_matches_oracle(rtw, oracle, kw):
    cam = rtw.book1_camera(max_depth=50, **kw).init()
    o = oracle.camera(image_width=kw["image_width"], aspect_ratio=kw["aspect_ratio"],
                      samples_per_pixel=kw["spp"], max_depth=50, background_mode=1)
    assert bytes(cam.derived) == bytes(o)


def test_camera_defaults_are_reference(rtw):
    """camera.zig:70-91 defaults: 800 wide, 16:9 -> 450 high, spp 100, depth 16."""
    cam = rtw.Camera().init()
    assert (cam.derived.image_width, cam.derived.image_height) == (800, 450)
    assert cam.samples_per_pixel == 100 and cam.max_depth == 16 and cam.pixel_offset == 1


def test_texture_from_accum_matches_gamma2(rtw, oracle):
    rng = np.random.default_rng(0)
    acc = np.concatenate([rng.random((500, 3), np.float32) * 40, rng.integers(1, 50, (500, 1)).astype(np.float32)], 1)
    acc[:5, :3] = 0
    acc[5:10, :3] = 1e6
    out = np.zeros((500, 4), np.uint8)
    rtw.lib().rtw_texture_from_accum(acc.ctypes.data, 500, out.ctypes.data)
    assert np.array_equal(out, oracle.gamma2(acc))


@pytest.mark.parametrize("scene,seed", [("book1", 0), ("book1", 17), ("ref_head", 0)])
def test_bvh_flatten_matches_oracle_tree(rtw, oracle, earth_rgba, scene, seed):
    """Product BVH builder (C++, pre-order + skip links) == oracle pointer tree."""
    imgs = [rtw.Image(earth_rgba)]
    objs = rtw.worlds.generate_world(0, scene, imgs)
    arr = rtw.flatten(objs, bvh_seed=seed, bvh_mode=rtw._abi.RTW_BVH_REFERENCE)
    nodes = rtw.scene.flatten_bvh(arr)
    ow = oracle.World(arr.spheres, arr.materials, arr.textures, images=[earth_rgba], bvh_seed=seed)
    d = ow.dump()
    assert len(nodes) == len(d) == 2 * len(arr.spheres) - 1
    a, b = nodes["a"], nodes["b"]
    wbits = a[:, 3].view(np.uint32)
    is_leaf = (wbits & 0x80000000) != 0
    skip = wbits & 0x7FFFFFFF
    assert np.array_equal(is_leaf, d[:, 6] >= 0)
    assert np.array_equal(skip, np.arange(len(d)) + d[:, 7].astype(np.int64))
    inner = ~is_leaf
    assert np.array_equal(a[inner, :3], d[inner, 0:3]) and np.array_equal(b[inner, :3], d[inner, 3:6])
    sid = b[is_leaf, 2].view(np.uint32)
    assert np.array_equal(sid, d[is_leaf, 6].astype(np.uint32))
    assert np.array_equal(a[is_leaf, :3], arr.spheres["center1"][sid])
    assert np.array_equal(b[is_leaf, 0], arr.spheres["radius"][sid])
    assert np.array_equal(b[is_leaf, 1].view(np.uint32), arr.spheres["material"][sid])


@pytest.mark.parametrize("mode", [0, 1])
def test_stress_scene_builds(rtw, mode):
    objs = rtw.worlds.stress_world(2000, 0)
    arr = rtw.flatten(objs, bvh_mode=mode)
    nodes = rtw.scene.flatten_bvh(arr)
    assert len(nodes) == 2 * len(objs) - 1


def test_sah_tree_is_valid_bvh(rtw):
    """SAH mode: every sphere appears in exactly one leaf, skip links are proper
    pre-order subtree ends, and every inner box encloses its subtree."""
    arr = rtw.flatten(rtw.worlds.generate_world(0, "book1"), bvh_mode=rtw._abi.RTW_BVH_SAH)
    nodes = rtw.scene.flatten_bvh(arr)
    n = len(nodes)
    a, b = nodes["a"], nodes["b"]
    w = a[:, 3].view(np.uint32)
    leaf = (w & 0x80000000) != 0
    skip = (w & 0x7FFFFFFF).astype(np.int64)
    sid = b[leaf, 2].view(np.uint32)
    assert sorted(sid.tolist()) == list(range(len(arr.spheres)))
    assert (skip[leaf] == np.nonzero(leaf)[0] + 1).all()
    r = arr.spheres["radius"]
    c = arr.spheres["center1"]
    for i in np.nonzero(~leaf)[0]:
        assert i + 1 < skip[i] <= n
        sub = np.arange(i + 1, skip[i])
        ls = b[sub[leaf[sub]], 2].view(np.uint32)
        assert (c[ls] - r[ls, None] >= a[i, :3]).all() and (c[ls] + r[ls, None] <= b[i, :3]).all()


def test_shard_rows_partition(rtw):
    L = rtw.lib()
    for H in (1, 7, 800, 2160):
        for rpb in (1, 8, 16):
            for n in (1, 2, 3, 8):
                assert sum(L.rtw_shard_rows(H, rpb, n, s) for s in range(n)) == H


def test_invalid_scene_rejected(rtw):
    objs = rtw.worlds.two_spheres_world()
    arr = rtw.flatten(objs)
    arr.materials["texture"][0] = 99
    d = arr.desc()
    h = C.c_void_p()
    rc = rtw.lib().rtw_scene_create(C.byref(d), 0, C.byref(h))
    assert rc in (rtw._abi.RTW_E_INVALID,)
    assert b"texture" in rtw.lib().rtw_last_error()


def source_build_id():
    """csrc/Makefile's SRC_HASH: sha256 of SRCS, HDRS and the Makefile, in that order."""
    import hashlib
    csrc = os.path.join(REPO, "zig-raytracing-weekend_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    srcs = re.search(r"^SRCS = (.*)$", mk, re.M).group(1).split()
    hdrs = re.search(r"^HDRS = (.*)$", mk, re.M).group(1).split()
    h = hashlib.sha256()
    for f in srcs + hdrs + ["Makefile"]:
        h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()[:16]


def test_build_id_is_the_sources(rtw):
    """The loaded library was built from the sources in the tree (rtw_build_id = the Makefile's
    sha256 of them), so a PMC pass stamped with this id was taken on this code."""
    assert rtw.lib().rtw_build_id().decode() == source_build_id()


def test_box_pad_extent_covers_hoisted_spheres(rtw):
    """The FMA slab test's pad E * 2^-19 covers origins |o| <= 7E (rtw_bvh.hip); E spans every
    object's box, including hoisted spheres outside the tree (Book-1's r = 1000 ground), whose
    horizon hits are secondary-ray origins hundreds of units out."""
    objs = rtw.worlds.generate_world(0, "ref_head")
    arr = rtw.flatten(objs)
    for hoist in (1, 0):
        w = rtw.World(arr, device=rtw._abi.RTW_DEVICE_CPU, tuning={"hoist": hoist})
        st = w.stats()
        w.close()
        assert st["n_hoisted"] == hoist
        assert st["extent"] >= 2000.0, st        # the ground's box: (-1000, -2000, -1000) .. (1000, 0, 1000)
        assert st["box_pad"] == np.float32(st["extent"]) * np.float32(2.0 ** -19)


def test_deal_bits_header_and_validation(rtw):
    """rtw_tuning.deal (ABI 8): the header's RTW_DEAL_* values are the binding's, the live bits are accepted and
    the removed modes (4: per-stripe tail claims, 64: the two-launch tail; diag/deal_tail_modes.patch) refused."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    hdr = {k: int(v) for k, v in re.findall(r"(RTW_DEAL_[A-Z_0-9]+)\s*=\s*(\d+)u", src)}
    A = rtw._abi
    assert hdr and all(getattr(A, k) == v for k, v in hdr.items()), hdr
    live = [v for k, v in hdr.items() if k != "RTW_DEAL_ALL"]
    assert sum(live) == hdr["RTW_DEAL_ALL"] == A.RTW_DEAL_ALL
    arr = rtw.flatten(rtw.worlds.two_spheres_world())
    for deal in (0, 59, A.RTW_DEAL_ALL, A.RTW_DEAL_SMALL_SORT):
        rtw.World(arr, device=A.RTW_DEVICE_CPU, tuning={"deal": deal}).close()
    for deal in (4, 64, 63, 123, 256):
        with pytest.raises(rtw.RtwError) as e:
            rtw.World(arr, device=A.RTW_DEVICE_CPU, tuning={"deal": deal})
        assert e.value.code == A.RTW_E_INVALID
    # (ABI 8: clds_shape 2 / 3, the 512- / 640-thread two-block shapes, were removed with the losing modes)
    for shape in (0, 1, 4):
        rtw.World(arr, device=A.RTW_DEVICE_CPU, tuning={"clds_shape": shape}).close()
    for shape in (2, 3, 5):
        with pytest.raises(rtw.RtwError):
            rtw.World(arr, device=A.RTW_DEVICE_CPU, tuning={"clds_shape": shape})


def test_resource_report_is_this_build(rtw):
    """profiles/isa_resources.json (make -C zig-raytracing-weekend_amd/csrc resources): VGPR / SGPR / scratch /
    occupancy of every wavefront kernel, read from the gfx950 assembly of these sources -- stamped with the build id
    of the in-tree library, so a source change without a regenerated table fails here."""
    import json
    path = os.path.join(REPO, "profiles", "isa_resources.json")
    rep = json.load(open(path))
    assert rep["build_id"] == rtw.lib().rtw_build_id().decode(), "stale: run make -C zig-raytracing-weekend_amd/csrc resources"
    k = rep["kernels"]
    # the product launches of C2 / C4 / Cornell / C5: counters compiled out (CNT 0), fused steps split into
    # iteration 0 (IT0 1) and the later iterations (IT0 0)
    for name in ("wf_step_clds2<0u, 768u, 0, 1>", "wf_step_clds2<0u, 768u, 0, 0>", "wf_tail_clds2<0u, 768u, 0>",
                 "wf_tail_w5<0u, 0>", "wf_trace<0u, false, false>", "wf_shade<0u, false>", "wf_step<49u, true, 0, 0>",
                 "wf_tail_lds<49u, 0>", "wf_step<7u, true, 0, 0>", "wf_reduce"):
        assert name in k, name
        assert k[name]["vgpr"] and k[name]["occupancy"], (name, k[name])
    # the 6-wave shapes fit 80 VGPRs (MI355X_MICROARCH.md: 80 allocated -> 6 waves / SIMD); round 6 took the fused
    # step's spills from 156 to 44 / 28 B/lane (iteration 0 / the rest) and the compact-LDS tail's to none
    # (profiles/r6_late_rest/, profiles/r6_waves/)
    for it in (0, 1):
        step = k[f"wf_step_clds2<0u, 768u, 0, {it}>"]
        assert step["vgpr"] <= 80 and step["occupancy"] == 6 and step["scratch"] <= 44, step
    tail = k["wf_tail_clds2<0u, 768u, 0>"]
    assert tail["vgpr"] <= 80 and tail["scratch"] == 0, tail
