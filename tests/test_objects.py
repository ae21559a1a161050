"""SURVEY §8f rows 1-2 on the CPU: Quad / HittableList / Translate / RotateY /
createBox / ConstantMedium (src/objects.zig:193-532), the scene builders that use
them (src/main.zig:127-251), the C-ABI flattening and the BVH over generic world
objects.  No GPU: oracle known answers, flattening, and the product's host BVH
builder (rtw_scene_flatten) against the oracle's pointer tree.

Parity status: no reference test or image covers quads, instances or media;
the oracle restates objects.zig line by line and the known answers below are
derived by hand from the formulas ("parity unpinned" beyond the restatement).
"""
import numpy as np
import pytest


def quad_rec(oracle, q, u, v):
    r = np.zeros(1, oracle.QUAD_DT)
    r["q"], r["u"], r["v"] = q, u, v
    return r


def quad_hit(oracle, rec, o, d, tmin=0.001, tmax=np.inf):
    out = np.zeros(10, np.float32)
    o, d = np.asarray(o, np.float32), np.asarray(d, np.float32)   # keep alive across the call
    h = oracle.lib().oracle_quad_hit(rec.ctypes.data, o.ctypes.data, d.ctypes.data, tmin, tmax, out.ctypes.data)
    return h, out


def test_quad_known_answers(oracle):
    """Quad.hit (objects.zig:222-255): plane t, planar (alpha, beta) as (u, v), face normal."""
    rec = quad_rec(oracle, [0, 0, 0], [1, 0, 0], [0, 1, 0])        # unit square in z=0, normal +z
    h, out = quad_hit(oracle, rec, [0.25, 0.5, 1], [0, 0, -1])
    assert h == 1
    assert out[0] == 1.0 and list(out[1:4]) == [0.25, 0.5, 0.0]
    assert list(out[4:7]) == [0.0, 0.0, 1.0] and out[7] == 1.0      # front face: d . n < 0
    assert out[8] == 0.25 and out[9] == 0.5                          # u = alpha, v = beta
    h, out = quad_hit(oracle, rec, [0.25, 0.5, -1], [0, 0, 1])      # from behind: back face
    assert h == 1 and out[7] == 0.0 and list(out[4:7]) == [0.0, 0.0, -1.0]
    assert quad_hit(oracle, rec, [1.5, 0.5, 1], [0, 0, -1])[0] == 0  # alpha > 1: outside
    assert quad_hit(oracle, rec, [0.5, -0.1, 1], [0, 0, -1])[0] == 0  # beta < 0
    assert quad_hit(oracle, rec, [0.5, 0.5, 1], [1, 0, 0])[0] == 0   # parallel: |denom| < 1e-8
    assert quad_hit(oracle, rec, [0.5, 0.5, 1], [0, 0, -1], tmax=0.5)[0] == 0
    # Interval.contains is inclusive (interval.zig:8-10), unlike the sphere's surrounds
    assert quad_hit(oracle, rec, [0.5, 0.5, 1], [0, 0, -1], tmax=1.0)[0] == 1
    assert quad_hit(oracle, rec, [1.0, 1.0, 1], [0, 0, -1])[0] == 1  # corner: alpha = beta = 1 inside


def test_medium_draw_is_keyed(oracle):
    """The ConstantMedium draw depends only on (path RNG state, medium index)."""
    d = oracle.lib().oracle_medium_draw
    a, b, c = d(12345, 0), d(12345, 1), d(99, 0)
    assert 0.0 <= a < 1.0 and a == d(12345, 0) and len({a, b, c}) == 3


def test_create_box_and_cornell_flatten(rtw):
    """createBox = 6 quads (objects.zig:510-532, negated edges keep -0.0); Translate(RotateY(box))
    becomes one instance with xf = [ROTATE_Y, TRANSLATE]."""
    white = rtw.Lambertian.fromColor([0.73, 0.73, 0.73])
    box = rtw.createBox([0, 0, 0], [165, 330, 165], white)
    assert len(box.objects) == 6
    assert np.signbit(box.objects[1].u[0]) and box.objects[1].u[2] == -165   # -dz = (-0, -0, -165)
    arr = rtw.flatten(rtw.worlds.cornell_box())
    A = rtw._abi
    assert len(arr.objects) == 8 and len(arr.quads) == 6 + 12 and len(arr.instances) == 2
    assert list(arr.objects["kind"]) == [A.RTW_OBJ_QUAD] * 6 + [A.RTW_OBJ_INSTANCE] * 2
    inst = arr.instances[0]
    assert inst["count"] == 6 and inst["n_xf"] == 2 and inst["flags"] == A.RTW_INST_LIST
    assert inst["xf"][0]["kind"] == A.RTW_XF_ROTATE_Y and inst["xf"][0]["v"][0] == 15
    assert inst["xf"][1]["kind"] == A.RTW_XF_TRANSLATE and list(inst["xf"][1]["v"]) == [265, 0, 295]
    assert (arr.members["kind"] == A.RTW_OBJ_QUAD).all() and len(arr.members) == 12
    smoke = rtw.flatten(rtw.worlds.cornell_smoke())
    assert len(smoke.media) == 2 and list(smoke.objects["kind"][-2:]) == [A.RTW_OBJ_MEDIUM] * 2
    assert smoke.media[0]["boundary"]["kind"] == A.RTW_OBJ_INSTANCE
    assert smoke.materials[smoke.media[1]["material"]]["kind"] == A.RTW_MAT_ISOTROPIC
    # sphere-only worlds keep the ABI-1 description (objects = NULL)
    assert rtw.flatten(rtw.worlds.generate_world(0, "book1")).objects is None


def scenes(rtw):
    return {"quads": rtw.worlds.quads_world(), "simple_light": rtw.worlds.simple_light_world(0),
            "cornell": rtw.worlds.cornell_box(), "cornell_smoke": rtw.worlds.cornell_smoke()}


@pytest.mark.parametrize("scene", ["quads", "simple_light", "cornell", "cornell_smoke"])
@pytest.mark.parametrize("seed", [0, 5])
def test_object_bvh_matches_oracle_tree(rtw, oracle, scene, seed):
    """Reference-topology BVH over generic world objects: the product's C++ builder
    (object boxes restated from Quad.init / HittableList / RotateY / Translate /
    ConstantMedium) == the oracle's pointer tree, node for node."""
    arr = rtw.flatten(scenes(rtw)[scene], bvh_seed=seed, bvh_mode=rtw._abi.RTW_BVH_REFERENCE)
    nodes = rtw.scene.flatten_bvh(arr)
    ow = oracle.World.from_arrays(arr)
    d = ow.dump()
    n_obj = len(arr.objects) if arr.objects is not None else len(arr.spheres)
    assert len(nodes) == len(d) == 2 * n_obj - 1
    a, b = nodes["a"], nodes["b"]
    wbits = a[:, 3].view(np.uint32)
    is_leaf = (wbits & 0x80000000) != 0
    assert np.array_equal(is_leaf, d[:, 6] >= 0)
    assert np.array_equal(wbits & 0x7FFFFFFF, np.arange(len(d)) + d[:, 7].astype(np.int64))
    inner = ~is_leaf
    assert np.array_equal(a[inner, :3], d[inner, 0:3]) and np.array_equal(b[inner, :3], d[inner, 3:6])
    # leaf -> (kind, index) of the world object the oracle leaf holds
    pos = d[is_leaf, 6].astype(np.int64)
    kinds = (b[is_leaf, 3].view(np.uint32) >> 8) & 0xFF
    idx = b[is_leaf, 2].view(np.uint32)
    if arr.objects is not None:
        assert np.array_equal(kinds, arr.objects["kind"][pos]) and np.array_equal(idx, arr.objects["index"][pos])
    else:
        assert (kinds == 0).all() and np.array_equal(idx, pos)


def test_object_sah_tree_is_valid(rtw):
    """SAH over generic objects: every world object in exactly one leaf; inner boxes
    enclose their subtree's inner boxes (the leaves carry no box)."""
    arr = rtw.flatten(rtw.worlds.cornell_smoke(), bvh_mode=rtw._abi.RTW_BVH_SAH)
    nodes = rtw.scene.flatten_bvh(arr)
    a, b = nodes["a"], nodes["b"]
    wbits = a[:, 3].view(np.uint32)
    is_leaf = (wbits & 0x80000000) != 0
    got = sorted(zip(((b[is_leaf, 3].view(np.uint32) >> 8) & 0xFF).tolist(), b[is_leaf, 2].view(np.uint32).tolist()))
    assert got == sorted(zip(arr.objects["kind"].tolist(), arr.objects["index"].tolist()))
    skip = wbits & 0x7FFFFFFF
    for i in np.nonzero(~is_leaf)[0]:
        for j in range(i + 1, skip[i]):
            if not is_leaf[j]:
                assert (a[j, :3] >= a[i, :3]).all() and (b[j, :3] <= b[i, :3]).all()


def test_invalid_object_graphs_rejected(rtw):
    arr = rtw.flatten(rtw.worlds.cornell_box())
    bad = rtw.flatten(rtw.worlds.cornell_box())
    bad.objects = bad.objects.copy()
    bad.objects[0]["index"] = 999                   # quad index out of range
    with pytest.raises(rtw.RtwError):
        rtw.scene.flatten_bvh(bad)
    bad = rtw.flatten(rtw.worlds.cornell_box())
    bad.instances = bad.instances.copy()
    bad.instances[0]["n_xf"] = 4                    # > RTW_MAX_XF
    with pytest.raises(rtw.RtwError):
        rtw.scene.flatten_bvh(bad)
    assert len(rtw.scene.flatten_bvh(arr)) == 15


@pytest.mark.parametrize("scene", ["quads", "cornell", "cornell_smoke"])
def test_oracle_object_scene_renders(oracle, rtw, scene):
    """The oracle renders the object scenes (finite radiance; light or colour visible)."""
    arr = rtw.flatten(scenes(rtw)[scene])
    ow = oracle.World.from_arrays(arr)
    if scene == "quads":
        ocam = oracle.camera(aspect_ratio=1.0, image_width=32, samples_per_pixel=4, max_depth=50,
                             background=(0.7, 0.8, 1.0), vfov=80.0, lookfrom=(0, 0, 9), lookat=(0, 0, 0),
                             defocus_angle=0.0)
    else:
        ocam = oracle.camera(aspect_ratio=1.0, image_width=32, samples_per_pixel=4, max_depth=50, vfov=40.0,
                             lookfrom=(278, 278, -800), lookat=(278, 278, 0), defocus_angle=0.0)
    out = ow.render_pixels(ocam, 0, np.arange(32 * 32, dtype=np.uint32), 0, 4, threads=4)
    assert np.isfinite(out).all() and out[:, :3].max() > 0


def test_object_tree_flattening_node_counts(rtw):
    """rtw_tuning.object_tree: Cornell's walls make four inner nodes under the root the whole room
    again; the default (90 %) leaves them out.  A scene with a quad that reaches outside its reference
    box (not axis-aligned) keeps the plain tree."""
    import ctypes as C
    import numpy as np

    def n_nodes(objs, tu):
        world = rtw.World(rtw.flatten(objs), device=-1, tuning=tu)
        buf = np.zeros((256, 8), np.float32)
        n = C.c_uint32()
        rtw._abi.check(rtw.lib().rtw_scene_nodes(world.handle, buf.ctypes.data, 256, C.byref(n)), "rtw_scene_nodes")
        world.close()
        return n.value

    assert n_nodes(rtw.worlds.cornell_box(), {"object_tree": 0}) == 15
    assert n_nodes(rtw.worlds.cornell_box(), None) == 11
    S = rtw.scene
    objs = rtw.worlds.cornell_box()
    mat = S.Lambertian.init(S.SolidColor.init([0.2, 0.4, 0.8]))
    roof = S.HittableList.init()
    roof.add(S.Quad.init([0, 0, 0], [100, 100, 0], [-50, 0, 120], mat))
    objs.append(S.Translate.init(S.RotateY.init(roof, 25), [150, 300, 250]))
    assert n_nodes(objs, None) == n_nodes(objs, {"object_tree": 0})
