"""The device SAH build (pbr_bvh_build.hip) against the host builder, which the reference pins
(tests/test_ref_fixtures.py: node-array and orderedPrims hashes of the reference's own BVHAccel).

Bit for bit: the LinearBVHNode array (BVHAccel.cpp:262-283) and orderedPrims (:107-112) — over random
boxes, tie-heavy grids with +-0 coordinates (the first element of a tie wins Union's std::min/max),
coincident centroids (the degenerate leaf, :121-130), two-element nodes (nth_element), leaf sizes
1/4/255, the 100k-triangle C2 stand-in and an 871k-triangle (real-dragon-sized) one.
"""
import numpy as np
import pytest

from pysicalbasedraytracer_amd import HipRenderer, capi, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    r = HipRenderer(0)
    yield r
    r.close()


def both(hip, b, max_prims=1):
    dn, di, dt = hip.build_bvh(b, capi.BVH_BUILD_DEVICE, max_prims)
    hn, hi, ht = hip.build_bvh(b, capi.BVH_BUILD_HOST, max_prims)
    assert np.array_equal(di, hi), "orderedPrims differ"
    assert np.array_equal(dn, hn), "LinearBVHNode arrays differ"
    return dn, di, dt, ht


def boxes_from_points(lo, ext):
    return np.concatenate([lo, lo + ext], axis=1).astype(np.float32)


def mesh_bounds(P, I):
    v = P[I]                       # [n, 3, 3]
    lo = np.minimum(np.minimum(v[:, 0], v[:, 1]), v[:, 2])
    hi = np.maximum(np.maximum(v[:, 0], v[:, 1]), v[:, 2])
    return np.concatenate([lo, hi], axis=1).astype(np.float32)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 17, 64, 65, 1000, 20000])
def test_random_boxes(hip, n):
    rng = np.random.default_rng(n)
    b = boxes_from_points(rng.normal(size=(n, 3)), rng.random((n, 3)) * 0.1)
    dn, di, _, _ = both(hip, b)
    assert dn.size == max(0, 2 * n - 1) * 32
    assert sorted(di.tolist()) == list(range(n))


@pytest.mark.parametrize("max_prims", [1, 4, 255])
def test_leaf_sizes(hip, max_prims):
    rng = np.random.default_rng(7)
    b = boxes_from_points(rng.random((5000, 3)) * 10, rng.random((5000, 3)))
    both(hip, b, max_prims)


def test_ties_and_signed_zeros(hip):
    rng = np.random.default_rng(11)
    n = 6000
    lo = rng.integers(-2, 3, size=(n, 3)).astype(np.float32) * 0.5
    ext = rng.integers(0, 3, size=(n, 3)).astype(np.float32) * 0.5
    hi = lo + ext
    # signed zeros: -0.0 and +0.0 compare equal, so which one a union keeps depends on the order
    z = rng.random((n, 3)) < 0.5
    lo[(lo == 0) & z] = -0.0
    hi[(hi == 0) & ~z] = -0.0
    b = np.concatenate([lo, hi], axis=1).astype(np.float32)
    dn, _, _, _ = both(hip, b)
    for mp in (2, 8):
        both(hip, b, mp)


def test_coincident_centroids(hip):
    # all centroids equal → one leaf holding everything (BVHAccel.cpp:121-130)
    b = np.tile(np.array([[-1, -1, -1, 1, 1, 1]], np.float32), (200, 1))
    b[::3, :3] -= 0.25
    b[::3, 3:] += 0.25
    dn, di, _, _ = both(hip, b)
    nodes = dn.view(np.int32).reshape(-1, 8)
    assert nodes.shape[0] == 1 and (nodes[0, 7] & 0xffff) == 200
    # a cluster of coincident centroids inside a larger set
    rng = np.random.default_rng(3)
    c = boxes_from_points(rng.random((300, 3)), rng.random((300, 3)) * 0.01)
    c[100:180] = c[100]
    both(hip, c)


@pytest.mark.parametrize("n", [224, 660])
def test_dragon_standins(hip, n):
    P, I = scenes.dragon_standin(n=n)
    b = mesh_bounds(P, I)
    _, _, dt, ht = both(hip, b)
    print(f"\n{I.shape[0]} triangles: host build {ht['ms']:.1f} ms, device build {dt['ms']:.1f} ms "
          f"({dt['kernel_ms']:.1f} ms of kernels)")


def test_upload_with_either_builder(hip):
    s, _ = scenes.config_c2(64, 36, 1, sky=np.ones((8, 16, 3), np.float32))
    got = {}
    for where in (capi.BVH_BUILD_HOST, capi.BVH_BUILD_DEVICE):
        hip.set_bvh_build(where)
        hip.upload(s)
        info = hip.bvh_build_info()
        assert info["where"] == ("device" if where == capi.BVH_BUILD_DEVICE else "host")
        assert info["ms"] > 0 and (info["kernel_ms"] > 0) == (where == capi.BVH_BUILD_DEVICE)
        got[where] = hip.get_bvh()
    hip.set_bvh_build(capi.BVH_BUILD_DEVICE)
    assert np.array_equal(got[0][0], got[1][0]) and np.array_equal(got[0][1], got[1][1])


def test_signed_zero_bounds_match_the_oracle(hip):
    """World vertices with -0 and +0 coordinates (-0 survives a transform only when every term is -0,
    hence the -0 translation): interior boxes are InitInterior's Union(c0, c1), whose first operand
    wins a -0/+0 tie (BVHAccel.cpp:33-38) — device and host builders against the oracle, bit for bit."""
    import oracle_lib as O
    rng = np.random.default_rng(5)
    n = 400
    P = rng.choice(np.array([-1.0, -0.5, 0.0, -0.0, 0.5], np.float32), size=(3 * n, 3)).astype(np.float32)
    P[:, 1:] = -np.abs(P[:, 1:]) - 0.25      # y, z < 0: 0*y and 0*z are -0
    I = np.arange(3 * n, dtype=np.int32).reshape(n, 3)
    s = scenes.Scene()
    s.mesh(P, I, s.matte((0.5, 0.5, 0.5)), xform=scenes.translate(-0.0, -0.0, -0.0))
    s.point_light((0, 2, 0), (1, 1, 1))
    cn, ci = O.build_bvh(s)
    box = cn.view(np.float32).reshape(-1, 8)[:, :6]
    assert ((box == 0) & np.signbit(box)).any() and ((box == 0) & ~np.signbit(box)).any()
    for where in (capi.BVH_BUILD_HOST, capi.BVH_BUILD_DEVICE):
        hip.set_bvh_build(where)
        hip.upload(s)
        gn, gi = hip.get_bvh()
        assert np.array_equal(gi, ci) and np.array_equal(gn, cn), where
    hip.set_bvh_build(capi.BVH_BUILD_DEVICE)


def test_upload_adopts_a_caller_built_tree(hip):
    """pbr_scene_desc::bvh_nodes (the reference-side binding hands over its BVHAccel this way): the
    primitives in leaf order plus the reference's LinearBVHNode array are used as given — the device's
    node array is that array, the frame equals the one of the device-built tree over the original
    order bit for bit — and a tree whose leaf box is not its primitives' bounds is refused."""
    import oracle_lib as O
    s, rd = scenes.config_c1(48, 32, 4)
    m = scenes.dragon_standin(n=24)
    s = scenes.Scene()
    s.mesh(m[0], m[1], s.matte((0.3, 0.7, 0.2)))
    s.point_light((1.0, 2.0, 2.0), (6.0, 6.0, 6.0))
    cam = scenes.camera(48, 32, (0.0, 0.4, 2.6), (0.0, 0.0, 0.0))
    rd = scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 4, 5)
    cn, ci = O.build_bvh(s)
    hip.upload(s)
    want, want8, _ = hip.render(rd)
    leaf = scenes.Scene()
    leaf.mesh(m[0], np.ascontiguousarray(m[1][ci]), leaf.matte((0.3, 0.7, 0.2)))
    leaf.point_light((1.0, 2.0, 2.0), (6.0, 6.0, 6.0))
    leaf.bvh_nodes = cn
    hip.upload(leaf)
    gn, gi = hip.get_bvh()
    assert np.array_equal(gn, cn) and np.array_equal(gi, np.arange(len(ci)))
    got, got8, _ = hip.render(rd)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)) and np.array_equal(got8, want8)
    bad = cn.copy().view(np.float32).reshape(-1, 8)
    rec = np.frombuffer(cn.tobytes(), dtype=[("b", "<f4", 6), ("off", "<i4"), ("np", "<u2"), ("ax", "u1"), ("pad", "u1")])
    k = int(np.nonzero(rec["np"] > 0)[0][0])
    bad[k, 0] -= 1.0                               # a leaf box no longer its triangle's bounds
    leaf.bvh_nodes = bad.view(np.uint8).reshape(-1)
    with pytest.raises(RuntimeError, match="leaf box"):
        hip.upload(leaf)
    hip.upload(s)   # the context stays usable
