"""The oracle (CPU restatement, oracle/) against the reference's own recorded outputs and
analytic known answers. CPU only."""
import json
import math
import os

import numpy as np
import pytest

import oracle_lib as O
from pysicalbasedraytracer_amd import capi, scenes

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def test_linear_bvh_node_is_32_bytes():
    assert O.load().oracle_sizeof_linear_bvh_node() == KATS["sizeof"]["LinearBVHNode"]


@pytest.mark.parametrize("pixel", ["0,0", "1,0", "1919,1079"])
def test_halton_kats_bit_exact(pixel):
    k = KATS["halton_1920x1080"]
    x, y = map(int, pixel.split(","))
    v = O.halton(1920, 1080, 64, [(x, y, 0, d) for d in k["get2d_x3_dims"]])
    assert ["%08x" % u for u in v.view(np.uint32)] == k["pixels"][pixel]


def test_halton_second_sample():
    v = O.halton(1920, 1080, 64, [(0, 0, 1, 0), (0, 0, 1, 1)])
    assert np.allclose(v, KATS["halton_1920x1080"]["pixel_0_0_sample_1_dims_0_1"], rtol=0, atol=6e-8)  # printed to 7 significant digits


def test_halton_permutations_are_permutations():
    perms = O.halton_perms(64)
    pos = 0
    p = 2
    primes = []
    while len(primes) < 64:
        if all(p % q for q in primes):
            primes.append(p)
        p += 1
    for b in primes:
        assert sorted(perms[pos:pos + b].tolist()) == list(range(b))
        pos += b


def li_capture_scene():
    k = KATS["li_capture"]
    s = scenes.Scene()
    m = s.matte((0.5, 0.5, 0.5))
    s.mesh(np.array(k["triangle"], np.float32), np.array([[0, 1, 2]], np.int32), m)
    s.point_light(tuple(k["point_light"]["pos"]), (k["point_light"]["I"],) * 3)
    cam = scenes.camera(k["width"], k["height"], tuple(k["camera"]["eye"]), tuple(k["camera"]["look"]))
    return s, scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, k["spp"], k["max_depth"])


def test_li_capture_bit_exact():
    """The reference's float Li capture, reproduced bit for bit."""
    k = KATS["li_capture"]
    s, rd = li_capture_scene()
    rgb, rgba, _ = O.render(s, rd)
    px = rgb.reshape(k["height"], k["width"], 3)[k["pixel"][1], k["pixel"][0]]
    assert np.float32(px[0]).view(np.uint32) == np.float32(k["value"]).view(np.uint32)
    assert px[0] == px[1] == px[2]
    # analytic centre value 0.5/π · 9/3²
    assert abs(px[0] - k["analytic_centre"]) < 1e-3


def test_point_light_background_is_grey_08():
    """F4: Whitted sums Light::Le = 0.8 over all lights on a miss → 8-bit 231."""
    s, rd = scenes.config_c1(32, 32, 1)
    rgb, rgba, _ = O.render(s, rd)
    assert np.allclose(rgb[0], 0.8)
    assert tuple(rgba[0]) == (231, 231, 231, 255)


def test_sphere_lambert_analytic():
    """F2 unpinned by the reference: a Lambertian sphere under a point light gives the analytic
    value at the point nearest the light (Kd/π · I/d²)."""
    s = scenes.Scene()
    m = s.matte((0.5, 0.5, 0.5))
    s.sphere((0.0, 0.0, 0.0), 1.0, m)
    s.point_light((0.0, 0.0, 4.0), (9.0, 9.0, 9.0))
    cam = scenes.camera(33, 33, (0.0, 0.0, 4.0), (0.0, 0.0, 0.0))
    rgb, _, _ = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 16, 5))
    c = rgb.reshape(33, 33, 3)[16, 16, 0]
    assert abs(c - 0.5 / math.pi * 9.0 / 9.0) < 2e-3


def test_render_tiles_equal_full_frame():
    """Per-pixel sample indices do not depend on tile ownership (Halton.cpp:61-81)."""
    s, rd = scenes.config_c1(48, 40, 2)
    full, full8, _ = O.render(s, rd)
    from pysicalbasedraytracer_amd import tile_grid, assemble
    tiles = tile_grid(48, 40, 16)
    rd2 = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, tiles=tiles)
    part, part8, _ = O.render(s, rd2)
    frame = assemble(48, 40, tiles, part, 3)
    assert np.array_equal(frame.reshape(-1, 3), full)


def test_bvh_structure_invariants():
    P, I = scenes.dragon_standin(n=24)
    s = scenes.Scene()
    m = s.matte((0.5, 0.5, 0.5))
    s.mesh(P, I, m)
    nodes, ids = O.build_bvh(s)
    assert sorted(ids.tolist()) == list(range(I.shape[0]))
    rec = nodes.view(np.uint8).reshape(-1, 32)
    nprims = rec[:, 28:30].copy().view(np.uint16).ravel()
    assert int(nprims.sum()) == I.shape[0]
    leaves = int((nprims > 0).sum())
    assert rec.shape[0] == 2 * leaves - 1            # full binary tree
    # maxPrimsInNode = 1: only coincident-centroid sets (the degenerate pole triangles) share a leaf
    assert leaves >= I.shape[0] - 2 * 24


def test_watertight_triangle_edge_tie_later_wins():
    """F8: t == tMax accepted → on a shared edge the later-tested primitive wins; our
    intersect reports it."""
    tri = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0], np.float32)
    hit = O.triangle_test(tri, np.array([0.25, 0.25, 1, 0, 0, -1, np.inf], np.float32))
    assert hit[0] == 1 and hit[1] == np.float32(1.0)
    miss = O.triangle_test(tri, np.array([0.75, 0.75, 1, 0, 0, -1, np.inf], np.float32))
    assert miss[0] == 0
    # tMax equal to the hit distance is still a hit
    tie = O.triangle_test(tri, np.array([0.25, 0.25, 1, 0, 0, -1, 1.0], np.float32))
    assert tie[0] == 1


SOBOL = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "sobol_kats.json")))


def test_sobol_index_and_pixel_dims_bit_exact():
    """pbrt-v3 SobolIntervalToIndex + SampleDimension as evaluated with the reference's own
    VdCSobolMatrices / SobolMatrices32 (tests/golden/make_sobol_kats.py), reproduced by the
    oracle's GF(2) solve at five rasters including 1×1 (index 0) and 3840×2160, with sample
    numbers whose 64-bit index needs bits >= 32: the index and dimensions 0-127, bit for bit."""
    wide = 0
    for c in SOBOL["cases"]:
        (w, h), (px, py), s = c["raster"], c["pixel"], c["sample"]
        q = [(px, py, s, d) for d in range(SOBOL["high_dims"])]
        v, idx = O.sobol(w, h, q)
        assert int(idx[0]) == c["index"], c
        bits = ["%08x" % u for u in v.view(np.uint32)]
        assert bits[:2] == [c["dim0"], c["dim1"]], c
        assert "".join(bits[2:]) == c["dims2_127"], c
        wide += c["index"] >= 2 ** 32
    assert wide >= 60   # the fixture exercises 64-bit indices


def test_sobol_builtin_is_the_reference_table():
    """The built-in matrices — regenerated from the Joe-Kuo direction numbers of pbr_sobol_jk.h —
    hash to the reference's whole SobolMatrices32 table (1024 dims × 52 columns) and to its
    dimension-0/1 rows; the device library's host builder produces the oracle's table."""
    import ctypes as C
    import hashlib
    m = O.sobol_matrices(1024)
    assert hashlib.sha256(m[:104].astype("<u4").tobytes()).hexdigest() == SOBOL["dims01_sha256"]
    assert hashlib.sha256(m.astype("<u4").tobytes()).hexdigest() == SOBOL["all_sha256"]
    d = np.empty(1024 * 52, np.uint32)
    assert capi.load_library().pbr_hip_sobol_matrices(1024, d.ctypes.data_as(C.POINTER(C.c_uint32))) == 0
    assert np.array_equal(d, m)


def test_sobol_samples_land_in_their_pixel():
    """Every sample's dims 0/1 offsets lie in [0, 1): the interval→index mapping is a bijection per pixel."""
    rng = np.random.default_rng(3)
    q = [(int(rng.integers(300)), int(rng.integers(200)), s, d) for _ in range(40) for s in range(16) for d in (0, 1)]
    v, idx = O.sobol(300, 200, q)
    assert np.all((v >= 0) & (v < 1))
    # distinct samples of one pixel have distinct indices with the sample number in the high bits
    assert np.all(idx.reshape(-1, 16, 2)[:, :, 0] >> 18 == np.arange(16))


def test_oracle_adopts_a_caller_built_tree():
    """pbr_scene_desc::bvh_nodes on the oracle: the reference's BVHAccel node array with the primitives
    in its leaf order renders the same bits as the oracle's own build over the original order (the
    parity harness renders the reference-side binding's flattened scenes this way)."""
    m = scenes.dragon_standin(n=24)
    s = scenes.Scene()
    s.mesh(m[0], m[1], s.matte((0.3, 0.7, 0.2)))
    s.point_light((1.0, 2.0, 2.0), (6.0, 6.0, 6.0))
    cam = scenes.camera(48, 32, (0.0, 0.4, 2.6), (0.0, 0.0, 0.0))
    rd = scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 4, 5)
    cn, ci = O.build_bvh(s)
    want, want8, _ = O.render(s, rd)
    leaf = scenes.Scene()
    leaf.mesh(m[0], np.ascontiguousarray(m[1][ci]), leaf.matte((0.3, 0.7, 0.2)))
    leaf.point_light((1.0, 2.0, 2.0), (6.0, 6.0, 6.0))
    leaf.bvh_nodes = cn
    got, got8, _ = O.render(leaf, rd)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)) and np.array_equal(got8, want8)
