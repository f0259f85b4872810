"""Edge cases of the device path against the oracle (SURVEY §8(c) fixture list, items 3 and 7-8):
exact edge/vertex hits that take the watertight test's double-precision fallback
(Triangle.cpp:102-113) and its t == tMax ties (F8), empty and light-less scenes, degenerate frame
and tile shapes, non-power-of-two spp, and the full-size C3/C5 frames checked through
size-independent properties plus spot pixels."""
import numpy as np
import pytest

import oracle_lib as O
from parity import assert_parity
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    r = HipRenderer(0)
    yield r
    r.close()


def grid_mesh(n=6, z=0.0):
    """n×n unit squares in the z plane, two triangles each, vertices on integer coordinates."""
    xs = np.arange(n + 1, dtype=np.float32)
    P = np.array([(x, y, z) for y in xs for x in xs], np.float32)
    I = []
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i, (j + 1) * (n + 1) + i + 1
            I += [(a, b, d), (a, d, c)]
    return P, np.array(I, np.int32)


def test_edge_and_vertex_hits_bit_exact(hip):
    """Axis-aligned rays through shared edges, diagonals and vertices make an edge function exactly
    zero (the double fallback) and hit two triangles at the same t (later primitive wins)."""
    s = scenes.Scene()
    m = s.matte((0.5, 0.5, 0.5))
    P, I = grid_mesh(6)
    s.mesh(P, I, m)
    s.mesh(P + np.float32([0.0, 0.0, -1.0]), I, m)   # a second sheet: ties across meshes behind
    hip.upload(s)
    pts = np.array([(x, y) for x in np.arange(0, 6.01, 0.5) for y in np.arange(0, 6.01, 0.5)], np.float32)
    rays = []
    for x, y in pts:
        rays.append((x, y, 2.0, 0.0, 0.0, -1.0, np.inf))        # straight down
        rays.append((x, y, 2.0, 0.25, -0.5, -1.0, np.inf))      # oblique
        rays.append((x, y, -3.0, 0.0, 0.0, 1.0, 4.0))           # from below, tMax at the top sheet
    rays = np.array(rays, np.float32)
    for any_hit in (False, True):
        g = hip.intersect(rays, any_hit)
        c = O.intersect(s, rays, any_hit)
        assert np.array_equal(g.view(np.uint32), c.view(np.uint32))
    assert (c[:, 0] > 0).sum() > len(rays) // 2


def test_scene_without_geometry_and_without_lights(hip):
    """No primitives (an empty BVH): every camera ray escapes — the F4 grey 0.8 per light under
    Whitted, black without lights; Path sees only infinite lights."""
    cam = scenes.camera(8, 6, (0, 0, 3), (0, 0, 0))
    s = scenes.Scene()
    s.point_light((0.0, 2.0, 0.0), (5.0, 5.0, 5.0))
    hip.upload(s)
    g, g8, _ = hip.render(scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 2, 5))
    c, c8, _ = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 2, 5))
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)) and np.allclose(g, 0.8)
    s2 = scenes.Scene()
    s2.sphere((0.0, 0.0, 0.0), 1.0, s2.matte((0.5, 0.5, 0.5)))
    hip.upload(s2)
    for integ in (capi.INTEGRATOR_WHITTED, capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH):
        rd = scenes.render_desc(cam, integ, 2, 5)
        g, _, _ = hip.render(rd)
        c, _, _ = O.render(s2, rd)
        assert np.array_equal(g.view(np.uint32), c.view(np.uint32)) and not g.any()


@pytest.mark.parametrize("w,h,spp", [(1, 1, 1), (7, 3, 3), (65, 1, 5), (1, 130, 2)])
def test_degenerate_frames_and_odd_spp(hip, w, h, spp):
    s, _ = scenes.config_c1(w, h, spp)
    cam = scenes.camera(w, h, (0.0, 0.0, 5.0), (0.0, 0.0, 0.0))
    hip.upload(s)
    for integ in (capi.INTEGRATOR_WHITTED, capi.INTEGRATOR_PATH):
        rd = scenes.render_desc(cam, integ, spp, 5)
        g, g8, st = hip.render(rd)
        c, c8, _ = O.render(s, rd)
        assert_parity(g, c, g8, c8)
        assert st.samples == w * h * spp


def test_ragged_tiles_and_single_pixel_tiles(hip):
    """Tiles that do not divide the frame, single pixels and a 1-row strip, in arbitrary order."""
    s, rd = scenes.config_c2(100, 37, 2, mesh=scenes.dragon_standin(n=32) + ("s",),
                             sky=np.ones((8, 16, 3), np.float32))
    tiles = [(64, 32, 100, 37), (0, 0, 1, 1), (99, 36, 100, 37), (3, 10, 97, 11), (0, 0, 64, 32)]
    rdt = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, tiles=tiles)
    hip.upload(s)
    g, g8, st = hip.render(rdt)
    c, c8, _ = O.render(s, rdt)
    assert np.array_equal(g.view(np.uint32), c.view(np.uint32)) and np.array_equal(g8, c8)
    assert st.samples == sum((x1 - x0) * (y1 - y0) for x0, y0, x1, y1 in tiles) * 2


@pytest.mark.parametrize("config", ["C3", "C5"])
def test_full_size_path_volpath_properties(hip, config):
    """BASELINE sizes of C3 (1080p, 256 spp, Path, Sobol — the sampler the reference lacks, F3, so
    the oracle is the only pin) and C5 (1080p, 512 spp, VolPath) on the default (benchmarked)
    schedule: finite, non-negative, deterministic frames, and 64 spot pixels against the oracle
    (same sampler indices: one-pixel tiles on the CPU) — L∞ within the north_star tolerance, the
    8-bit output identical wherever the float pixel is, and at least 95% of the pixels bit-exact."""
    s, rd = scenes.CONFIGS[config]()
    W, H = rd.camera.width, rd.camera.height
    hip.upload(s)
    g, g8, st = hip.render(rd)
    assert g.shape == (W * H, 3) and np.isfinite(g).all() and (g >= 0).all()
    assert st.samples == W * H * rd.spp
    rng = np.random.default_rng(7)
    picks = rng.choice(W * H, 64, replace=False)
    tiles = [(int(p % W), int(p // W), int(p % W) + 1, int(p // W) + 1) for p in picks]
    rdt = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                             rd.sampler, tiles=tiles)
    c, c8, _ = O.render(s, rdt)
    linf, exact = assert_parity(g[picks], c, g8[picks], c8)
    assert exact >= 0.95, f"{config}: only {exact:.3f} of the pixels bit-identical to the oracle"
    print(f"{config}: L∞ {linf:.3g}, bit-identical {exact:.3f}")
    again, _, _ = hip.render(rdt)
    assert np.array_equal(again.view(np.uint32), g[picks].view(np.uint32))


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_WHITTED, capi.INTEGRATOR_PATH])
def test_spp_beyond_one_finish_tile(hip, integrator):
    """spp > 2048: the finish kernels fold and sum a pixel's samples in slices of 2048, still in
    sample order (colObj += Li)."""
    s, _ = scenes.config_c1(4, 3, 1)
    cam = scenes.camera(4, 3, (0.0, 0.0, 5.0), (0.0, 0.0, 0.0))
    rd = scenes.render_desc(cam, integrator, 4100, 5)
    hip.upload(s)
    g, g8, st = hip.render(rd)
    c, c8, _ = O.render(s, rd)
    assert st.samples == 4 * 3 * 4100
    assert_parity(g, c, g8, c8)


def test_deep_whitted_mirror_box(hip):
    """Two facing mirrors bounce camera rays until Whitted's depth limit: the wavefront schedule
    (up to 16 levels) and the megakernel (up to 64) agree bit for bit and with the oracle, and a
    deeper maxDepth is refused rather than truncated."""
    s = scenes.Scene()
    mirror = s.mirror((0.9, 0.9, 0.9))
    matte = s.matte((0.6, 0.3, 0.2))
    for z, flip in ((-1.0, False), (1.5, True)):
        P = np.array([(-3, -3, z), (3, -3, z), (3, 3, z), (-3, 3, z)], np.float32)
        I = np.array([(0, 1, 2), (0, 2, 3)] if not flip else [(0, 2, 1), (0, 3, 2)], np.int32)
        s.mesh(P, I, mirror)
    s.sphere((0.0, 0.0, 0.2), 0.3, matte)
    s.point_light((0.0, 1.0, 0.5), (4.0, 4.0, 4.0))
    cam = scenes.camera(40, 30, (0.2, 0.1, 1.2), (0.0, 0.0, -1.0))
    hip.upload(s)
    for depth in (5, 12, 16, 40):
        rd = scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 4, depth)
        g, g8, _ = hip.render(rd)
        c, c8, _ = O.render(s, rd)
        assert_parity(g, c, g8, c8)
        hip.set_schedule(kernels=capi.KERNELS_MEGAKERNEL)
        mk, _, _ = hip.render(rd)
        hip.set_schedule()
        assert np.array_equal(mk.view(np.uint32), g.view(np.uint32)), depth
    with pytest.raises(RuntimeError):
        hip.render(scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 1, 65))


def test_sobol_raster_limit_is_refused(hip):
    """The device keeps a Sobol sample's (px << m) | py and the low 32 index bits in 32-bit words,
    with the higher bits from frame >> (32 - 2m): rasters of 2^16 and more per side (m >= 16,
    max(width, height) > 32768) are refused with PBR_E_UNSUPPORTED instead of silently wrong
    samples; 32768 is still accepted."""
    s, _ = scenes.config_c1(8, 8, 1)
    hip.upload(s)
    for w, ok in ((40000, False), (32768, True)):
        cam = scenes.camera(w, 2, (0.0, 0.0, 5.0), (0.0, 0.0, 0.0))
        rd = scenes.render_desc(cam, capi.INTEGRATOR_PATH, 1, 1, sampler=capi.SAMPLER_SOBOL, tiles=[(0, 0, 4, 2)])
        if ok:
            g, _, _ = hip.render(rd)
            assert np.isfinite(g).all()
        else:
            with pytest.raises(RuntimeError, match="32768"):
                hip.render(rd)
