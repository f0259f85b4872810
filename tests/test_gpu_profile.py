"""The per-kernel profile (pbr_hip_set_profiling / pbr_hip_get_profile) that bench.py's roofline
reads: launch counts, units and pushes must agree with each other and with the frame's geometry, and
profiling must not change the image."""
import numpy as np
import pytest

from pysicalbasedraytracer_amd import HipRenderer, capi, scenes


@pytest.fixture(scope="module")
def hip():
    r = HipRenderer(0)
    yield r
    r.close()


def _c2_small():
    return scenes.config_c2(192, 108, 16)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["0", "1"])
def test_whitted_profile_counts_are_consistent(hip, fused):
    # several chunks over the lanes; fused: the level-0 shade traces its own camera rays
    # (multi-chunk frames, the default)
    hip.set_schedule(chunk_log2=16, fuse_camera=capi.FUSE_ON if fused == "1" else capi.FUSE_OFF)
    s, rd = _c2_small()
    hip.upload(s)
    ref, ref8, _ = hip.render(rd)
    hip.set_profiling(2)
    g, g8, _ = hip.render(rd)
    prof = hip.get_profile()
    hip.set_profiling(0)
    assert np.array_equal(g, ref) and np.array_equal(g8, ref8)   # profiling changes nothing
    n = 192 * 108 * 16
    shade, shadow, extend, fin = (prof[k] for k in ("k_wf_shade", "k_wf_shadow", "k_wf_extend", "k_wf_finish"))
    assert fin["units"] == 192 * 108 and fin["counts"][1] == n and fin["launches"] > 1
    if fused == "0":
        cam = prof["k_wf_camera_extend"]
        assert cam["units"] == n and cam["launches"] == fin["launches"]
        assert "k_wf_shade_l0" not in prof
        shades = [shade]
        assert shade["launches"] == fin["launches"] * rd.max_depth == shadow["launches"]
        # shade's level-0 input is every sample; deeper levels read what the previous level pushed
        assert shade["units"] == n + extend["units"]
    else:
        # the fused level-0 launches (camera rays traced in the shade) are their own family
        assert "k_wf_camera_extend" not in prof
        l0 = prof["k_wf_shade_l0"]
        shades = [l0, shade]
        assert l0["launches"] == fin["launches"] and shade["launches"] == fin["launches"] * (rd.max_depth - 1)
        assert l0["launches"] + shade["launches"] == shadow["launches"]
        assert l0["units"] == n and shade["units"] == extend["units"]
        assert l0["counts"][5] == 0
    assert shadow["units"] == sum(v["counts"][1] for v in shades) and 0 < shadow["counts"][1] <= shadow["units"]
    assert extend["units"] == sum(v["counts"][4] for v in shades) == sum(v["counts"][5] for v in shades)
    for v in prof.values():
        assert v["ms"] > 0 and v["bytes"] > 0
    # round 4 fields: f[6] = level-0 samples of fused launches (they read no queue entry), f[7] =
    # shadow pushes that carry a SkyBox direction (C2: every one), shadow f[2] = those that got
    # through (the sky lookup reads the direction); the byte formulas of pbr_kernels.hip
    assert sum(v["counts"][6] for v in shades) == (n if fused == "1" else 0)
    for v in shades:
        f = v["counts"]
        assert f[7] == f[1]
        assert v["bytes"] == 72 * f[0] - 48 * f[6] + 4 * f[5] + 52 * f[1] + 52 * f[4] + 16 * f[7]
    assert shadow["counts"][2] == shadow["counts"][1]
    rec = sum(16 * v["counts"][0] + 20 * v["counts"][4] for v in shades)
    assert fin["bytes"] == 16 * fin["counts"][0] + 4 * fin["counts"][1] + rec
    g2 = shadow["counts"]
    assert shadow["bytes"] == 52 * g2[0] + 32 * g2[1] + 16 * g2[2]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_path_profile_counts_are_consistent(hip, cfg):
    s, rd = getattr(scenes, f"config_{cfg}")(64, 48, 16)
    hip.upload(s)
    hip.set_profiling(2)
    hip.render(rd)
    prof = hip.get_profile()
    hip.set_profiling(0)
    n = 64 * 48 * 16
    shade = prof["k_wfv_shade" if cfg == "c5" else "k_wfp_shade"]
    assert prof["k_wfp_camera_extend"]["units"] == n
    assert shade["units"] == n + prof["k_wf_extend"]["units"]
    anyhit = prof["k_wfv_tr"] if cfg == "c5" else prof["k_wfp_shadow"]
    assert anyhit["units"] == shade["counts"][1]
    assert prof["k_wfp_probe"]["units"] == shade["counts"][2]
    assert prof["k_wfv_resolve" if cfg == "c5" else "k_wfp_resolve"]["units"] == shade["counts"][3]
    assert prof["k_wfp_finish"]["units"] == 64 * 48


@pytest.mark.gpu
def test_profile_timing_only_window(hip):
    s, rd = _c2_small()
    hip.upload(s)
    hip.set_profiling(1)
    hip.render(rd)
    hip.render(rd)
    prof = hip.get_profile()
    hip.set_profiling(0)
    assert prof["k_wf_camera_extend"]["launches"] == 2
    assert prof["k_wf_camera_extend"]["units"] == 0   # timings only: no counting launches
    assert all(v["ms"] > 0 for v in prof.values())


@pytest.mark.gpu
def test_classed_shade_one_launch_per_material_set(hip):
    """C4's materials hold four lobe sets (rough glass, metal, plastic, matte): the Path shade runs one
    launch per set and bounce (k_wfp_shade CLASSED), each shading only its set's hits, and the
    counts of the bounce still add up (every queued ray shaded once)."""
    s, rd = scenes.config_c4(64, 48, 8)
    hip.upload(s)
    hip.set_profiling(2)
    hip.render(rd)
    prof = hip.get_profile()
    hip.set_profiling(0)
    n = 64 * 48 * 8
    shade = prof["k_wfp_shade"]
    assert shade["launches"] == 4 * prof["k_wfp_resolve"]["launches"]
    assert shade["units"] == n + prof["k_wf_extend"]["units"]
    assert prof["k_wfp_shadow"]["units"] == shade["counts"][1]
    assert prof["k_wfp_probe"]["units"] == shade["counts"][2]


@pytest.mark.gpu
def test_classed_volpath_shade_passes(hip):
    """C5's VolPath scene (matte floor and light, rough glass dragon filled with a medium): pass 0,
    the medium pass, takes the rays inside the medium and the misses; the matte hits and the glass
    hits (from outside, and from inside once the medium pass has sampled the medium) get a pass
    each — three k_wfv_shade launches per bounce."""
    s, rd = scenes.config_c5(64, 48, 8)
    hip.upload(s)
    hip.set_profiling(2)
    hip.render(rd)
    prof = hip.get_profile()
    hip.set_profiling(0)
    assert prof["k_wfv_shade"]["launches"] == 3 * prof["k_wfv_resolve"]["launches"]
