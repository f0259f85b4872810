"""InfiniteAreaLight (Light/InfiniteAreaLight.cpp) — the reference's own main.cpp scene lights its
VolPath render with one (main.cpp:377-381, RotateX(-90)·RotateY(-0)·RotateZ(-50), L = 1).

CPU tier: the oracle's MIPMap / Distribution2D / Sample_Li / Pdf_Li checked against closed forms
(the reference ships no fixture for this light: parity is pinned analytically here and by the
device-vs-oracle tier below).  GPU tier: the device render against the oracle for every
integrator, with a non-power-of-two image (Lanczos resampling, MIPMap.h:86-150) under the rotated
light-to-world transform.
"""
import numpy as np
import pytest

import oracle_lib as O
from pysicalbasedraytracer_amd import capi, scenes


def main_cpp_xform():
    """InfinityLightToWorld = RotateX(-90) * RotateY(-0) * RotateZ(-50) (main.cpp:377)."""
    return scenes.compose(scenes.compose(scenes.rotate_x(-90), scenes.rotate_y(-0.0)), scenes.rotate_z(-50))


def floor_scene(L=(0.5, 0.5, 0.5), env=None, kd=0.6, xform=None):
    s = scenes.Scene()
    m = s.matte((kd, kd, kd))
    Pf, If = scenes.quad(0.0, 50.0)
    s.mesh(Pf, If, m)
    s.infinite_light(env, L=L, xform=xform)
    return s


def test_constant_map_le_on_miss():
    """A 1x1 map of L (no image): escaping camera rays see L under Whitted (bilinear weights of a
    constant map sum to 1 up to rounding)."""
    s = scenes.Scene()
    m = s.matte((0.5, 0.5, 0.5))
    s.sphere((0.0, -100.0, 0.0), 1.0, m)          # far outside the view
    s.infinite_light(None, L=(0.25, 0.5, 0.75))
    cam = scenes.camera(16, 16, (0, 0, 3), (0, 0, 0))
    rgb, _, _ = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 1, 5))
    assert np.allclose(rgb, [0.25, 0.5, 0.75], rtol=1e-6, atol=0)


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH])
def test_lambertian_floor_under_constant_sky(integrator):
    """Direct light on a Lambertian plane under a constant environment: Lo = Kd·L (E = πL).  The
    light sample goes through Distribution2D::SampleContinuous and the MIS weights through Pdf_Li,
    so a wrong pdf in either biases the mean."""
    s = floor_scene(L=(0.5, 0.5, 0.5), kd=0.6)
    cam = scenes.camera(32, 32, (0.0, 2.0, 0.0), (0.0, 0.0, -1.0), up=(0.0, 1.0, 0.0))
    rd = scenes.render_desc(cam, integrator, 64, 1, sampler=capi.SAMPLER_HALTON)
    rgb, _, _ = O.render(s, rd)
    rgb = rgb.reshape(32, 32, 3)
    floor = rgb[20:, :, :]                        # rows looking down at the plane
    assert abs(float(floor.mean()) - 0.3) < 0.3 * 0.02, float(floor.mean())


def test_importance_sampling_unbiased_with_sun():
    """A small bright sun in a dim sky: the Distribution2D-importance-sampled light estimate and
    the BSDF-sampled estimate are combined by MIS; the frame mean must match a high-spp render of
    the same frame within Monte Carlo noise, and the estimate concentrates (low variance) because
    the sun is importance sampled."""
    env = np.full((16, 32, 3), 0.05, np.float32)
    env[4, 9] = 400.0                             # the sun texel (rows as stbi_loadf returns them)
    s = floor_scene(L=(1.0, 1.0, 1.0), env=env, kd=0.5)
    cam = scenes.camera(24, 24, (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    lo = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_PATH, 16, 1))[0].reshape(24, 24, 3)[14:]
    hi = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_PATH, 256, 1))[0].reshape(24, 24, 3)[14:]
    assert np.isfinite(lo).all() and (lo >= 0).all()
    assert abs(lo.mean() - hi.mean()) < 0.05 * hi.mean(), (lo.mean(), hi.mean())


def test_power_distribution_uses_infinite_power():
    """Power() = 4π²R²·Lookup(.5,.5,.5) (InfiniteAreaLight.cpp:63-67) feeds the power light
    distribution: with a point light of equal power both are picked equally often, so the render
    under LIGHTS_POWER equals the one under LIGHTS_UNIFORM for two lights of equal power."""
    s = floor_scene(L=(0.5, 0.5, 0.5), kd=0.6)
    # the floor quad spans ±50 (the scene bound), so R = |c − pMax| = 50·√2; Power = 4π²R²·0.5
    R = np.float32(np.sqrt(np.float32(50.0) ** 2 * 2))
    p_inf = np.float32(4 * np.pi * np.pi) * R * R * np.float32(0.5)
    I = float(p_inf / np.float32(4 * np.pi))
    s.point_light((0.0, 3.0, 0.0), (I, I, I))
    cam = scenes.camera(16, 16, (0.0, 2.0, 0.0), (0.0, 0.0, -1.0))
    a = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_PATH, 4, 1, light_strategy=capi.LIGHTS_POWER))[0]
    b = O.render(s, scenes.render_desc(cam, capi.INTEGRATOR_PATH, 4, 1, light_strategy=capi.LIGHTS_UNIFORM))[0]
    assert np.allclose(a, b, rtol=2e-3, atol=1e-6)


# ----------------------------------------------------------------------------- device parity
def sky_small():
    return scenes.procedural_sky(100, 50, seed=3)     # not a power of two: Lanczos resampling


def dragon_scene(material, xform=None, medium=False, extra_light=None):
    s = scenes.Scene()
    P, I = scenes.dragon_standin(n=40)
    if medium:
        med = s.homogeneous_medium(0.5, 4.4, -0.5)
        s.mesh(P, I, material(s), medium_inside=med, medium_outside=-1)
    else:
        s.mesh(P, I, material(s))
    Pf, If = scenes.quad(-1.12, 6.0)
    s.mesh(Pf, If, s.matte((0.8, 0.8, 0.8)))
    s.infinite_light(sky_small(), L=(1.0, 1.0, 1.0), xform=xform if xform is not None else main_cpp_xform())
    if extra_light:
        extra_light(s)
    return s


@pytest.fixture(scope="module")
def hip():
    from pysicalbasedraytracer_amd import HipRenderer
    r = HipRenderer(0)
    yield r
    r.close()


def pair(hip, s, rd):
    from test_gpu_parity import compare
    hip.upload(s)
    g, g8, _ = hip.render(rd)
    c, c8, _ = O.render(s, rd)
    return compare(g, c, g8, c8)


CAM = dict(eye=(0.0, 0.55, 2.6), look=(0.0, -0.25, 0.0))


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["whitted", "whitted_two_lights", "path", "path_power_area", "volpath"])
def test_infinite_light_device_vs_oracle(hip, case):
    cam = scenes.camera(64, 40, CAM["eye"], CAM["look"])
    if case == "whitted":
        s = dragon_scene(lambda sc: sc.matte((0.1, 0.8, 0.2)))
        rd = scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 8, 5)
    elif case == "whitted_two_lights":
        s = dragon_scene(lambda sc: sc.mirror(), extra_light=lambda sc: sc.point_light((0.5, 2.0, 1.0), (4.0, 4.0, 4.0)))
        rd = scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 8, 5)
    elif case == "path":
        s = dragon_scene(lambda sc: sc.plastic())
        rd = scenes.render_desc(cam, capi.INTEGRATOR_PATH, 8, 6, rr_threshold=0.8, sampler=capi.SAMPLER_SOBOL)
    elif case == "path_power_area":
        def area(sc):
            Pl, Il = scenes.quad(2.45, 1.4, flip=True)
            sc.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), sc.matte((0.8, 0.8, 0.8)), n_samples=5)
        s = dragon_scene(lambda sc: sc.metal(), extra_light=area)
        rd = scenes.render_desc(cam, capi.INTEGRATOR_PATH, 8, 6, light_strategy=capi.LIGHTS_POWER)
    else:
        s = dragon_scene(lambda sc: sc.glass(), medium=True)
        rd = scenes.render_desc(cam, capi.INTEGRATOR_VOLPATH, 8, 10)
    pair(hip, s, rd)


@pytest.mark.gpu
def test_infinite_light_wavefront_equals_megakernel(hip):
    cam = scenes.camera(64, 40, CAM["eye"], CAM["look"])
    for integ, mat in ((capi.INTEGRATOR_WHITTED, lambda sc: sc.matte((0.1, 0.8, 0.2))),
                       (capi.INTEGRATOR_PATH, lambda sc: sc.plastic())):
        s = dragon_scene(mat)
        rd = scenes.render_desc(cam, integ, 8, 6)
        hip.upload(s)
        hip.set_schedule()
        wf, _, _ = hip.render(rd)
        hip.set_schedule(kernels=capi.KERNELS_MEGAKERNEL)
        mk, _, _ = hip.render(rd)
        assert np.array_equal(wf.view(np.uint32), mk.view(np.uint32)), float(np.abs(wf - mk).max())
