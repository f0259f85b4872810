"""Material and shape options the BASELINE configs do not exercise, device vs oracle
(per-pixel L∞ ≤ 1e-3, 8-bit ≤ 1): Oren-Nayar matte (sigma > 0, Reflection.cpp:176-199), an
anisotropic metal on a mesh with per-vertex UVs (the shading frame follows dpdu,
Triangle.cpp:148-170), two-sided area lights (DiffuseLight.h:17-19), reversed orientation under a
handedness-swapping transform, and a material-less medium interface crossed by Path/VolPath."""
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


def check(hip, s, rd):
    hip.upload(s)
    g, g8, _ = hip.render(rd)
    c, c8, _ = O.render(s, rd)
    assert_parity(g, c, g8, c8)
    return g


def uv_patch(n=12, z=-0.2):
    """A wavy n×n patch with per-vertex UVs stretched in u (so dpdu ≠ the edge directions)."""
    xs = np.linspace(-1.5, 1.5, n + 1, dtype=np.float32)
    P, UV = [], []
    for j, y in enumerate(xs):
        for i, x in enumerate(xs):
            P.append((x, y * 0.6 - 0.4, z + 0.15 * np.sin(2.0 * x) * np.cos(1.5 * y)))
            UV.append((3.0 * i / n, j / n))
    I = []
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i, (j + 1) * (n + 1) + i + 1
            I += [(a, b, d), (a, d, c)]
    return np.array(P, np.float32), np.array(I, np.int32), np.array(UV, np.float32)


def lit_scene(material_fn, two_sided=False, uv=True):
    s = scenes.Scene()
    P, I, UV = uv_patch()
    s.mesh(P, I, material_fn(s), uv=UV if uv else None)
    s.sphere((0.6, 0.1, 0.3), 0.35, s.matte((0.3, 0.6, 0.3), sigma=25.0))
    Pl, Il = scenes.quad(1.8, 0.8, flip=True)
    s.area_light_mesh(Pl, Il, (4.0, 4.0, 4.0), s.matte((0.5, 0.5, 0.5)), n_samples=2, two_sided=two_sided)
    s.point_light((-1.0, 1.5, 1.5), (3.0, 3.0, 3.0))
    return s


CAM = dict(eye=(0.0, 0.8, 2.6), look=(0.0, -0.2, 0.0))


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_WHITTED, capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH])
def test_oren_nayar_matte(hip, integrator):
    s = lit_scene(lambda sc: sc.matte((0.7, 0.5, 0.3), sigma=20.0))
    cam = scenes.camera(48, 32, CAM["eye"], CAM["look"])
    check(hip, s, scenes.render_desc(cam, integrator, 8, 5))


@pytest.mark.parametrize("uv", [True, False])
def test_anisotropic_metal_uv_mesh(hip, uv):
    s = lit_scene(lambda sc: sc.metal(urough=0.05, vrough=0.4), uv=uv)
    cam = scenes.camera(48, 32, CAM["eye"], CAM["look"])
    check(hip, s, scenes.render_desc(cam, capi.INTEGRATOR_PATH, 8, 6, sampler=capi.SAMPLER_SOBOL))


def test_two_sided_area_light(hip):
    """The light quad faces down; seen from below (two-sided) it lights the floor, and the
    camera above sees its back emitting too."""
    s = lit_scene(lambda sc: sc.plastic(), two_sided=True)
    cam = scenes.camera(48, 32, (0.0, 2.6, 0.5), (0.0, -0.5, 0.0))
    for integ in (capi.INTEGRATOR_PATH, capi.INTEGRATOR_WHITTED):
        check(hip, s, scenes.render_desc(cam, integ, 8, 5))


def test_reversed_orientation_mirrored_transform(hip):
    """ReverseOrientation ^ TransformSwapsHandedness flips the geometric normal
    (Triangle.cpp:186-190, Shape.h:35): a mirrored (scale -1) emitter mesh and a reversed sphere."""
    s = scenes.Scene()
    P, I, UV = uv_patch()
    s.mesh(P, I, s.matte((0.6, 0.6, 0.6)))
    xf = scenes.compose(scenes.translate(0.0, 1.8, 0.0), scenes.scale(-1.0, 1.0, 1.0))
    Pl, Il = scenes.quad(0.0, 0.8, flip=True)
    s.area_light_mesh(Pl, Il, (4.0, 4.0, 4.0), s.matte((0.5, 0.5, 0.5)), xform=xf)
    s.sphere((0.5, 0.2, 0.3), 0.3, s.glass(urough=0.0, vrough=0.0), reverse=True)
    cam = scenes.camera(48, 32, CAM["eye"], CAM["look"])
    for integ in (capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH):
        check(hip, s, scenes.render_desc(cam, integ, 8, 6))


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH])
def test_material_less_medium_interface(hip, integrator):
    """A material-less sphere bounding a homogeneous medium (pbrt's interface idiom): rays cross it
    without a bounce (PathIntegrator.cpp:70-75, VolPathIntegrator.cpp:77-82); the wavefront
    schedule equals the megakernel bit for bit."""
    s = scenes.Scene()
    P, I, UV = uv_patch()
    s.mesh(P, I, s.matte((0.6, 0.6, 0.6)))
    med = s.homogeneous_medium(0.3, 1.5, 0.3)
    s.sphere((0.0, 0.1, 0.2), 0.5, -1, medium_inside=med, medium_outside=-1)
    s.sphere((0.0, 0.1, 0.2), 0.25, -1)                  # a second pass-through shell inside
    Pl, Il = scenes.quad(1.8, 0.8, flip=True)
    s.area_light_mesh(Pl, Il, (4.0, 4.0, 4.0), s.matte((0.5, 0.5, 0.5)))
    cam = scenes.camera(48, 32, CAM["eye"], CAM["look"])
    rd = scenes.render_desc(cam, integrator, 8, 6)
    g = check(hip, s, rd)
    hip.set_schedule(kernels=capi.KERNELS_MEGAKERNEL)
    mk, _, _ = hip.render(rd)
    assert np.array_equal(mk.view(np.uint32), g.view(np.uint32))


def nested_shells(n, r0=0.05, r1=0.6, medium=True, center=(0.0, 0.1, 0.2)):
    """A matte patch behind n concentric material-less spheres (pass-through surfaces), the
    outermost one bounding a homogeneous medium, and an area light."""
    s = scenes.Scene()
    P, I, UV = uv_patch()
    s.mesh(P, I, s.matte((0.6, 0.6, 0.6)))
    med = s.homogeneous_medium(0.3, 1.5, 0.3) if medium else -1
    for k, r in enumerate(np.linspace(r1, r0, n)):
        if k == 0 and medium:
            s.sphere(center, float(r), -1, medium_inside=med, medium_outside=-1)
        else:
            s.sphere(center, float(r), -1)
    Pl, Il = scenes.quad(1.8, 0.8, flip=True)
    s.area_light_mesh(Pl, Il, (4.0, 4.0, 4.0), s.matte((0.5, 0.5, 0.5)))
    return s


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH])
def test_many_material_less_crossings(hip, integrator):
    """20 nested material-less shells: a path through the centre crosses 40 surfaces before its
    first bounce, more than the 32 extra levels the wavefront schedules up front.  The schedule
    keeps extending while continuations are queued, so it equals the megakernel (which loops
    without a bound, as the reference does) bit for bit, and the oracle."""
    s = nested_shells(20)
    cam = scenes.camera(40, 28, CAM["eye"], CAM["look"])
    rd = scenes.render_desc(cam, integrator, 4, 5)
    g = check(hip, s, rd)
    hip.set_schedule(kernels=capi.KERNELS_MEGAKERNEL)
    mk, _, _ = hip.render(rd)
    assert np.array_equal(mk.view(np.uint32), g.view(np.uint32))


def test_transmittance_walk_bound_fails_loudly(hip):
    """300 nested shells centred on a point of the patch: a shadow ray from there to the light
    crosses 300 interfaces (VisibilityTester::Tr), past the 256-interface safety bound, so the
    render fails with an error (both schedules) instead of returning a truncated transmittance.
    The camera rays' 300 pass-through crossings are followed (the wavefront keeps extending).
    Asynchronous frames report the failure at the next call (pbr_hip_sync)."""
    import torch
    s = nested_shells(300, r0=0.3, r1=0.6, center=(0.0, 0.0, -0.2))
    cam = scenes.camera(16, 12, CAM["eye"], CAM["look"])
    rd = scenes.render_desc(cam, capi.INTEGRATOR_VOLPATH, 2, 3)
    hip.upload(s)
    with pytest.raises(RuntimeError, match="transmittance walk"):
        hip.render(rd)
    g, _, _ = hip.render(scenes.render_desc(cam, capi.INTEGRATOR_PATH, 2, 3))   # Path has no Tr walk
    assert np.isfinite(g).all()
    n = 16 * 12
    rgb = torch.empty((n, 3), dtype=torch.float32, device="cuda")
    rgba = torch.empty((n, 4), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    hip.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream, sync=False)
    with pytest.raises(RuntimeError, match="transmittance walk"):
        hip.sync()
    hip.sync()   # the failure is reported once
    # ... or by the next render call, even one enqueued right behind the failing frame: the call
    # waits for that frame before reading the flag, and blames the frame that tripped it
    hip.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream, sync=False)
    with pytest.raises(RuntimeError, match="transmittance walk"):
        hip.render_device(scenes.render_desc(cam, capi.INTEGRATOR_PATH, 2, 3), rgb.data_ptr(), rgba.data_ptr(),
                          stream=stream.cuda_stream, sync=False)
    g2, _, _ = hip.render(scenes.render_desc(cam, capi.INTEGRATOR_PATH, 2, 3))   # reported once
    assert np.array_equal(g2.view(np.uint32), g.view(np.uint32))
    hip.set_schedule(kernels=capi.KERNELS_MEGAKERNEL)
    with pytest.raises(RuntimeError, match="transmittance walk"):
        hip.render(rd)


def test_none_material_is_no_material(hip):
    """A PBR_MAT_NONE material is `material == nullptr` (include/pbr_hip.h): primitives that use it
    are pass-through medium boundaries, on the device and in the oracle, exactly like index -1
    (VolPath's Tr walk crosses them instead of being blocked, VisibilityTester::Tr, Light.cpp:31-47)."""
    def scene(none_index):
        s = scenes.Scene()
        P, I, UV = uv_patch()
        s.mesh(P, I, s.matte((0.6, 0.6, 0.6)))
        med = s.homogeneous_medium(0.3, 1.5, 0.3)
        mat = -1
        if none_index:
            s.materials.append(capi.MaterialDesc(type=capi.MAT_NONE))
            mat = len(s.materials) - 1
        s.sphere((0.0, 0.1, 0.2), 0.5, mat, medium_inside=med, medium_outside=-1)
        Pl, Il = scenes.quad(1.8, 0.8, flip=True)
        s.area_light_mesh(Pl, Il, (4.0, 4.0, 4.0), s.matte((0.5, 0.5, 0.5)))
        return s
    cam = scenes.camera(48, 32, CAM["eye"], CAM["look"])
    rd = scenes.render_desc(cam, capi.INTEGRATOR_VOLPATH, 8, 6)
    g_none = check(hip, scene(True), rd)
    hip.upload(scene(False))
    g_idx, _, _ = hip.render(rd)
    assert np.array_equal(g_none.view(np.uint32), g_idx.view(np.uint32))
