"""ImageTexture (Texture/ImageTexture.h:43-91, ImageTexture.cpp:13-92) on the device path.

The reference itself pins the oracle and the device on two textured scenes (tests/test_ref_fixtures.py,
*_image_textures).  Here: the device against the oracle at larger sizes on every integrator (bar:
per-pixel L∞ ≤ 1e-3 on linear RGB, 8-bit exact wherever the float pixel is bit-identical), the
wavefront schedules against the megakernel bit for bit, and the upload's refusals.
"""
import numpy as np
import pytest

import oracle_lib as O
import ref_scenes as RS
from parity import assert_parity
from pysicalbasedraytracer_amd import HipRenderer, PbrError, capi, scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    r = HipRenderer(0)
    yield r
    r.close()


def textured_scene(integrator, w, h, spp, depth):
    s, rd = RS.render_cases()["path_image_textures"]
    if integrator == capi.INTEGRATOR_VOLPATH:
        med = s.homogeneous_medium(0.2, 0.8, -0.3)
        Pb, Ib = RS.box((-1.4, -1.1, -1.4), (1.4, 1.4, 1.4))
        s.mesh(Pb, Ib, -1, medium_inside=med, medium_outside=-1)
    cam = scenes.camera(w, h, **RS.CAM_C)
    return s, scenes.render_desc(cam, integrator, spp, depth, 0.8 if integrator != capi.INTEGRATOR_WHITTED else 1.0)


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_WHITTED, capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH])
def test_textured_scene_device_equals_oracle(hip, integrator):
    s, rd = textured_scene(integrator, 96, 54, 8, 6)
    hip.upload(s)
    g, g8, _ = hip.render(rd)
    c, c8, _ = O.render(s, rd)
    linf, exact = assert_parity(g, c, g8, c8)
    assert exact >= 0.99, exact


@pytest.mark.parametrize("integrator", [capi.INTEGRATOR_WHITTED, capi.INTEGRATOR_PATH, capi.INTEGRATOR_VOLPATH])
def test_textured_wavefront_equals_megakernel(hip, integrator):
    s, rd = textured_scene(integrator, 128, 72, 8, 6)
    hip.upload(s)
    hip.set_schedule()
    wf, wf8, _ = hip.render(rd)
    hip.set_schedule(kernels=capi.KERNELS_MEGAKERNEL)
    mk, mk8, _ = hip.render(rd)
    assert np.array_equal(wf.view(np.uint32), mk.view(np.uint32)), float(np.abs(wf - mk).max())
    assert np.array_equal(wf8, mk8)


def test_texture_changes_the_image(hip):
    """A textured Kd renders differently from its constant (the texture is really read)."""
    s, rd = textured_scene(capi.INTEGRATOR_WHITTED, 64, 36, 4, 5)
    hip.upload(s)
    a, _, _ = hip.render(rd)
    for m in s.materials:
        m.tex[capi.TEX_KD] = 0
    hip.upload(s)
    b, _, _ = hip.render(rd)
    assert np.abs(a - b).max() > 1e-2


def test_upload_refuses_bad_texture_use(hip):
    s = scenes.Scene()
    P, I = scenes.quad(0.0, 1.0)
    t_rgb = s.image_texture(np.ones((4, 4, 3), np.float32))
    t_f = s.image_texture(np.ones((4, 4, 3), np.float32), is_float=True)
    m = s.matte((0.5, 0.5, 0.5))
    s.mesh(P, I, m)
    s.point_light((0, 1, 0), (1, 1, 1))
    for slot, tex, why in ((capi.TEX_KD, t_f, "RGB"), (capi.TEX_SIGMA, t_rgb, "float"), (capi.TEX_KS, t_rgb, "slot")):
        s.materials[m].tex[:] = [0] * 6
        s.materials[m].tex[slot] = tex + 1
        with pytest.raises(PbrError, match=why):
            hip.upload(s)
    s.materials[m].tex[:] = [0] * 6
    s.materials[m].tex[capi.TEX_KD] = 9
    with pytest.raises(PbrError, match="out of range"):
        hip.upload(s)
    s2 = scenes.Scene()
    sm = s2.set_texture(s2.matte((0.5, 0.5, 0.5)), capi.TEX_KD, s2.image_texture(None))
    s2.sphere((0, 0, 0), 1.0, sm)
    with pytest.raises(PbrError, match="triangle meshes"):
        hip.upload(s2)
