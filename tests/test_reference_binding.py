"""The reference-side drop-in (integration/reference_binding, VERDICT r3 missing 1), compiled against
the reference's own headers and exercised the way a user of the reference would use it.

oracle/ref/refbind_scenes.cpp assembles C2/C3/C5-shaped scenes from the reference's OWN classes as
Main/main.cpp:186-413 does, then renders each twice into the reference's FrameBuffer: once with the
reference's own SamplerIntegrator::Render (Integrator.cpp:280-356, Whitted/Path/VolPath) and once with
pbrhip::Hip{Whitted,Path,VolPath}Integrator — the same constructor arguments — which flattens the
reference Scene (its BVHAccel's tree included) into pbr_scene_desc and renders through the C-ABI.

Bar: the device walks the reference's own tree (its LinearBVHNode array, uploaded byte for byte);
the FrameBuffers are identical except where a last-bit libm difference (glibc's float sinf/expf/logf
in the reference, correctly rounded transcendentals on the device) moves a byte by one —
or, rarely, flips one sample's discrete decision (Russian roulette, a lobe or medium-event choice) and
moves its pixel further.  The oracle, which follows the device's rounding policy, shows the same
against the reference on its own scenes: C3 at 96×96×16 on Halton, 68 of 9216 float pixels differ,
one u8 byte by 4; C3 64×64×16 and C5 48×48×8, u8 identical (tests/ref_lib vs tests/oracle_lib, CPU).
So at most 0.1% of the pixels may differ by more than one."""
import ctypes as C
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libpbr_refbind.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="oracle/_ref/libpbr_refbind.so not built")


def lib():
    from pysicalbasedraytracer_amd import capi
    capi.load_library()   # torch first, then the product's HIP runtime (see capi.load_library)
    L = C.CDLL(LIB)
    L.refbind_render.restype = C.c_int
    L.refbind_render.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_double),
                                 C.POINTER(C.c_int), C.c_char_p, C.c_int]
    L.refbind_flatten.restype = C.c_int
    L.refbind_flatten.argtypes = [C.c_int, C.POINTER(C.c_int), C.c_char_p, C.c_int]
    return L


@pytest.mark.parametrize("config", [2, 3, 5])
def test_flattener_hands_over_the_reference_scene(config):
    """SceneFlattener over the reference's own objects: every primitive of the BVHAccel and every
    light reaches the descriptor, with the reference's whole node array (at most 2n - 1 nodes:
    leaves of one primitive, main.cpp's maxPrimsInNode 1, except where SAH keeps primitives with
    coincident centroids together — the stand-in's pole triangles)."""
    L = lib()
    counts = (C.c_int * 8)()
    err = C.create_string_buffer(512)
    assert L.refbind_flatten(config, counts, err, 512) == 0, err.value.decode()
    shapes, tris, mats, lights, media, nodes, ref_prims, ref_lights = list(counts)
    assert tris == ref_prims and lights == ref_lights and ref_prims < nodes <= 2 * ref_prims - 1
    assert media == (1 if config == 5 else 0)
    assert shapes >= 2 and mats >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("config,res,spp", [(2, 96, 8), (3, 64, 16), (5, 48, 8)])
def test_reference_render_equals_binding_render(config, res, spp):
    L = lib()
    ref = np.zeros(res * res * 4, np.uint8)
    hip = np.zeros(res * res * 4, np.uint8)
    secs = (C.c_double * 2)()
    same_tree = C.c_int(0)
    err = C.create_string_buffer(512)
    rc = L.refbind_render(config, res, spp, ref.ctypes.data, hip.ctypes.data, secs, C.byref(same_tree), err, 512)
    assert rc == 0, err.value.decode()
    assert same_tree.value == 1, "the device did not get the reference's BVHAccel node array"
    r = ref.reshape(-1, 4).astype(int)
    h = hip.reshape(-1, 4).astype(int)
    diff = np.abs(r - h).max(axis=1)
    same = float((diff == 0).mean())
    print(f"config {config}: {same:.4f} of the pixels identical, max |Δ| {int(diff.max())}, "
          f"reference {secs[0]:.2f} s, binding {secs[1]:.3f} s")
    assert (r[:, 3] == 255).all() and (h[:, 3] == 255).all()
    assert (diff <= 1).mean() >= 0.999, f"{int((diff > 1).sum())} pixels differ by more than one"
    assert same >= 0.98, f"only {same:.4f} of the pixels identical"
    assert r[:, :3].std() > 1.0   # a real image, not a blank frame
