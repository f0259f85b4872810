"""ctypes mirror of include/pbr_hip.h (the C-ABI drop-in boundary).

The structures here are byte-for-byte the C descriptors; `load_library()` opens the in-tree
`libpbr_hip.so` and fails loudly when it is missing — there is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 5

PBR_OK = 0
PBR_E_INVALID = -1
PBR_E_HIP = -2
PBR_E_NOSCENE = -3
PBR_E_UNSUPPORTED = -4
PBR_E_NODEVICE = -5

SHAPE_TRIANGLE_MESH, SHAPE_SPHERE = 0, 1
MAT_NONE, MAT_MATTE, MAT_MIRROR, MAT_GLASS, MAT_METAL, MAT_PLASTIC = range(6)
LIGHT_POINT, LIGHT_DIFFUSE_AREA, LIGHT_SKYBOX, LIGHT_INFINITE_AREA = 0, 1, 2, 3
INTEGRATOR_WHITTED, INTEGRATOR_PATH, INTEGRATOR_VOLPATH = 0, 1, 2
SAMPLER_HALTON, SAMPLER_SOBOL, SAMPLER_TABLE = 0, 1, 2
LIGHTS_UNIFORM, LIGHTS_POWER = 0, 1
BVH_BUILD_HOST, BVH_BUILD_DEVICE = 0, 1
SPLIT_SAH, SPLIT_HLBVH, SPLIT_MIDDLE, SPLIT_EQUAL_COUNTS = 0, 1, 2, 3
WRAP_REPEAT, WRAP_BLACK, WRAP_CLAMP = 0, 1, 2
TEX_KD, TEX_KS, TEX_KR, TEX_KT, TEX_SIGMA, TEX_ROUGHNESS = range(6)

F3 = C.c_float * 3
F16 = C.c_float * 16


class Transform(C.Structure):
    _fields_ = [("m", F16), ("m_inv", F16)]


class ShapeDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int),
        ("object_to_world", Transform),
        ("reverse_orientation", C.c_int),
        ("n_triangles", C.c_int),
        ("n_vertices", C.c_int),
        ("indices", C.POINTER(C.c_int32)),
        ("P", C.POINTER(C.c_float)),
        ("N", C.POINTER(C.c_float)),
        ("UV", C.POINTER(C.c_float)),
        ("radius", C.c_float),
        ("material", C.c_int),
        ("area_light_first", C.c_int),
        ("medium_inside", C.c_int),
        ("medium_outside", C.c_int),
    ]


class MaterialDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int),
        ("Kd", F3),
        ("sigma", C.c_float),
        ("Kr", F3),
        ("Kt", F3),
        ("Ks", F3),
        ("eta", C.c_float),
        ("metal_eta", F3),
        ("metal_k", F3),
        ("roughness", C.c_float),
        ("uroughness", C.c_float),
        ("vroughness", C.c_float),
        ("has_uv_roughness", C.c_int),
        ("remap_roughness", C.c_int),
        ("tex", C.c_int * 6),
    ]


class TextureDesc(C.Structure):
    _fields_ = [
        ("is_float", C.c_int),
        ("width", C.c_int),
        ("height", C.c_int),
        ("components", C.c_int),
        ("data", C.POINTER(C.c_float)),
        ("scale", C.c_float),
        ("gamma", C.c_int),
        ("wrap", C.c_int),
        ("trilinear", C.c_int),
        ("max_aniso", C.c_float),
        ("su", C.c_float),
        ("sv", C.c_float),
        ("du", C.c_float),
        ("dv", C.c_float),
        ("level0", C.c_int),
    ]


class LightDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int),
        ("light_to_world", Transform),
        ("I", F3),
        ("Le", F3),
        ("shape", C.c_int),
        ("triangle", C.c_int),
        ("two_sided", C.c_int),
        ("n_samples", C.c_int),
        ("medium_inside", C.c_int),
        ("medium_outside", C.c_int),
        ("world_center", F3),
        ("world_radius", C.c_float),
        ("env_width", C.c_int),
        ("env_height", C.c_int),
        ("env_components", C.c_int),
        ("env_data", C.POINTER(C.c_float)),
    ]


class MediumDesc(C.Structure):
    _fields_ = [("sigma_a", F3), ("sigma_s", F3), ("g", C.c_float)]


class SceneDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int),
        ("n_shapes", C.c_int),
        ("shapes", C.POINTER(ShapeDesc)),
        ("n_materials", C.c_int),
        ("materials", C.POINTER(MaterialDesc)),
        ("n_lights", C.c_int),
        ("lights", C.POINTER(LightDesc)),
        ("n_media", C.c_int),
        ("media", C.POINTER(MediumDesc)),
        ("max_prims_in_node", C.c_int),
        ("n_textures", C.c_int),
        ("textures", C.POINTER(TextureDesc)),
        ("split_method", C.c_int),
        ("bvh_nodes", C.c_void_p),
        ("n_bvh_nodes", C.c_int),
    ]


class CameraDesc(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("camera_to_world", Transform),
        ("use_look_at", C.c_int),
        ("eye", F3),
        ("look", F3),
        ("up", F3),
        ("fov", C.c_float),
        ("lens_radius", C.c_float),
        ("focal_distance", C.c_float),
        ("medium", C.c_int),
        ("use_raster_to_camera", C.c_int),
        ("raster_to_camera", Transform),
    ]


class Tile(C.Structure):
    _fields_ = [("x0", C.c_int), ("y0", C.c_int), ("x1", C.c_int), ("y1", C.c_int)]


class RenderDesc(C.Structure):
    _fields_ = [
        ("integrator", C.c_int),
        ("max_depth", C.c_int),
        ("rr_threshold", C.c_float),
        ("light_strategy", C.c_int),
        ("sampler", C.c_int),
        ("spp", C.c_int),
        ("camera", CameraDesc),
        ("n_tiles", C.c_int),
        ("tiles", C.POINTER(Tile)),
        ("outputs_on_device", C.c_int),
        ("stream", C.c_void_p),
        ("collect_stats", C.c_int),
        ("sobol_matrices", C.POINTER(C.c_uint32)),
        ("sobol_dims", C.c_int),
        ("sample_table", C.POINTER(C.c_float)),
        ("table_dims", C.c_int),
    ]


class RenderStats(C.Structure):
    _fields_ = [
        ("seconds", C.c_double),
        ("kernel_ms", C.c_double),
        ("film_ms", C.c_double),
        ("samples", C.c_uint64),
        ("rays", C.c_uint64),
        ("node_visits", C.c_uint64),
        ("prim_tests", C.c_uint64),
        ("shading_events", C.c_uint64),
        ("n_launches", C.c_int),
    ]


class SurfaceHit(C.Structure):
    _fields_ = [
        ("hit", C.c_int), ("prim", C.c_int), ("t", C.c_float), ("b", C.c_float * 3),
        ("p", C.c_float * 3), ("p_error", C.c_float * 3), ("n", C.c_float * 3), ("ns", C.c_float * 3),
        ("dpdu", C.c_float * 3), ("wo", C.c_float * 3), ("uv", C.c_float * 2),
        ("medium_inside", C.c_int), ("medium_outside", C.c_int),
    ]


class KernelProfile(C.Structure):
    _fields_ = [
        ("name", C.c_char * 40),
        ("launches", C.c_int),
        ("ms", C.c_double),
        ("units", C.c_uint64),
        ("bytes", C.c_uint64),
        ("counts", C.c_uint64 * 8),
    ]


KERNELS_AUTO, KERNELS_MEGAKERNEL = 0, 1
FUSE_AUTO, FUSE_OFF, FUSE_ON = 0, 1, 2


class Schedule(C.Structure):
    _fields_ = [("kernels", C.c_int), ("chunk_log2", C.c_int), ("lanes", C.c_int), ("fuse_camera", C.c_int),
                ("serial", C.c_int)]


# Every symbol include/pbr_hip.h declares, with its ctypes signature.
EXPORTS = {
    "pbr_hip_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "pbr_hip_upload_scene": (C.c_int, [C.c_void_p, C.POINTER(SceneDesc)]),
    "pbr_hip_render": (C.c_int, [C.c_void_p, C.POINTER(RenderDesc), C.c_void_p, C.c_void_p,
                                 C.POINTER(RenderStats)]),
    "pbr_hip_destroy": (C.c_int, [C.c_void_p]),
    "pbr_hip_last_error": (C.c_char_p, [C.c_void_p]),
    "pbr_hip_sync": (C.c_int, [C.c_void_p]),
    "pbr_hip_render_frames": (C.c_int, [C.c_void_p, C.POINTER(RenderDesc), C.c_int, C.POINTER(C.c_void_p),
                                        C.POINTER(C.c_void_p)]),
    "pbr_hip_wait_frame": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "pbr_hip_get_bvh": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int32),
                                  C.POINTER(C.c_int)]),
    "pbr_hip_sampler_values": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_float)]),
    "pbr_hip_sample_index": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "pbr_hip_sample_dimensions": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int64),
                                            C.POINTER(C.c_int32), C.POINTER(C.c_float)]),
    "pbr_hip_camera_rays": (C.c_int, [C.c_void_p, C.POINTER(CameraDesc), C.c_int, C.POINTER(C.c_float),
                                      C.POINTER(C.c_float)]),
    "pbr_hip_intersect": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int]),
    "pbr_hip_abi_version": (C.c_int, []),
    "pbr_hip_build_info": (C.c_char_p, []),
    "pbr_hip_sobol_matrices": (C.c_int, [C.c_int, C.POINTER(C.c_uint32)]),
    "pbr_hip_query": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_float), C.c_int, C.c_int, C.POINTER(SurfaceHit)]),
    "pbr_hip_bounds": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_float)]),
    "pbr_hip_li": (C.c_int, [C.c_void_p, C.POINTER(RenderDesc), C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int32),
                             C.c_int, C.POINTER(C.c_float)]),
    "pbr_hip_set_schedule": (C.c_int, [C.c_void_p, C.POINTER(Schedule)]),
    "pbr_hip_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "pbr_hip_get_profile": (C.c_int, [C.c_void_p, C.POINTER(KernelProfile), C.c_int, C.POINTER(C.c_int)]),
    "pbr_hip_set_bvh_build": (C.c_int, [C.c_void_p, C.c_int]),
    "pbr_hip_bvh_build_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double),
                                         C.POINTER(C.c_double)]),
    "pbr_hip_build_bvh": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float), C.c_int, C.c_void_p,
                                    C.POINTER(C.c_int), C.POINTER(C.c_int32), C.POINTER(C.c_double)]),
}

PACKAGE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PACKAGE_DIR, "libpbr_hip.so")

_lib = None


OPTIONAL_FOR_AB = ("pbr_hip_sync", "pbr_hip_set_profiling", "pbr_hip_get_profile", "pbr_hip_query", "pbr_hip_bounds",
                   "pbr_hip_li", "pbr_hip_set_bvh_build", "pbr_hip_bvh_build_info", "pbr_hip_build_bvh",
                   "pbr_hip_set_schedule", "pbr_hip_sample_index", "pbr_hip_sample_dimensions",
                   "pbr_hip_render_frames", "pbr_hip_wait_frame")


def load_library(path: str | None = None) -> C.CDLL:
    """Open the in-tree HIP library. Raises if it has not been built: no fallback exists."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libpbr_hip.so not built at {p}; run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: torch bundles its own libamdhip64 (same soname as /opt/rocm's).
    # Whichever loads first serves both, and torch fails to initialise ("No HIP GPUs are
    # available") on the newer system runtime, so let torch load first when it is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        if path is not None and name in OPTIONAL_FOR_AB and not hasattr(lib, name):
            continue   # an older experimental build (A/B timing runs) may predate this entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.pbr_hip_abi_version()
    # (v5 changed the texture and camera descriptors: an older build cannot take these structures)
    if v != ABI_VERSION:
        raise RuntimeError("libpbr_hip.so ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def fptr(a):
    """float32 numpy array → POINTER(c_float) (array must stay alive)."""
    return a.ctypes.data_as(C.POINTER(C.c_float))


def iptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))
