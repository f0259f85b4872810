"""The C-ABI library loads and exports every symbol include/pbr_hip.h declares (no GPU calls)."""
import ctypes as C
import os
import re

import pytest

from pysicalbasedraytracer_amd import capi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "pbr_hip.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(pbr_hip_[a-z_]+)\s*\(", txt)))


def test_header_and_ctypes_table_agree():
    assert declared_symbols() == sorted(capi.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = capi.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.pbr_hip_abi_version() == capi.ABI_VERSION


def test_struct_sizes_match_c():
    # the ctypes mirror must match the C layout (x86-64 SysV)
    assert C.sizeof(capi.Transform) == 128
    assert C.sizeof(capi.Tile) == 16
    assert C.sizeof(capi.RenderStats) == 8 * 8 + 8
    assert C.sizeof(capi.SurfaceHit) == 112
    assert C.sizeof(capi.KernelProfile) == 136


def test_no_device_returns_error_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = capi.load_library()
    ctx = C.c_void_p()
    assert lib.pbr_hip_create(0, C.byref(ctx)) in (capi.PBR_E_NODEVICE, capi.PBR_E_HIP)


def test_null_arguments_are_rejected():
    lib = capi.load_library()
    assert lib.pbr_hip_create(0, None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_upload_scene(None, None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_render(None, None, None, None, None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_destroy(None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_query(None, 1, None, 0, -1, None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_bounds(None, -1, None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_li(None, None, 1, None, None, 0, None) == capi.PBR_E_INVALID
    assert lib.pbr_hip_set_profiling(None, 1) == capi.PBR_E_INVALID
    assert lib.pbr_hip_get_profile(None, None, 0, None) == capi.PBR_E_INVALID


def test_release_library_reads_no_environment():
    """The shipped library has one measured schedule (include/pbr_hip.h pbr_hip_set_schedule is the
    only run-time switch): it imports no getenv, and it is not a development-knob build."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--undefined-only", capi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert not [l for l in out.splitlines() if "getenv" in l], "libpbr_hip.so imports getenv"
    build = capi.load_library().pbr_hip_build_info().decode()
    assert "dev-knobs" not in build, build


def test_schedule_arguments_are_validated():
    lib = capi.load_library()
    assert lib.pbr_hip_set_schedule(None, None) == capi.PBR_E_INVALID
