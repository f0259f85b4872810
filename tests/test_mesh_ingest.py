"""Mesh ingest: the reference's ".3d" reader (Shape/plyRead.h plyInfo: "vertex N
face M", vertices ×20) in Python (scenes.load_3d) and C++ (plyInfo), pinned to what the reference's
own reader returns for tests/golden/mesh_small.3d (tests/golden/mesh_ref.json, written by
make_mesh_fixtures.py through oracle/_ref); and the standard-PLY reader the real Stanford Dragon
needs (scenes.load_ply, C++ LoadPLY: ascii / binary_little_endian, extra properties, quads and
polygons fan-triangulated) — the reference has no PLY reader (it goes through assimp), so those are
pinned analytically: both formats of one mesh give the same triangles."""
import base64
import json
import os
import struct
import subprocess

import numpy as np
import pytest

from pysicalbasedraytracer_amd import scenes

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = os.path.join(HERE, "golden")


def _fixture():
    d = json.load(open(os.path.join(GOLD, "mesh_ref.json")))
    v = np.frombuffer(base64.b64decode(d["vertices_f32"]), "<f4").reshape(-1, 3)
    i = np.frombuffer(base64.b64decode(d["indices_i32"]), "<i4").reshape(-1, 3)
    return d, v, i


def _cpp(mode, path):
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp")], check=True)
    out = subprocess.run([os.path.join(HERE, "cpp", "host_api_test"), mode, path], capture_output=True, text=True,
                         check=True).stdout.split("\n")
    v = np.array([[int(t, 16) for t in l.split()[1:]] for l in out if l.startswith("v ")], np.uint32).reshape(-1, 3)
    f = np.array([[int(t) for t in l.split()[1:]] for l in out if l.startswith("f ")], np.int32).reshape(-1, 3)
    return v.view(np.float32), f


def test_fixture_file_is_the_one_recorded():
    import hashlib
    d, _, _ = _fixture()
    assert hashlib.sha256(open(os.path.join(GOLD, "mesh_small.3d"), "rb").read()).hexdigest() == d["file_sha256"]


def test_load_3d_is_the_reference_reader():
    _, v, i = _fixture()
    V, F = scenes.load_3d(os.path.join(GOLD, "mesh_small.3d"))
    assert V.dtype == np.float32 and np.array_equal(V.view(np.uint32), v.view(np.uint32))
    assert np.array_equal(F, i)


def test_cpp_plyinfo_is_the_reference_reader():
    _, v, i = _fixture()
    V, F = _cpp("ply3d", os.path.join(GOLD, "mesh_small.3d"))
    assert np.array_equal(V.view(np.uint32), v.view(np.uint32)) and np.array_equal(F, i)


def test_3d_scale_is_x20():
    toks = open(os.path.join(GOLD, "mesh_small.3d")).read().split()
    raw = np.array(toks[4:4 + 3 * 64], dtype=np.float32).reshape(-1, 3)
    _, v, _ = _fixture()
    assert np.array_equal(v, raw * np.float32(20))


# a small mesh with a quad and a pentagon, plus per-vertex normals and a colour property
VERTS = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0.5, 1.5, 0.25], [2, 0.5, -1]], np.float32)
FACES = [[0, 1, 2, 3], [1, 5, 2], [3, 2, 4, 0, 5]]
EXPECT = np.array([[0, 1, 2], [0, 2, 3], [1, 5, 2], [3, 2, 4], [3, 4, 0], [3, 0, 5]], np.int32)


def _write_ply(path, binary):
    hdr = ["ply", "format binary_little_endian 1.0" if binary else "format ascii 1.0", "comment test mesh",
           f"element vertex {len(VERTS)}", "property float x", "property float y", "property float z",
           "property float nx", "property float ny", "property float nz", "property uchar red",
           f"element face {len(FACES)}", "property list uchar int vertex_indices", "end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(hdr) + "\n").encode())
        for k, p in enumerate(VERTS):
            n = (0.0, 0.0, 1.0)
            if binary:
                f.write(struct.pack("<6fB", *p, *n, k * 10))
            else:
                f.write((" ".join(repr(float(c)) for c in p) + " 0 0 1 %d\n" % (k * 10)).encode())
        for face in FACES:
            if binary:
                f.write(struct.pack("<B%di" % len(face), len(face), *face))
            else:
                f.write((" ".join(str(c) for c in [len(face)] + face) + "\n").encode())


@pytest.mark.parametrize("binary", [False, True])
def test_load_ply_formats(tmp_path, binary):
    path = str(tmp_path / ("m_bin.ply" if binary else "m_ascii.ply"))
    _write_ply(path, binary)
    V, F = scenes.load_ply(path)
    assert np.array_equal(V, VERTS)   # PLY vertices are not scaled
    assert np.array_equal(F, EXPECT)
    Vc, Fc = _cpp("ply", path)
    assert np.array_equal(Vc, VERTS) and np.array_equal(Fc, EXPECT)


def test_loaded_mesh_renders_like_its_arrays():
    """A .3d mesh through the scene API builds the same BVH as the arrays it holds."""
    import oracle_lib
    V, F = scenes.load_3d(os.path.join(GOLD, "mesh_small.3d"))
    s1, _ = scenes.config_c2(16, 8, 1, mesh=(V, F, "mesh_small.3d"))
    s2, _ = scenes.config_c2(16, 8, 1, mesh=(V.copy(), F.copy(), "copy"))
    n1, i1 = oracle_lib.build_bvh(s1)
    n2, i2 = oracle_lib.build_bvh(s2)
    assert np.array_equal(n1, n2) and np.array_equal(i1, i2)


def test_real_dragon_file_is_picked_up(tmp_path, monkeypatch):
    """PBR_DRAGON_PLY names the real Stanford Dragon (.ply, or the reference's .3d): the BASELINE
    configs then load it instead of the stand-in and say so in scene.info."""
    path = str(tmp_path / "dragon.ply")
    _write_ply(path, True)
    monkeypatch.setenv("PBR_DRAGON_PLY", path)
    s, _ = scenes.config_c2(8, 8, 1)
    assert s.info["dragon"] == path and s.info["triangles"] == len(EXPECT)
    monkeypatch.setenv("PBR_DRAGON_PLY", os.path.join(GOLD, "mesh_small.3d"))
    s, _ = scenes.config_c3(8, 8, 1)
    assert s.info["triangles"] == 110
