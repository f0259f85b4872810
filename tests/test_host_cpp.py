"""The C++ host API (include/pbr/pbr.h), driven like the reference's Main/main.cpp, in a compiled
test program (tests/cpp/host_api_test.cpp) that checks it against the oracle."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "pysicalbasedraytracer_amd", "host")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpp")], check=True)
    return os.path.join(HERE, "cpp", "host_api_test")


def _run(mode, timeout):
    exe = _build()
    p = subprocess.run([exe, mode], capture_output=True, text=True, timeout=timeout)
    print(p.stdout)
    assert p.returncode == 0, p.stdout + p.stderr


def test_host_api_cpu():
    """Scene building + flattening, the oracle on the flattened scene, and Render failing loudly
    without a device."""
    if os.path.exists("/dev/kfd") and os.environ.get("PBR_EXPECT_NO_GPU") is None:
        pytest.skip("a GPU is present: the no-device check does not apply")
    _run("cpu", 120)


def _decode_png(path):
    """Minimal PNG reader (8-bit, non-interlaced, all five filter types) for the round trip."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        assert struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0] == zlib.crc32(typ + body)
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    assert depth == 8 and interlace == 0
    comp = {0: 1, 4: 2, 2: 3, 6: 4}[ctype]
    raw = zlib.decompress(idat)
    stride = w * comp
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f, line = raw[y * (stride + 1)], np.frombuffer(raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)], np.uint8).astype(np.int32)
        cur = np.zeros(stride, np.int32)
        for i in range(stride):
            a = cur[i - comp] if i >= comp else 0
            b = prev[i]
            c = prev[i - comp] if i >= comp else 0
            p = a + b - c
            pred = [0, a, b, (a + b) // 2,
                    a if abs(p - a) <= abs(p - b) and abs(p - a) <= abs(p - c) else (b if abs(p - b) <= abs(p - c) else c)][f]
            cur[i] = (line[i] + pred) & 255
        out[y], prev = cur, cur
    return out.reshape(h, w, comp)


def test_png_output_stage(tmp_path):
    """main.cpp's save: stbi_flip_vertically_on_write(true) + stbi_write_png of the FrameBuffer
    (main.cpp:419-429), and FrameBuffer::update_f_u_c (FrameBuffer.h:112-126) — CPU only."""
    exe = _build()
    png = str(tmp_path / "fb.png")
    p = subprocess.run([exe, "png", png], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stdout + p.stderr
    W, H = 37, 23
    buf = np.fromfile(png + ".raw", np.uint8).reshape(H, W, 4)
    y, x, c = np.meshgrid(np.arange(H), np.arange(W), np.arange(4), indexing="ij")
    expect = ((x * 7 + y * 13 + c * 29) & 255).astype(np.uint8)
    expect[6, 5, 1] = np.uint8(np.float32(0.5) * 255)   # the running average of .25, .5, .75
    assert np.array_equal(buf, expect)
    assert np.array_equal(_decode_png(png), buf[::-1])   # written bottom row first


@pytest.mark.gpu
def test_host_api_gpu_matches_oracle():
    """Whitted / Path / VolPath rendered through the C++ API match the oracle (L∞ ≤ 1e-3, u8 ≤ 1)."""
    _run("gpu", 600)


@pytest.mark.parametrize("W,H,world", [(1920, 1080, 8), (1920, 1080, 3), (77, 45, 2), (31, 5, 4)])
def test_cpp_tile_partition_matches_python(W, H, world):
    """The C++ multi-GPU Render deals the same tiles to the same ranks as bench.py's ranks."""
    import sys
    sys.path.insert(0, ROOT)
    from pysicalbasedraytracer_amd import tiles_for_rank
    exe = _build()
    out = subprocess.run([exe, "tiles", str(W), str(H), str(world)], capture_output=True, text=True, check=True).stdout
    cpp = [tuple(int(v) for v in line.split()) for line in out.splitlines()]
    py = [(r,) + tuple(t) for r in range(world) for t in tiles_for_rank(W, H, r, world)]
    assert cpp == py
