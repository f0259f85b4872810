"""Shared parity assertions for the device-vs-oracle tests.

Floating point: per-pixel L∞ on linear RGB within north_star's 1e-3.  Bytes: the 8-bit output is a
pure function of the pixel's float sum (Integrator.cpp:327-344 on both sides), so wherever the
float pixel is bit-identical the RGBA8 pixel must be identical too; only pixels whose floats differ
may differ by one 8-bit step."""
import numpy as np

LINF = 1e-3


def assert_u8(gpu_rgb, cpu_rgb, gpu8, cpu8):
    same = np.all(gpu_rgb.reshape(gpu_rgb.shape[0], -1).view(np.uint32) ==
                  cpu_rgb.reshape(cpu_rgb.shape[0], -1).view(np.uint32), axis=1)
    g8 = gpu8.reshape(gpu8.shape[0], -1).astype(int)
    c8 = cpu8.reshape(cpu8.shape[0], -1).astype(int)
    assert np.array_equal(g8[same], c8[same]), "8-bit output differs where the float pixel is bit-identical"
    if (~same).any():
        assert np.abs(g8[~same] - c8[~same]).max() <= 1
    return float(same.mean()) if same.size else 1.0


def assert_parity(gpu_rgb, cpu_rgb, gpu8=None, cpu8=None, linf=LINF):
    """Returns (L∞, fraction of bit-identical pixels)."""
    gpu_rgb = np.asarray(gpu_rgb, np.float32)
    cpu_rgb = np.asarray(cpu_rgb, np.float32)
    assert gpu_rgb.shape == cpu_rgb.shape
    assert np.isfinite(gpu_rgb).all()
    d = np.abs(gpu_rgb.astype(np.float64) - cpu_rgb.astype(np.float64))
    m = float(np.nanmax(d)) if d.size else 0.0
    exact = float(np.mean(np.all(gpu_rgb.reshape(gpu_rgb.shape[0], -1).view(np.uint32) ==
                                 cpu_rgb.reshape(cpu_rgb.shape[0], -1).view(np.uint32), axis=1))) if d.size else 1.0
    assert m <= linf, f"per-pixel L∞ {m} > {linf} (bit-exact pixels {exact:.4f})"
    if gpu8 is not None:
        assert_u8(gpu_rgb, cpu_rgb, gpu8, cpu8)
    return m, exact
