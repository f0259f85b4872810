"""Dense parity of the BENCHMARKED frames, through the path bench.py times (bench.py `frames`):
the BASELINE configs' own scenes (scenes.CONFIGS) rendered as one pbr_hip_render_frames batch of two
frames, asynchronously into device buffers on a caller stream, under the default schedule (chunks
over three lanes, the fused level-0 Whitted shade, the classed Path/VolPath shades) — then compared
with the oracle (the CPU restatement of SamplerIntegrator::Render, Integrator.cpp:286-344):

- C2 (1920x1080, 64 spp, Whitted): EVERY pixel, float colObj/spp and RGBA8, bit for bit;
- C3 (Sobol), C4 (3840x2160x1024) and C5: a seeded 1/64 of the pixels plus both pixels either side
  of every chunk boundary of the default schedule (where one lane's chunk hands over to the next),
  float colObj/spp and RGBA8 bit for bit (the share is printed: profiles/r6_gpu_tests.log);
- the batch's second frame equal to the first over the whole raster, bit for bit.

The oracle renders the picked pixels as one-pixel tiles at the full raster and spp, so their sample
indices are the benchmarked ones (Halton.cpp:61-81; pbrt-v3's SobolSampler for C3).  On the GPU box
the oracle takes ~10-40 s per config on its 16 cores."""
import time

import numpy as np
import pytest
import torch

import oracle_lib as O
from parity import assert_parity
from ref_scenes import default_chunk_starts
from pysicalbasedraytracer_amd import HipRenderer, scenes

pytestmark = pytest.mark.gpu

# share of the picked pixels bit-identical to the oracle: every one (round 6, profiles/r6_gpu_tests.log:
# C3 32,416, C4 129,850 and C5 32,432 pixels, all bit-identical, L∞ 0)
MIN_EXACT = {"C3": 1.0, "C4": 1.0, "C5": 1.0}


@pytest.fixture(scope="module")
def hip():
    r = HipRenderer(0)
    yield r
    r.close()


def bench_batch(hip, config, nframes=2):
    """bench.py's timed window for one config: an nframes batch on a caller stream, device outputs."""
    s, rd = scenes.CONFIGS[config]()
    W, H = rd.camera.width, rd.camera.height
    full = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                              rd.sampler, tiles=[(0, 0, W, H)])
    hip.upload(s)
    hip.set_schedule()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    rgbs = [torch.full((W * H, 3), float("nan"), dtype=torch.float32, device=dev) for _ in range(nframes)]
    rgbas = [torch.zeros((W * H, 4), dtype=torch.uint8, device=dev) for _ in range(nframes)]
    t0 = time.time()
    hip.render_frames(full, [t.data_ptr() for t in rgbs], [t.data_ptr() for t in rgbas], stream=stream.cuda_stream)
    hip.sync()
    stream.synchronize()
    gpu_s = time.time() - t0
    return s, rd, rgbs, rgbas, gpu_s


def picked_pixels(W, H, rd, seed):
    """A seeded 1/64 of the packed (row-major) pixels, plus both sides of every chunk boundary."""
    n = W * H
    rng = np.random.default_rng(seed)
    picks = set(rng.choice(n, n // 64, replace=False).tolist())
    for p0 in default_chunk_starts(n, rd.spp, rd.integrator, rd.max_depth)[1:]:
        picks.update((p0 - 1, p0))
    picks.update((0, n - 1))
    return np.array(sorted(picks), dtype=np.int64)


def test_c2_whole_frame_batch_equals_oracle(hip):
    s, rd, rgbs, rgbas, gpu_s = bench_batch(hip, "C2")
    W, H = rd.camera.width, rd.camera.height
    assert len(default_chunk_starts(W * H, rd.spp, rd.integrator, rd.max_depth)) == 4   # 4 chunks, 3 lanes, fused level 0
    t0 = time.time()
    c, c8, _ = O.render(s, scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold,
                                              rd.light_strategy, rd.sampler, tiles=[(0, 0, W, H)]))
    cpu_s = time.time() - t0
    for f in range(2):
        g = rgbs[f].cpu().numpy()
        g8 = rgbas[f].cpu().numpy()
        diff = np.flatnonzero(np.any(g.view(np.uint32) != c.view(np.uint32), axis=1))
        linf = float(np.abs(g.astype(np.float64) - c).max())
        print(f"C2 frame {f}: {W * H} px, {diff.size} float pixels differ (L∞ {linf:.3g}); GPU batch {gpu_s:.2f} s, "
              f"oracle {cpu_s:.1f} s")
        assert diff.size == 0, f"frame {f}: {diff.size} pixels differ from the oracle, first {diff[:5]}"
        assert np.array_equal(g8, c8), f"frame {f}: RGBA8 differs from the oracle"


@pytest.mark.parametrize("config,seed", [("C3", 3), ("C4", 4), ("C5", 5)])
def test_path_volpath_bench_batch_matches_oracle(hip, config, seed):
    s, rd, rgbs, rgbas, gpu_s = bench_batch(hip, config)
    W, H = rd.camera.width, rd.camera.height
    g0 = rgbs[0].cpu().numpy()
    assert np.isfinite(g0).all() and (g0 >= 0).all()
    # the batch's frames are the same bits (the classed shades reorder queue entries across launches)
    assert np.array_equal(rgbs[1].cpu().numpy().view(np.uint32), g0.view(np.uint32))
    assert torch.equal(rgbas[1], rgbas[0])
    picks = picked_pixels(W, H, rd, seed)
    tiles = [(int(p % W), int(p // W), int(p % W) + 1, int(p // W) + 1) for p in picks]
    rdt = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                             rd.sampler, tiles=tiles)
    t0 = time.time()
    c, c8, _ = O.render(s, rdt)
    cpu_s = time.time() - t0
    g8 = rgbas[0].cpu().numpy()
    linf, exact = assert_parity(g0[picks], c, g8[picks], c8)
    print(f"{config}: {picks.size} px ({picks.size / (W * H):.4f} of the frame) x {rd.spp} spp, L∞ {linf:.3g}, "
          f"bit-identical {exact:.5f}; GPU batch of 2 {gpu_s:.2f} s, oracle {cpu_s:.1f} s")
    assert exact >= MIN_EXACT[config], f"{config}: only {exact:.5f} of the picked pixels bit-identical to the oracle"
