"""pbr_hip_render_frames: n frames of one descriptor in one call, their chunks continuing one rotation
over the lanes with no join between frames (bench.py's timed window).  Every frame of a batch is the
same bits as pbr_hip_render's single frame, under the default schedule, many small chunks, one-chunk
frames (a multi-GPU rank's shard), the serial schedule and the megakernel; pbr_hip_wait_frame orders
another stream after one frame of the batch."""
import numpy as np
import pytest
import torch

from pysicalbasedraytracer_amd import HipRenderer, capi, scenes, tiles_for_rank

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    r = HipRenderer(0)
    yield r
    r.close()


def small_dragon(n=40):
    P, I = scenes.dragon_standin(n=n)
    return P, I, "standin-small"


SCENES = {
    "whitted": lambda: scenes.config_c2(128, 72, 8, mesh=small_dragon(48), sky=scenes.procedural_sky(128, 64)),
    "path": lambda: scenes.config_c4(96, 54, 8, mesh=small_dragon(40)),
    "volpath": lambda: scenes.config_c5(80, 45, 8, mesh=small_dragon(40)),
}
SCHEDULES = {
    "default": {},
    "chunks_3_lanes": {"chunk_log2": 12},
    "chunks_2_lanes": {"chunk_log2": 11, "lanes": 2},
    "serial": {"chunk_log2": 12, "serial": True},
    "megakernel": {"kernels": capi.KERNELS_MEGAKERNEL},
}


def batch(hip, rd, npx, n, stream):
    dev = torch.device("cuda", 0)
    rgbs = [torch.full((npx, 3), float("nan"), dtype=torch.float32, device=dev) for _ in range(n)]
    rgbas = [torch.zeros((npx, 4), dtype=torch.uint8, device=dev) for _ in range(n)]
    hip.render_frames(rd, [t.data_ptr() for t in rgbs], [t.data_ptr() for t in rgbas], stream=stream.cuda_stream)
    return rgbs, rgbas


@pytest.mark.parametrize("sched", sorted(SCHEDULES))
@pytest.mark.parametrize("kind", sorted(SCENES))
def test_batch_frames_equal_single_frames(hip, kind, sched):
    s, rd = SCENES[kind]()
    npx = rd.camera.width * rd.camera.height
    hip.upload(s)
    hip.set_schedule(**SCHEDULES[sched])
    ref, ref8, _ = hip.render(rd)
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    rgbs, rgbas = batch(hip, rd, npx, 3, stream)
    hip.sync()
    torch.cuda.synchronize()
    for f in range(3):
        g = rgbs[f].cpu().numpy()
        assert np.array_equal(g.view(np.uint32), ref.reshape(npx, 3).view(np.uint32)), f"frame {f}"
        assert np.array_equal(rgbas[f].cpu().numpy(), ref8.reshape(npx, 4)), f"frame {f}"
    hip.set_schedule()


def test_batch_of_rank_shards(hip):
    """One-chunk frames — rank 1 of a 4-GPU job's 32x32 tiles — rotate over the lanes frame by frame."""
    s, rd = SCENES["whitted"]()
    W, H = rd.camera.width, rd.camera.height
    tiles = tiles_for_rank(W, H, 1, 4, 32)
    d = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                           rd.sampler, tiles=tiles)
    npx = sum((t[2] - t[0]) * (t[3] - t[1]) for t in tiles)
    hip.upload(s)
    ref, ref8, _ = hip.render(d)
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    rgbs, rgbas = batch(hip, d, npx, 4, stream)
    hip.sync()
    for f in range(4):
        assert np.array_equal(rgbs[f].cpu().numpy().view(np.uint32), ref.reshape(npx, 3).view(np.uint32))
        assert np.array_equal(rgbas[f].cpu().numpy(), ref8.reshape(npx, 4))


def test_wait_frame_orders_another_stream(hip):
    s, rd = SCENES["path"]()
    npx = rd.camera.width * rd.camera.height
    hip.upload(s)
    hip.set_schedule(chunk_log2=12)
    ref, _, _ = hip.render(rd)
    dev = torch.device("cuda", 0)
    stream, other = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    rgbs, _ = batch(hip, rd, npx, 3, stream)
    copies = []
    for f in range(3):   # each copy on `other` runs after its frame, whatever the rest of the batch does
        hip.wait_frame(other.cuda_stream, f)
        with torch.cuda.stream(other):
            copies.append(rgbs[f].clone())
    other.synchronize()
    hip.sync()
    for c in copies:
        assert np.array_equal(c.cpu().numpy().view(np.uint32), ref.reshape(npx, 3).view(np.uint32))
    hip.set_schedule()


def test_batch_refusals(hip):
    s, rd = SCENES["whitted"]()
    hip.upload(s)
    with pytest.raises(RuntimeError):
        hip.wait_frame(None, 10**6)
    rd.outputs_on_device = 0
    import ctypes as C
    rc = hip.lib.pbr_hip_render_frames(hip.ctx, C.byref(rd), 0, None, None)
    assert rc == capi.PBR_E_INVALID


def test_batch_of_frames_at_the_chunk_cap_bounds_lane_memory(hip):
    """A one-chunk Path frame of 2^26 samples (256x256 at 1024 spp, ≈ 24 GB of lane buffers): a batch
    rotates such frames over as many lanes as fit the lane budget (lane_budget: 3/4 of the device memory
    free or held by the context).  With the device to itself the batch keeps its three lanes; with all
    but ~60 GB taken by another allocation it keeps two and still renders the single call's bits."""
    s, rd = scenes.config_c4(256, 256, 1024, mesh=small_dragon(40))
    npx = 256 * 256
    hip.upload(s)
    hip.set_schedule()
    ref, ref8, _ = hip.render(rd)   # one lane
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    free0, _ = torch.cuda.mem_get_info(0)
    hog = torch.empty(max(0, int(free0 - 60e9)), dtype=torch.uint8, device="cuda")
    free1, _ = torch.cuda.mem_get_info(0)
    rgbs, rgbas = batch(hip, rd, npx, 3, stream)
    hip.sync()
    torch.cuda.synchronize()
    used = (free1 - torch.cuda.mem_get_info(0)[0]) / 1e9
    print(f"free before the batch {free1 / 1e9:.1f} GB; lane buffers + outputs added by it: {used:.1f} GB")
    assert used < 0.75 * free1 / 1e9 + 1, f"{used:.1f} GB: the batch kept more lanes than the budget allows"
    for f in range(3):
        assert np.array_equal(rgbs[f].cpu().numpy().view(np.uint32), ref.reshape(npx, 3).view(np.uint32)), f"frame {f}"
        assert np.array_equal(rgbas[f].cpu().numpy(), ref8.reshape(npx, 4)), f"frame {f}"
    del hog
    torch.cuda.empty_cache()
