"""Multi-GPU path on the CPU: world size 2 over gloo.  Each rank renders its round-robin 32×32
tiles (here with the oracle, standing in for the device) and `gather_frame` — the same exchange
bench.py runs over RCCL — must reassemble the single-process frame bit for bit."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    import oracle_lib
    from pysicalbasedraytracer_amd import gather_frame, scenes, tiles_for_rank
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    scene, rd = scenes.config_c1(150, 100, 2)
    W, H = rd.camera.width, rd.camera.height
    tiles = tiles_for_rank(W, H, rank, world)
    rdr = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, tiles=tiles)
    rgb, rgba, _ = oracle_lib.render(scene, rdr, threads=2)
    frame = gather_frame(torch.from_numpy(rgb), W, H, rank, world)
    # the RGBA8 FrameBuffer spans (what bench.py gathers over RCCL)
    frame8 = gather_frame(torch.from_numpy(np.ascontiguousarray(rgba.reshape(-1, 4))), W, H, rank, world)
    if rank == 0:
        np.save(out_path, frame)
        np.save(out_path + ".u8.npy", frame8)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tile_gather_reassembles_frame(tmp_path):
    import oracle_lib
    from pysicalbasedraytracer_amd import scenes, tiles_for_rank
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    frame = np.load(out)
    scene, rd = scenes.config_c1(150, 100, 2)
    full, full8, _ = oracle_lib.render(scene, rd, threads=2)
    assert np.array_equal(frame.reshape(-1, 3).view(np.uint32), full.view(np.uint32))
    assert np.array_equal(np.load(out + ".u8.npy").reshape(-1, 4), full8.reshape(-1, 4))
    # both ranks own work and no tile is dealt twice
    t0, t1 = tiles_for_rank(150, 100, 0, 2), tiles_for_rank(150, 100, 1, 2)
    assert t0 and t1 and not set(t0) & set(t1)


def _gpu_worker(rank, world, port, out_path):
    """bench.py's per-rank leg on the device: render this rank's tiles into device buffers
    (render_device, the asynchronous path bench.py times), then FrameGather the RGBA8 and float
    spans to rank 0 — here over gloo with host copies, both ranks sharing the one GPU."""
    import torch
    import torch.distributed as dist
    from pysicalbasedraytracer_amd import FrameGather, HipRenderer, scenes, tiles_for_rank
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    scene, rd = scenes.config_c2(200, 120, 4, mesh=scenes.dragon_standin(n=40) + ("standin-40",),
                                 sky=scenes.procedural_sky(64, 32))
    W, H = rd.camera.width, rd.camera.height
    tiles = tiles_for_rank(W, H, rank, world)
    rdr = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, tiles=tiles)
    r = HipRenderer(0)
    r.upload(scene)
    dev = torch.device("cuda", 0)
    npx = sum((x1 - x0) * (y1 - y0) for (x0, y0, x1, y1) in tiles)
    rgb = torch.empty((npx, 3), dtype=torch.float32, device=dev)
    rgba = torch.empty((npx, 4), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    r.render_device(rdr, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream, sync=False)
    torch.cuda.synchronize(dev)
    f32 = FrameGather(W, H, world, torch.device("cpu"))(rgb.cpu(), rank)
    f8 = FrameGather(W, H, world, torch.device("cpu"), channels=4, dtype=torch.uint8)(rgba.cpu(), rank)
    if rank == 0:
        full, full8, _ = r.render(rd)
        np.save(out_path, np.stack([np.array_equal(f32.numpy().view(np.uint32), full.view(np.uint32)),
                                    np.array_equal(f8.numpy(), full8)]))
    r.close()
    dist.barrier()
    dist.destroy_process_group()


@__import__("pytest").mark.gpu
def test_two_rank_device_render_gather_equals_one_render(tmp_path):
    out = str(tmp_path / "ok.npy")
    mp.spawn(_gpu_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert np.load(out).all()
