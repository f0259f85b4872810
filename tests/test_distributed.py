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
