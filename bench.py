"""Headline benchmark: Msamples/s of the MI355X render path on BASELINE config C2
(1920×1080, 64 spp, WhittedIntegrator, dragon + mirror floor + SkyBox HDR), with the roofline of the
dominant kernel and the CPU restatement timed beside it.

One step = one full frame.  With --gpus N (launched by torch.distributed.run, one rank per GPU)
the frame's 32×32 tiles are dealt round-robin over ranks and rank 0 gathers the per-tile RGBA8
FrameBuffer spans over RCCL — total work is fixed, so scaling is strong.  The gather of frame k
runs on a communication stream while frame k+1 renders into the other of two output buffers.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from pysicalbasedraytracer_amd import FrameGather, HipRenderer, scenes, tiles_for_rank  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Algorithmic bytes model: 32 B per LinearBVHNode test, 48 B per primitive test,
# 96 B of ray-queue traffic per traced ray, 64 B per shading event.  The counts come from an
# instrumented pass that counts tests exactly as BVHAccel performs them (pbr_device.h traverse).
B_NODE, B_PRIM, B_RAY, B_SHADE = 32, 48, 96, 64
# rocprofv3 PMC HBM bytes per frame (tools/pmc.sh + tools/summarize_prof.py --json=...); used only
# when it was measured on the very build that is loaded (source hash from pbr_hip_build_info).
TRAFFIC_JSON = os.path.join(ROOT, "profiles", "c2_traffic.json")


def pmc_traffic(build_info):
    try:
        t = json.load(open(TRAFFIC_JSON))
    except (OSError, ValueError):
        return None, "no PMC summary"
    if not t.get("build") or not build_info.endswith(t["build"]):
        return None, f"PMC summary is for build {t.get('build')}, not this one"
    return t["frame_read_bytes"] + t["frame_write_bytes"], f"{os.path.relpath(TRAFFIC_JSON, ROOT)} ({t['method']})"


def cpu_baseline(scene, rd, budget_s=12.0):
    """Oracle (CPU restatement, the reference algorithm) on the host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    W, H, spp = rd.camera.width, rd.camera.height, rd.spp
    rows_per_chunk = 24
    done_px = 0
    secs = 0.0
    y = 0
    while secs < budget_s and y < H:          # top-down row bands until the budget or the frame ends
        y1 = min(H, y + rows_per_chunk)
        rdc = scenes.render_desc(rd.camera, rd.integrator, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                                 rd.sampler, tiles=[(0, y, W, y1)])
        _, _, sec = oracle_lib.render(scene, rdc, threads=threads)
        secs += sec
        done_px += W * (y1 - y)
        y = y1
    samples = done_px * spp
    return {"value": samples / secs / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"C2 rows [0,{y}) × {W} px × {spp} spp = {samples} samples in {secs:.1f} s "
                      f"(oracle/ CPU restatement, OpenMP dynamic schedule)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    scene, rd = scenes.CONFIGS[args.config]()
    W, H, spp = rd.camera.width, rd.camera.height, rd.spp
    tiles = tiles_for_rank(W, H, rank, world) if world > 1 else [(0, 0, W, H)]
    rdr = scenes.render_desc(rd.camera, rd.integrator, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                             rd.sampler, tiles=tiles)
    npx = sum((t[2] - t[0]) * (t[3] - t[1]) for t in tiles)

    r = HipRenderer(local)
    build_info = r.lib.pbr_hip_build_info().decode()
    t0 = time.time()
    r.upload(scene)
    upload_s = time.time() - t0

    # a real stream (torch's default one has handle 0, which the C-ABI reads as "context stream")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    # multi-GPU: rank 0 gathers the packed RGBA8 tile spans (the FrameBuffer the reference's Render
    # fills) over RCCL and scatters them into the frame; double-buffered outputs let the gather of
    # frame k (communication stream) overlap the render of frame k+1 (render stream)
    nbuf = 2 if world > 1 else 1
    rgbs = [torch.empty((npx, 3), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    rgbas = [torch.empty((npx, 4), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    exchange = FrameGather(W, H, world, dev, channels=4, dtype=torch.uint8) if world > 1 else None
    comm = torch.cuda.Stream(dev) if world > 1 else None
    released = [None] * nbuf   # event: the gather that read buffer b has finished
    frame_no = [0]

    def render(ev0=None, ev1=None):
        b = frame_no[0] % nbuf
        frame_no[0] += 1
        if released[b] is not None:
            stream.wait_event(released[b])
        if ev0 is not None:
            ev0.record(stream)
        # asynchronous: the frame is enqueued on `stream` and the next one queues behind it
        r.render_device(rdr, rgbs[b].data_ptr(), rgbas[b].data_ptr(), stream=stream.cuda_stream, sync=False)
        if ev1 is not None:
            ev1.record(stream)
        if exchange is not None:
            rendered = torch.cuda.Event()
            rendered.record(stream)
            comm.wait_event(rendered)
            with torch.cuda.stream(comm):
                exchange(rgbas[b], rank)
                done = torch.cuda.Event()
                done.record(comm)
            released[b] = done

    # roofline counters: one instrumented, untimed pass on the same workload
    st = r.render_device(rdr, rgbs[0].data_ptr(), rgbas[0].data_ptr(), stream=stream.cuda_stream, stats=True)
    torch.cuda.synchronize(dev)
    samples_rank = npx * spp
    alg_bytes = B_NODE * st.node_visits + B_PRIM * st.prim_tests + B_RAY * st.rays + B_SHADE * st.shading_events

    for _ in range(args.warmup):
        render()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # HIP events bracket each frame's launches on the render stream; read after the final sync
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for ev0, ev1 in evs:
        render(ev0, ev1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kernel_ms = [ev0.elapsed_time(ev1) for ev0, ev1 in evs]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # roofline over the whole job: every rank's algorithmic bytes over the slowest rank's frame
        ab = torch.tensor([float(alg_bytes)], dtype=torch.float64, device=dev)
        dist.all_reduce(ab, op=dist.ReduceOp.SUM)
        km = torch.tensor([float(np.mean(kernel_ms))], dtype=torch.float64, device=dev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        alg_bytes, kernel_ms, samples_rank = float(ab.item()), [float(km.item())], W * H * spp
    ms_per_step = elapsed / args.steps * 1e3
    total_samples = W * H * spp
    value = total_samples / (elapsed / args.steps) / 1e6

    if rank == 0:
        k_ms = float(np.mean(kernel_ms))
        achieved = alg_bytes / (k_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(build_info) if (world == 1 and args.config == "C2") else (None, "C2, 1 GPU only")
        out = {
            "metric": "Msamples/sec (whole node) + wall-clock to 1080p/64spp frame; %HBM roofline",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.config}: {W}x{H}, {spp} spp, "
                                   f"{['Whitted', 'Path', 'VolPath'][rd.integrator]} d{rd.max_depth}",
                       "scene": scene.info.get("dragon", ""), "triangles": scene.info.get("triangles"),
                       "parallelism": f"tiles32x32 round-robin over {world} GPU(s), RCCL gather of RGBA8 spans",
                       "frame_ms": round(ms_per_step, 3), "scene_upload_s": round(upload_s, 3)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         # measured HBM bytes over the same frame time: what HBM actually moved
                         # (the algorithmic bytes include BVH/mesh fetches that L2 and the
                         # Infinity Cache serve, which is how `frac` can exceed 1)
                         "traffic_gbs": None if traffic is None else round(traffic / (k_ms * 1e-3) / 1e9, 1),
                         "traffic_frac": None if traffic is None else round(traffic / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "kernel": ["wavefront frame: k_wf_camera_extend, (k_wf_shade, k_wf_shadow, k_wf_extend) per "
                                    "level, k_wf_finish, per 2^25-sample chunk",
                                    "wavefront frame: k_wfp_camera_extend, (k_wfp_shade, k_wfp_shadow, k_wfp_probe, "
                                    "k_wfp_resolve, k_wf_extend) per bounce, k_wfp_finish, per 2^25-sample chunk",
                                    "wavefront frame: k_wfp_camera_extend, (k_wfv_shade, k_wfv_tr, k_wfp_probe, "
                                    "k_wfv_resolve, k_wf_extend) per bounce, k_wfp_finish, per 2^25-sample chunk"][rd.integrator],
                         "kernel_ms": round(k_ms, 3),
                         "bytes_per_sample": round(alg_bytes / samples_rank, 1),
                         "model": "per sample: 32*node_tests + 48*prim_tests + 96*rays + 64*shading_events "
                                  "(SURVEY 8(d)); counts from an instrumented pass over this frame",
                         "note": "frac counts every BVH-node and triangle fetch as HBM bytes (the SURVEY 8(d) "
                                 "model), but the 10 MB BVH + mesh are served by L2, the Infinity Cache and the "
                                 "scalar cache, so frac can exceed 1; traffic_frac is the measured HBM fraction",
                         "build": build_info},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, rd)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
