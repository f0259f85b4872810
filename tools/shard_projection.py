"""Multi-GPU projection on one GPU: the frame time of every rank's shard of an N-GPU tile-sharded
job (bench.py's partition: 32x32 tiles dealt round-robin, tiles_for_rank), rendered one after the
other on this GPU, for N = 1, 2, 4, 8.  The job's frame is its slowest rank (plus the gather, which
bench.py overlaps with the next frame); the projected speed-up is the whole frame / slowest rank.

    python tools/shard_projection.py --config C4 [--steps 1] [--json out.json]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes, tiles_for_rank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--json", default=None)
    ap.add_argument("--schedule", default="", help="pbr_hip_set_schedule for every render: comma-separated "
                                                     "kernels=mega, chunk_log2=N, lanes=N, fuse=on|off (tune_wavefront.py)")
    ap.add_argument("--lib", default=None, help="an experimental build of libpbr_hip.so")
    ap.add_argument("--batch", type=int, default=5, help="frames per pbr_hip_render_frames batch, as bench.py's "
                                                         "timed window (0: one pbr_hip_render per frame)")
    a = ap.parse_args()
    if a.lib:
        capi._lib = capi.load_library(a.lib)
    scene, rd = scenes.CONFIGS[a.config]()
    W, H, spp = rd.camera.width, rd.camera.height, rd.spp
    r = HipRenderer(0)
    r.upload(scene)
    kw = dict(kv.split("=") for kv in a.schedule.split(",") if kv)
    r.set_schedule(kernels=capi.KERNELS_MEGAKERNEL if kw.get("kernels") == "mega" else capi.KERNELS_AUTO,
                   chunk_log2=int(kw.get("chunk_log2", 0)), lanes=int(kw.get("lanes", 0)),
                   fuse_camera={"on": capi.FUSE_ON, "off": capi.FUSE_OFF}.get(kw.get("fuse"), capi.FUSE_AUTO))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    nb = max(1, a.batch)
    rgbs = [torch.empty((W * H, 3), dtype=torch.float32, device=dev) for _ in range(nb)]
    rgbas = [torch.empty((W * H, 4), dtype=torch.uint8, device=dev) for _ in range(nb)]

    def timed(desc):
        r.render_device(desc, rgbs[0].data_ptr(), rgbas[0].data_ptr(), stream=stream.cuda_stream)   # warm-up / tile upload
        torch.cuda.synchronize(dev)
        ms = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            if a.batch > 0:   # bench.py's window: frames of one batch overlap on the lanes
                r.render_frames(desc, [t.data_ptr() for t in rgbs], [t.data_ptr() for t in rgbas], stream=stream.cuda_stream)
                r.sync()
            else:
                r.render_device(desc, rgbs[0].data_ptr(), rgbas[0].data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            ms.append((time.perf_counter() - t0) * 1e3 / nb)
        return sorted(ms)[len(ms) // 2]

    full = timed(rd)
    out = {"config": a.config, "raster": [W, H], "spp": spp, "tile": a.tile, "full_ms": round(full, 3), "batch": a.batch,
           "schedule": a.schedule or "default",
           "build": capi.load_library().pbr_hip_build_info().decode(), "ranks": {}}
    print(f"{a.config} whole frame {full:.2f} ms", flush=True)
    for n in (int(x) for x in a.ns.split(",")):
        per = []
        for k in range(n):
            tiles = tiles_for_rank(W, H, k, n, a.tile)
            d = scenes.render_desc(rd.camera, rd.integrator, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                                   rd.sampler, tiles=tiles)
            per.append(timed(d))
        slow = max(per)
        out["ranks"][str(n)] = {"ms": [round(x, 3) for x in per], "slowest_ms": round(slow, 3),
                                "ideal_ms": round(full / n, 3), "speedup": round(full / slow, 3)}
        print(f"{a.config} N={n}: ranks {min(per):.2f}-{slow:.2f} ms, ideal {full / n:.2f} ms, "
              f"speed-up {full / slow:.2f}x", flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
