"""Time one config under several schedules on one GPU (frames must stay bit-identical across them).

    python tools/tune_wavefront.py [--config C2] [--steps 3] [--profile] "" "fuse=off" "serial=1" ...

Each positional argument is one schedule (pbr_hip_set_schedule): a comma-separated list of
kernels=mega, chunk_log2=N, lanes=N, fuse=on|off, serial=1; "" is the default schedule.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes, tiles_for_rank  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lib", default=None, help="an experimental build of libpbr_hip.so")
    ap.add_argument("--shard", default=None, help="R/N: render only rank R's tiles of an N-GPU job "
                                                   "(per-rank frame time of the sharded bench)")
    ap.add_argument("--tile", type=int, default=32, help="tile edge of the --shard partition")
    ap.add_argument("--ref-file", default=None, help=".npy frame to compare against (written if absent), "
                                                     "so experimental builds can be checked against each other")
    ap.add_argument("--profile", action="store_true", help="per-kernel-family ms per frame (HIP events)")
    ap.add_argument("--batch", type=int, default=0, help="time K-frame pbr_hip_render_frames batches (bench.py's "
                                                           "timed window) instead of single frames; ms per frame")
    ap.add_argument("--user-stream", action="store_true", help="render on a torch-created stream (as bench.py) "
                                                                   "instead of torch's null stream (the context's own)")
    ap.add_argument("variants", nargs="*", default=[""])
    a = ap.parse_args()
    if a.lib:
        capi._lib = capi.load_library(a.lib)
    print("build:", capi.load_library().pbr_hip_build_info().decode(), flush=True)
    scene, rd = scenes.CONFIGS[a.config]()
    W, H, spp = rd.camera.width, rd.camera.height, rd.spp
    npx = W * H
    if a.shard:
        rk, n = (int(x) for x in a.shard.split("/"))
        tiles = tiles_for_rank(W, H, rk, n, a.tile)
        rd = scenes.render_desc(rd.camera, rd.integrator, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                                rd.sampler, tiles=tiles)
        npx = sum((t[2] - t[0]) * (t[3] - t[1]) for t in tiles)
    r = HipRenderer(0)
    r.upload(scene)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev) if a.user_stream else torch.cuda.current_stream(dev)
    if a.user_stream:
        torch.cuda.set_stream(stream)
    rgb = torch.empty((npx, 3), dtype=torch.float32, device=dev)
    rgba = torch.empty((npx, 4), dtype=torch.uint8, device=dev)
    ref = None
    if a.ref_file and os.path.exists(a.ref_file):
        ref = np.load(a.ref_file)
    for v in a.variants:
        # a variant is a schedule (pbr_hip_set_schedule; the library reads no environment variables):
        # comma-separated kernels=mega, chunk_log2=N, lanes=N, fuse=on|off, serial=1
        kw = dict(kv.split("=") for kv in v.split(",") if kv)
        r.set_schedule(kernels=capi.KERNELS_MEGAKERNEL if kw.get("kernels") == "mega" else capi.KERNELS_AUTO,
                       chunk_log2=int(kw.get("chunk_log2", 0)), lanes=int(kw.get("lanes", 0)),
                       fuse_camera={"on": capi.FUSE_ON, "off": capi.FUSE_OFF}.get(kw.get("fuse"), capi.FUSE_AUTO),
                       serial=kw.get("serial") == "1")
        r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ms = []
        if a.batch > 0:   # K frames per batch into K buffers; the last frame is the one compared
            rgbs = [rgb] + [torch.empty_like(rgb) for _ in range(a.batch - 1)]
            rgbas = [rgba] + [torch.empty_like(rgba) for _ in range(a.batch - 1)]
            rgbs, rgbas = rgbs[::-1], rgbas[::-1]
        for _ in range(a.steps):
            t0 = time.perf_counter()
            if a.batch > 0:
                r.render_frames(rd, [x.data_ptr() for x in rgbs], [x.data_ptr() for x in rgbas], stream=stream.cuda_stream)
            else:
                r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            ms.append((time.perf_counter() - t0) * 1e3 / max(1, a.batch))
        out = rgb.cpu().numpy()
        same = "ref" if ref is None else ("identical" if np.array_equal(out.view(np.uint32), ref.view(np.uint32))
                                          else "DIFFERENT max|d|=%g" % np.abs(out - ref).max())
        if ref is None:
            ref = out
            if a.ref_file:
                np.save(a.ref_file, out)
        m = float(np.median(ms))
        kern = ""
        if a.profile and hasattr(r.lib, "pbr_hip_set_profiling"):
            r.set_profiling(1)
            for _ in range(a.steps):
                r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            prof = r.get_profile()
            r.set_profiling(0)
            kern = "  [" + ", ".join(f"{k.replace('k_', '')} {v['ms'] / a.steps:.2f}" for k, v in prof.items()) + "]"
        tag = f" shard {a.shard} tile {a.tile} ({npx} px)" if a.shard else ""
        if a.batch > 0:   # device memory in use after the variant (the lanes' buffers dominate)
            fr, tot = torch.cuda.mem_get_info(dev)
            tag += f" [device memory in use {(tot - fr) / 1e9:.1f} of {tot / 1e9:.1f} GB]"
        print(f"{a.config}{tag} {os.path.basename(a.lib or 'lib')} {v or 'default':30s} {m:8.2f} ms  "
              f"{npx * spp / m / 1e3:8.1f} Msamples/s  {same}{kern}", flush=True)
        r.set_schedule()


if __name__ == "__main__":
    main()
