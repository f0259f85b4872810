"""Frames queued back to back as bench.py queues them (a torch stream, no host sync between frames),
under a given lane count: run under `rocprofv3 --kernel-trace` to see how the lanes' kernels overlap
across frame boundaries.

    python tools/r5_lanes_trace.py --config C2 --lanes 4 --frames 6 [--sync]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--frames", type=int, default=6)
    ap.add_argument("--sync", action="store_true", help="host sync after every frame (tune_wavefront's way)")
    ap.add_argument("--default-stream", action="store_true", help="render on the context's own stream")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    scene, rd = scenes.CONFIGS[a.config]()
    r = HipRenderer(0)
    r.upload(scene)
    r.set_schedule(lanes=a.lanes)
    W, H = rd.camera.width, rd.camera.height
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    handle = 0 if a.default_stream else stream.cuda_stream
    rgb = torch.empty((W * H, 3), dtype=torch.float32, device=dev)
    rgba = torch.empty((W * H, 4), dtype=torch.uint8, device=dev)
    for _ in range(2):
        r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=handle, sync=False)
    r.sync()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.frames):
        r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=handle, sync=False)
        if a.sync:
            r.sync()
            torch.cuda.synchronize(dev)
    r.sync()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / a.frames * 1e3
    print(f"{a.config} lanes {a.lanes or 3} {'sync' if a.sync else 'queued'} "
          f"{'ctx-stream' if a.default_stream else 'torch-stream'}: {ms:.3f} ms/frame", flush=True)


if __name__ == "__main__":
    main()
