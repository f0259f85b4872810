"""A/B timing of library builds in ONE process on one GPU, interleaved, with bit-identity checks.

    python tools/ab_libs.py --configs C2 C3 --rounds 3 --steps 5 xso/base.so pysicalbasedraytracer_amd/libpbr_hip.so

Each round renders every config with every library, one context at a time (default schedule, frames queued back to back on
one stream, as bench.py's timed window); the frame of each library must equal the first library's
bit for bit.  Prints per (config, library) the median frame ms over the rounds."""
import argparse
import ctypes as C
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C2"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    libs = [capi.load_library(os.path.abspath(p)) for p in a.libs]
    for p, lib in zip(a.libs, libs):
        print(f"{p}: {lib.pbr_hip_build_info().decode()}", flush=True)
    for cfg in a.configs:
        scene, rd = scenes.CONFIGS[cfg]()
        W, H, spp = rd.camera.width, rd.camera.height, rd.spp
        rgb = torch.empty((W * H, 3), dtype=torch.float32, device=dev)
        rgba = torch.empty((W * H, 4), dtype=torch.uint8, device=dev)
        times = [[] for _ in libs]
        ref = None
        for rnd in range(a.rounds):
            for k, lib in enumerate(libs):
                # one context at a time: a Path/VolPath context holds ~60 GB of queues (3 lanes)
                capi._lib = lib
                r = HipRenderer(0)
                r.upload(scene)
                r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream, sync=False)
                r.sync()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream, sync=False)
                r.sync()
                torch.cuda.synchronize(dev)
                times[k].append((time.perf_counter() - t0) / a.steps * 1e3)
                frame = rgb.cpu().numpy().view(np.uint32)
                if ref is None:
                    ref = frame.copy()
                same = np.array_equal(frame, ref)
                print(f"{cfg} round {rnd} {a.libs[k]}: {times[k][-1]:.3f} ms {'bit-identical' if same else 'DIFFERS'}",
                      flush=True)
                if not same:
                    print(f"  differing pixels: {int((frame != ref).any(axis=1).sum())}", flush=True)
                r.close()
        for k in range(len(libs)):
            print(f"RESULT {cfg} {a.libs[k]}: median {statistics.median(times[k]):.3f} ms "
                  f"(min {min(times[k]):.3f}, {len(times[k])} rounds)", flush=True)


if __name__ == "__main__":
    main()
