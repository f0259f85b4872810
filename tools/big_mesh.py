"""C2 with a displaced-sphere stand-in of the real Stanford Dragon's size (871,200 triangles vs the
100,352 of the default stand-in): scene upload (host SAH build) time and frame time on one GPU.

    python tools/big_mesh.py [n]     # n×n×2 triangles (660 → 871,200)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, scenes  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 660
    P, I = scenes.dragon_standin(n=n)
    s, rd = scenes.config_c2(mesh=(P, I, f"standin-{n}"))
    r = HipRenderer(0)
    t0 = time.time()
    r.upload(s)
    up = time.time() - t0
    dev = torch.device("cuda", 0)
    npx = rd.camera.width * rd.camera.height
    rgb = torch.empty((npx, 3), dtype=torch.float32, device=dev)
    rgba = torch.empty((npx, 4), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)
    ms = []
    for _ in range(3):
        t0 = time.perf_counter()
        r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        ms.append((time.perf_counter() - t0) * 1e3)
    m = sorted(ms)[1]
    print(f"C2 with {I.shape[0]} triangles: upload {up:.2f} s, frame {m:.2f} ms, "
          f"{npx * rd.spp / m / 1e3:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
