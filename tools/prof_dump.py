"""Per kernel family of one frame: launches, HIP-event ms, work units, algorithmic bytes and the raw
counters of pbr_hip_get_profile (profiling level 2), as JSON lines.

    python tools/prof_dump.py --config C4 [--lib xso/x.so]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--lib", default=None)
    a = ap.parse_args()
    if a.lib:
        capi._lib = capi.load_library(a.lib)
    scene, rd = scenes.CONFIGS[a.config]()
    r = HipRenderer(0)
    r.upload(scene)
    n = rd.camera.width * rd.camera.height
    rgb = torch.empty((n, 3), dtype=torch.float32, device="cuda")
    rgba = torch.empty((n, 4), dtype=torch.uint8, device="cuda")
    r.render_device(rd, rgb.data_ptr(), rgba.data_ptr())
    r.set_profiling(2)
    r.render_device(rd, rgb.data_ptr(), rgba.data_ptr())
    prof = r.get_profile()
    r.set_profiling(0)
    samples = n * rd.spp
    for k, v in prof.items():
        v = dict(v, family=k, config=a.config, bytes_per_sample=round(v["bytes"] / samples, 2),
                 units_per_sample=round(v["units"] / samples, 4))
        print(json.dumps(v), flush=True)


if __name__ == "__main__":
    main()
