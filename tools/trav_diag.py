"""Traversal-loop diagnostics of a PBR_TRAV_DIAG build (make EXTRA=-DPBR_TRAV_DIAG=1): per traversal
kernel family, rays, mean loop steps per ray and the SIMD utilisation of the loop (lane steps /
(wave steps x 64)).

    python tools/trav_diag.py --lib xso/diag.so --config C3"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--lib", required=True)
    a = ap.parse_args()
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
    for k, v in prof.items():
        c = v["counts"]
        if c[7]:
            print(f"{a.config} {k:22s} rays {c[0] / 1e6:9.2f} M  steps/ray {c[6] / max(1, c[0]):6.2f}  "
                  f"SIMD utilisation {c[6] / c[7]:.3f}  ms {v['ms']:.2f}", flush=True)


if __name__ == "__main__":
    main()
