"""Time the host and device SAH builds (pbr_hip_build_bvh) on the C2 stand-ins.

    python tools/bvh_build_time.py [n ...]      # n x n x 2 triangles (224 -> 100,352; 660 -> 871,200)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [224, 660]
    r = HipRenderer(0)
    for n in sizes:
        P, I = scenes.dragon_standin(n=n)
        v = P[I]
        b = np.concatenate([v.min(axis=1), v.max(axis=1)], axis=1).astype(np.float32)
        dev = [r.build_bvh(b, capi.BVH_BUILD_DEVICE) for _ in range(3)]
        host = r.build_bvh(b, capi.BVH_BUILD_HOST)
        same = np.array_equal(dev[-1][0], host[0]) and np.array_equal(dev[-1][1], host[1])
        t = sorted(d[2]["ms"] for d in dev)[1]
        k = sorted(d[2]["kernel_ms"] for d in dev)[1]
        print(f"{I.shape[0]} triangles: host {host[2]['ms']:.1f} ms, device {t:.1f} ms ({k:.1f} ms kernels), "
              f"identical={same}", flush=True)
    r.close()


if __name__ == "__main__":
    main()
