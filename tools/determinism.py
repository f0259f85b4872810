"""Does a render depend on what ran before it in the process?  Renders the same scenes in fresh
contexts, in different orders, with device memory filled with junk and handed back to the driver in
between (hipMalloc'd queues of a new context may then start out as that junk), and prints each
frame's hash.  Every hash of one scene must be the same.

    python tools/determinism.py [--w 960 --h 540 --spp 256] [--junk-gb 64]
"""
import argparse
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from pysicalbasedraytracer_amd import HipRenderer, capi  # noqa: E402
from r5_shade_probe import scene  # noqa: E402


def junk(gb):
    dev = torch.device("cuda", 0)
    bufs = []
    for _ in range(int(gb)):
        bufs.append(torch.full((1 << 30,), 0xA5, dtype=torch.uint8, device=dev))
    torch.cuda.synchronize(dev)
    del bufs
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=960)
    ap.add_argument("--h", type=int, default=540)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--junk-gb", type=float, default=64)
    ap.add_argument("order", nargs="*", default=["c5", "c5", "c5@host", "junk", "c5", "mixed", "c5@host", "c3", "junk", "c3", "mixed"])
    a = ap.parse_args()
    seen = {}
    for kind in a.order:
        if kind == "junk":
            junk(a.junk_gb)
            print("junk", a.junk_gb, "GB written and released", flush=True)
            continue
        base, _, where = kind.partition("@")   # kind@host: the BVH built by the host builder
        s, rd = scene(base, 2 * a.w, 2 * a.h, a.spp) if base in ("c3", "c5") else scene(base, a.w, a.h, a.spp)
        r = HipRenderer(0)
        if where == "host":
            r.set_bvh_build(capi.BVH_BUILD_HOST)
        r.upload(s)
        nodes, ids = r.get_bvh()
        bh = hashlib.sha256(nodes.tobytes() + ids.tobytes()).hexdigest()[:12]
        rgb, rgba, _ = r.render(rd)
        r.close()
        h = hashlib.sha256(rgb.tobytes()).hexdigest()[:16]
        seen.setdefault(base, set()).add(h)
        print(f"{kind:8s} frame {h} bvh {bh}", flush=True)
    bad = {k: v for k, v in seen.items() if len(v) > 1}
    print("DETERMINISTIC" if not bad else f"DIFFERS: {bad}", flush=True)


if __name__ == "__main__":
    main()
