"""How much of the Path shade's cost is material divergence?  C4's scene with the three dragons'
materials varied (mixed as in C4, or all one recipe), serial schedule, per-family ns per unit.

    python tools/shade_probe.py [--w 1920 --h 1080 --spp 256] [--lib path]
"""
import argparse
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes  # noqa: E402


def scene(kind, w, h, spp):
    if kind in ("c3", "c5"):   # the C3 / C5 scenes at a quarter of their raster
        return scenes.CONFIGS[kind.upper()](w // 2, h // 2, spp)
    if kind == "c2":           # C2 as benchmarked (1920x1080, 64 spp)
        return scenes.CONFIGS["C2"]()
    s = scenes.Scene()
    white = s.matte((0.8, 0.8, 0.8))
    recipes = {"glass": s.glass, "metal": s.metal, "plastic": s.plastic, "matte": lambda: s.matte((0.5, 0.5, 0.5))}
    if kind == "mixed":
        mats = [s.glass(), s.metal(), s.plastic()]
    else:
        m = recipes[kind]()
        mats = [m, m, m]
    for mat, dx in zip(mats, (-2.3, 0.0, 2.3)):
        scenes._dragon(s, mat, None, xform=scenes.translate(dx, 0.0, 0.0))
    Pf, If = scenes.quad(-1.12, 10.0)
    s.mesh(Pf, If, white)
    Pl, Il = scenes.quad(2.9, 1.8, flip=True)
    s.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), white, n_samples=5)
    cam = scenes.camera(w, h, (0.0, 1.2, 5.0), (0.0, -0.3, 0.0))
    return s, scenes.render_desc(cam, capi.INTEGRATOR_PATH, spp, 8, rr_threshold=0.8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--libs", nargs="*", default=[None], help="library builds to compare (one context at a time)")
    ap.add_argument("--counters", action="store_true", help="profiling 2: work counters too (units)")
    ap.add_argument("--frames", type=int, default=0, help="then time this many frames under the default schedule")
    ap.add_argument("kinds", nargs="*", default=["mixed", "glass", "metal", "plastic", "matte"])
    a = ap.parse_args()
    for lib in a.libs:
        if lib:
            capi._lib = capi.load_library(os.path.abspath(lib))
        print("build:", lib, capi._lib.pbr_hip_build_info().decode() if capi._lib else capi.load_library().pbr_hip_build_info().decode(), flush=True)
        run(a)


def run(a):
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)   # (not the default stream: its handle 0 means "the context's stream")
    rgb = torch.empty((a.w * a.h, 3), dtype=torch.float32, device=dev)
    rgba = torch.empty((a.w * a.h, 4), dtype=torch.uint8, device=dev)
    for kind in a.kinds:
        s, rd = scene(kind, a.w, a.h, a.spp)
        r = HipRenderer(0)
        r.upload(s)
        r.set_schedule(serial=True)
        r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        r.set_profiling(2 if a.counters else 1)
        r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        prof = r.get_profile()
        r.set_profiling(0)
        parts = []
        for k, v in prof.items():
            if v["launches"] == 0:
                continue
            ns = v["ms"] * 1e6 / max(1, v["units"])
            extra = ""
            if a.counters and any(v["counts"][2:6]):   # PBR_STACK_DIAG: rays with a stack deeper than 6/10/16/24
                extra = " stack>6/10/16/24 " + "/".join(f"{c / max(1, v['units']):.4f}" for c in v["counts"][2:6])
            parts.append(f"{k.replace('k_', '')} {v['ms']:.1f} ms {v['units'] / 1e6:.1f} M {ns:.3f} ns/u{extra}")
        npx = rd.camera.width * rd.camera.height   # (the buffers are sized for the largest kind)
        h = hashlib.sha256(rgb[:npx].cpu().numpy().tobytes()).hexdigest()[:16]
        if a.frames:
            r.set_schedule()
            for _ in range(2):
                r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.frames):
                r.render_device(rd, rgb.data_ptr(), rgba.data_ptr(), stream=stream.cuda_stream, sync=False)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            timing = f"default {e0.elapsed_time(e1) / a.frames:.2f} ms/frame"
            if hasattr(r.lib, "pbr_hip_render_frames"):   # the same frames as one batch (timing only)
                r.render_frames(rd, [rgb.data_ptr()] * a.frames, [rgba.data_ptr()] * a.frames, stream=stream.cuda_stream)
                torch.cuda.synchronize(dev)
                e0.record(stream)
                r.render_frames(rd, [rgb.data_ptr()] * a.frames, [rgba.data_ptr()] * a.frames, stream=stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                timing += f", batch {e0.elapsed_time(e1) / a.frames:.2f}"
            parts.insert(0, timing)
        print(f"{kind:8s} frame {h} " + " | ".join(parts), flush=True)
        r.close()


if __name__ == "__main__":
    main()
