"""Writes tests/golden/ref_fullsize.json: the REFERENCE ITSELF on the BASELINE configs at full size
(tests/ref_scenes.fullsize_cases: C2, C3 on Halton, C4 at 3840x2160x1024, C5 — the 100,352-triangle
dragon stand-in, full raster, spp and depth), 64 one-pixel tiles each, through ref_render
(SamplerIntegrator::Render's per-pixel body, Integrator.cpp:286-344).

Run in the development container after `make -C oracle/ref`:

    python tests/golden/make_ref_fullsize.py

Recorded per case: the descriptor digest, the tile list, per pixel colObj/spp (float32 RGB bits) and
the 8-bit RGBA, and the reference's render seconds (informative)."""
import base64
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]

import numpy as np  # noqa: E402

import ref_lib as R  # noqa: E402
import ref_scenes as RS  # noqa: E402

OUT = os.path.join(HERE, "ref_fullsize.json")


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def main():
    t0 = time.time()
    out = {"generator": "tests/golden/make_ref_fullsize.py",
           "library": "oracle/_ref/libpbr_ref.so (reference sources unmodified, oracle/ref/Makefile)", "cases": {}}
    for name, (s, rd) in RS.fullsize_cases().items():
        rgb, rgba, sec = R.render(s, rd)
        tiles = [[rd.tiles[i].x0, rd.tiles[i].y0, rd.tiles[i].x1, rd.tiles[i].y1] for i in range(rd.n_tiles)]
        out["cases"][name] = {"digest": RS.scene_digest(s, rd), "raster": [rd.camera.width, rd.camera.height],
                              "spp": rd.spp, "tiles": tiles, "rgb": b64(rgb.astype("<f4")), "rgba": b64(rgba),
                              "reference_seconds": round(sec, 3)}
        print(f"{name}: {rgb.shape[0]} px x {rd.spp} spp in {sec:.2f} s", flush=True)
    json.dump(out, open(OUT, "w"), indent=0)
    print(f"wrote {OUT} ({os.path.getsize(OUT) // 1024} KB) in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
