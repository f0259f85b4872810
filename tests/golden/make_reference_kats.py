"""Writes tests/golden/reference_kats.json.

The values are outputs of the reference renderer itself, recorded by the survey that built and ran
it ("Verified capture paths"): Halton bit patterns from three GlobalSampler::Get2D()
calls (dims 0,1 / 2,3 / 5,6 — Get2D at dimension 4 skips to 5, Sampler.cpp:138-143), the
second-sample dims 0,1 at pixel (0,0), one float Li capture and the LinearBVHNode size.  The scene
of the Li capture (camera and light at (0,0,3) over a z=0 triangle) is the one the oracle
reproduces bit-exactly; it is stated here so the test can rebuild it.
"""
import json
import os

KATS = {
    "halton_1920x1080": {
        "base_scales": [128, 243], "base_exponents": [7, 5], "sample_stride": 31104,
        "get2d_x3_dims": [0, 1, 2, 3, 5, 6],
        "pixels": {
            "0,0": ["00000000", "00000000", "3f400000", "3f000001", "3ed55556", "3f500000"],
            "1,0": ["3f1e0000", "3eca458a", "3ea7f5ea", "3f12eaf9", "3ead2d8b", "3f636dfe"],
            "1919,1079": ["3eac0000", "3f30fcd9", "3f1bd2fb", "3f55bd54", "3f39969a", "3ea4f1aa"],
        },
        "pixel_0_0_sample_1_dims_0_1": [0.8085938, 0.7572018],
    },
    "li_capture": {
        "integrator": "whitted", "max_depth": 5, "width": 32, "height": 32, "spp": 4, "pixel": [16, 16],
        "material": "matte Kd 0.5", "triangle": [[-1, -1, 0], [1, -1, 0], [0, 1, 0]],
        "point_light": {"pos": [0, 0, 3], "I": 9}, "camera": {"eye": [0, 0, 3], "look": [0, 0, 0], "up": [0, 1, 0]},
        "value": 0.15856609, "analytic_centre": 0.15915494,
    },
    "sizeof": {"LinearBVHNode": 32, "Ray": 40, "SurfaceInteraction": 264},
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump(KATS, f, indent=1, sort_keys=True)
    print("wrote", out)
