"""Writes tests/golden/ref_fixtures.json: outputs of the REFERENCE ITSELF on the scenes of
tests/ref_scenes.py.

Run in the development container, after `make -C oracle/ref` has built oracle/_ref/libpbr_ref.so
from the reference's unmodified sources (plus the harness oracle/ref/ref_harness.cpp):

    python tests/golden/make_ref_fixtures.py

Recorded (all values bit patterns; arrays base64 of little-endian raw data):
  * renders  — per pixel colObj/spp (float32 RGB) and the 8-bit RGBA of Integrator.cpp:327-344,
               from SamplerIntegrator::Render's per-pixel body (ref_render), 12 scenes covering the
               Whitted/Path/VolPath integrators, every material, point/area/SkyBox/InfiniteArea
               lights, media and material-less medium interfaces;
  * frames   — the FrameBuffer bytes of the reference's own Integrator::Render on square rasters;
  * bvh      — SHA-256 of BVHAccel's LinearBVHNode array (the bytes it writes: ref_scenes.canonical_nodes)
               and of its primitive order;
  * intersect— Scene::Intersect {hit, t, primitive} / IntersectP records for 3000 rays (incl. vertex
               and edge hits; the rays are regenerated from ref_scenes and checked by hash);
  * camera   — PerspectiveCamera::GenerateRayDifferential rays.
Each entry keeps the SHA-256 of its scene/render descriptors (ref_scenes.scene_digest).
"""
import base64
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]

import numpy as np  # noqa: E402

import ref_lib as R  # noqa: E402
from pysicalbasedraytracer_amd import scenes  # noqa: E402
import ref_scenes as RS  # noqa: E402

OUT = os.path.join(HERE, "ref_fixtures.json")


def b64(a):
    return base64.b64encode(np.ascontiguousarray(a).tobytes()).decode()


def main():
    t0 = time.time()
    out = {"generator": "tests/golden/make_ref_fixtures.py", "library": "oracle/_ref/libpbr_ref.so "
           "(reference sources unmodified, oracle/ref/Makefile)", "renders": {}, "frames": {}, "bvh": {}}
    for name, (s, rd) in RS.render_cases().items():
        if "mesh_3d" in s.info:   # an ingested mesh: the reference's own reader gives the arrays the scene holds
            v, i = R.ply_info(s.info["mesh_3d"])
            V, F = scenes.load_3d(s.info["mesh_3d"])
            assert np.array_equal(v.view(np.uint32), V.view(np.uint32)) and np.array_equal(i, F), name
        rgb, rgba, sec = R.render(s, rd)
        out["renders"][name] = {"digest": RS.scene_digest(s, rd), "n": int(rgb.shape[0]),
                                "rgb": b64(rgb.astype("<f4")), "rgba": b64(rgba)}
        print(f"render {name}: {rgb.shape[0]} px in {sec:.2f} s", flush=True)
    for name, (s, rd) in RS.frame_cases().items():
        fb, sec = R.render_frame(s, rd)
        out["frames"][name] = {"digest": RS.scene_digest(s, rd), "shape": list(fb.shape), "fb": b64(fb)}
        print(f"frame {name}: {fb.shape} in {sec:.2f} s", flush=True)
    for name, s in RS.bvh_cases().items():
        nodes, ids = R.build_bvh(s)
        out["bvh"][name] = {"digest": RS.scene_digest(s), "n_nodes": int(nodes.size // 32),
                            "nodes_sha256": hashlib.sha256(RS.canonical_nodes(nodes).tobytes()).hexdigest(),
                            "prim_ids_sha256": hashlib.sha256(ids.astype("<i4").tobytes()).hexdigest()}
        print(f"bvh {name}: {nodes.size // 32} nodes", flush=True)
    s, rays = RS.intersect_case()
    hit = R.intersect(s, rays)
    anyhit = R.intersect(s, rays, any_hit=True)
    out["intersect"] = {"digest": RS.scene_digest(s), "rays_sha256": hashlib.sha256(rays.astype("<f4").tobytes()).hexdigest(),
                        "closest": b64(hit[:, :3].astype("<f4")), "any": b64(anyhit[:, 0].astype(np.uint8))}
    print(f"intersect: {int(hit[:, 0].sum())} of {rays.shape[0]} rays hit", flush=True)
    cams, pfs = RS.camera_case()
    out["camera"] = []
    for cam, pf in zip(cams, pfs):
        r = R.camera_rays(cam, pf)
        out["camera"].append({"raster": [cam.width, cam.height], "pfilm": b64(pf.astype("<f4")), "rays": b64(r.astype("<f4"))})
    json.dump(out, open(OUT, "w"), indent=0)
    print(f"wrote {OUT} ({os.path.getsize(OUT) // 1024} KB) in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
