"""Writes the mesh-ingest fixtures: tests/golden/mesh_small.3d (a deterministic mesh in the
reference's ".3d" text format) and tests/golden/mesh_ref.json — what the REFERENCE's own reader
(Shape/plyRead.h plyInfo, through oracle/_ref/libpbr_ref.so) returns for it: the vertex floats
(×20) as bit patterns and the triangle indices.

    python tests/golden/make_mesh_fixtures.py      (development container, after make -C oracle/ref)
"""
import base64
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]
import ref_lib as R  # noqa: E402

MESH = os.path.join(HERE, "mesh_small.3d")
OUT = os.path.join(HERE, "mesh_ref.json")


def write_mesh():
    rng = np.random.default_rng(20261016)
    nv, nf = 64, 110
    v = rng.uniform(-0.12, 0.12, size=(nv, 3))
    f = rng.integers(0, nv, size=(nf, 3))
    lines = [f"vertex {nv}", f"face {nf}"]
    # the Stanford .3d conversions carry 6-7 significant digits; some exponent forms too
    for i, (x, y, z) in enumerate(v):
        fmt = "{:.7g}" if i % 5 else "{:.6e}"
        lines.append(" ".join(fmt.format(c) for c in (x, y, z)))
    lines += [f"3 {a} {b} {c}" for a, b, c in f]
    open(MESH, "w").write("\n".join(lines) + "\n")


def main():
    write_mesh()
    v, i = R.ply_info(MESH)
    out = {"generator": "tests/golden/make_mesh_fixtures.py", "reader": "Shape/plyRead.h plyInfo (oracle/_ref)",
           "file_sha256": hashlib.sha256(open(MESH, "rb").read()).hexdigest(),
           "n_vertices": int(v.shape[0]), "n_triangles": int(i.shape[0]),
           "vertices_f32": base64.b64encode(v.astype("<f4").tobytes()).decode(),
           "indices_i32": base64.b64encode(i.astype("<i4").tobytes()).decode()}
    json.dump(out, open(OUT, "w"), indent=1)
    print(f"wrote {OUT}: {v.shape[0]} vertices, {i.shape[0]} triangles")


if __name__ == "__main__":
    main()
