import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes

def scene(sphere=True):
    s = scenes.Scene()
    mirror = s.mirror((0.9, 0.9, 0.9))
    matte = s.matte((0.6, 0.3, 0.2))
    for z, flip in ((-1.0, False), (1.5, True)):
        P = np.array([(-3, -3, z), (3, -3, z), (3, 3, z), (-3, 3, z)], np.float32)
        I = np.array([(0, 1, 2), (0, 2, 3)] if not flip else [(0, 2, 1), (0, 3, 2)], np.int32)
        s.mesh(P, I, mirror)
    if sphere:
        s.sphere((0.0, 0.0, 0.2), 0.3, matte)
    s.point_light((0.0, 1.0, 0.5), (4.0, 4.0, 4.0))
    return s

r = HipRenderer(0)
cam = scenes.camera(40, 30, (0.2, 0.1, 1.2), (0.0, 0.0, -1.0))
for sph in (True, False):
    s = scene(sph)
    r.upload(s)
    for depth in (2, 5, 8, 9, 12):
        rd = scenes.render_desc(cam, capi.INTEGRATOR_WHITTED, 4, depth)
        os.environ["PBR_WAVEFRONT"] = "1"; g1, _, _ = r.render(rd)
        os.environ["PBR_WAVEFRONT"] = "0"; g0, _, _ = r.render(rd)
        c, _, _ = O.render(s, rd)
        d1 = np.abs(g1 - c).max(axis=1); d0 = np.abs(g0 - c).max(axis=1)
        i1 = int(d1.argmax()); i0 = int(d0.argmax())
        print(f"sphere={sph} depth={depth}: wf-vs-cpu {d1.max():.4g} at px {i1 % 40},{i1 // 40} (gpu {g1[i1]}, cpu {c[i1]}); "
              f"mk-vs-cpu {d0.max():.4g} at px {i0 % 40},{i0 // 40}; wf==mk {np.array_equal(g1, g0)}; bad px wf {(d1 > 1e-3).sum()} mk {(d0 > 1e-3).sum()}", flush=True)
