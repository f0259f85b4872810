import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from pysicalbasedraytracer_amd import HipRenderer, scenes, capi
import oracle_lib as O
P, I = scenes.dragon_standin(n=40)
s, rd = scenes.config_c4(96, 54, 1, mesh=(P, I, "small"))
print("maxdepth", rd.max_depth, "rr", rd.rr_threshold)
r = HipRenderer(0); r.upload(s)
for depth in [1, 2, 3, 4, 8]:
    rd2 = scenes.render_desc(rd.camera, rd.integrator, 1, depth, rd.rr_threshold, rd.light_strategy, rd.sampler)
    os.environ["PBR_WAVEFRONT"] = "0"; mk, _, _ = r.render(rd2)
    os.environ["PBR_WAVEFRONT"] = "1"; wf, _, _ = r.render(rd2)
    d = np.abs(wf - mk).max(axis=1)
    idx = np.nonzero(d)[0]
    print("depth", depth, "differing", idx.size, "max", float(d.max()))
    for i in idx[:4]:
        print("   ", i % 96, i // 96, "wf", wf[i], "mk", mk[i])
