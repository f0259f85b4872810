import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pysicalbasedraytracer_amd import HipRenderer, scenes, capi
capi._lib = capi.load_library(os.path.join(ROOT, "exp", "libdbg.so"))
P, I = scenes.dragon_standin(n=40)
s, rd = scenes.config_c4(96, 54, 1, mesh=(P, I, "small"))
r = HipRenderer(0); r.upload(s)
rd2 = scenes.render_desc(rd.camera, rd.integrator, 1, 2, rd.rr_threshold, rd.light_strategy, rd.sampler)
os.environ["PBR_WAVEFRONT"] = "0"; mk, _, _ = r.render(rd2)
sys.stdout.flush()
os.environ["PBR_WAVEFRONT"] = "1"; wf, _, _ = r.render(rd2)
print("pixel", wf[24 * 96 + 65], mk[24 * 96 + 65])
