"""Debug: nested material-less shells under VolPath — wavefront / megakernel / oracle per shell count."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import oracle_lib as O
from pysicalbasedraytracer_amd import HipRenderer, capi, scenes
from test_gpu_materials import nested_shells, CAM

hip = HipRenderer(0)
for integ in (capi.INTEGRATOR_VOLPATH,):
    for medium in (True, False):
        for n in (2, 5, 10, 14, 16, 20):
            s = nested_shells(n, medium=medium)
            cam = scenes.camera(40, 28, CAM["eye"], CAM["look"])
            rd = scenes.render_desc(cam, integ, 4, 5)
            hip.upload(s)
            os.environ["PBR_WAVEFRONT"] = "1"
            wf, _, _ = hip.render(rd)
            os.environ["PBR_WAVEFRONT"] = "0"
            mk, _, _ = hip.render(rd)
            c, _, _ = O.render(s, rd)
            d = lambda a, b: (float(np.abs(a - b).max()), int((a.view(np.uint32) != b.view(np.uint32)).any(1).sum()))
            print(f"medium={medium} n={n}: wf-oracle {d(wf, c)} mk-oracle {d(mk, c)} wf-mk {d(wf, mk)}", flush=True)
