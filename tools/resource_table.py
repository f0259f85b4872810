"""Tabulate `make -C pysicalbasedraytracer_amd/csrc resource-usage` remarks (one row per kernel):
VGPRs, AGPRs, SGPRs, scratch bytes/lane, occupancy (waves/SIMD), LDS bytes/block."""
import re
import sys
from collections import OrderedDict

rows = OrderedDict()
cur = None
for line in open(sys.argv[1], errors="replace"):
    m = re.search(r"remark: (?:\./)?([^:]+):\d+:\d+: (?:remark: )?", line)
    m2 = re.search(r"Function Name: (\S+)", line)
    if m2:
        cur = m2.group(1)
        rows[cur] = {}
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"TotalSGPRs: (\d+)"),
                     ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)"), ("spill_v", r"VGPRs Spill: (\d+)"),
                     ("spill_s", r"SGPRs Spill: (\d+)")):
        mm = re.search(pat, line)
        if mm:
            rows[cur][key] = int(mm.group(1))


def _cxxfilt(names):
    import shutil
    import subprocess
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt") or "c++filt"
    try:
        out = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True).stdout.split("\n")
        return dict(zip(names, out))
    except Exception:
        return {}


_DEM = _cxxfilt(list(rows))


def demangle(n):
    """kernel name with its template arguments, e.g. k_wf_shade<5, true, 4, true>"""
    d = _DEM.get(n)
    if d:
        d = d.replace("(anonymous namespace)::", "").replace("pbr::", "")
        return re.sub(r"\(.*\)$", "", d).replace("void ", "")
    m = re.search(r"N_1\d+(k_\w+?)(?:I|E)", n) or re.search(r"(k_\w+)", n)
    return m.group(1) if m else n


print(f"{'kernel':52s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'spillV':>6s} {'scratch B/lane':>14s} {'waves/SIMD':>10s} {'LDS B':>7s}")
for n, r in rows.items():
    print(f"{demangle(n):52s} {r.get('vgpr', 0):5d} {r.get('agpr', 0):5d} {r.get('sgpr', 0):5d} {r.get('spill_v', 0):6d} "
          f"{r.get('scratch', 0):14d} {r.get('occ', 0):10d} {r.get('lds', 0):7d}")
