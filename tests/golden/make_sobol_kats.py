"""Generates tests/golden/sobol_kats.json from the reference's own Sobol tables.

The reference ships pbrt-v3's SobolMatrices32 / VdCSobolMatrices / VdCSobolMatricesInv
(Sampler/SobolMatrices.cpp) but no SobolSampler.  This script — run in the
development container, where /root/reference exists — reads those tables as text and evaluates
pbrt-v3's published SobolIntervalToIndex and SobolSampler::SampleDimension on a set of rasters,
pixels and sample numbers — including sample numbers whose global index needs more than 32 bits
(pbrt-v3's index is an int64_t) — for dimensions 0-127.  The fixture keeps only the computed
outputs (the sample index and the float bit patterns) plus SHA-256s of the reference's
dimension-0/1 matrix words and of the whole SobolMatrices32 table (1024 x 52 words,
little-endian); no table content is stored.

    python tests/golden/make_sobol_kats.py [/root/reference]
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(REF, "Sampler", "SobolMatrices.cpp")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sobol_kats.json")
MATRIX_SIZE = 52
HIGH_DIMS = 128   # dims2_127: one 8-hex-digit float bit pattern per dimension 2..127, concatenated
ONE_MINUS_EPS = np.float32(0.99999994)


def numbers(block):
    return [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]+)", block)]


def table(text, name):
    start = text.index(name)
    body = text[text.index("{", start) + 1:]
    depth, end = 1, 0
    for k, ch in enumerate(body):
        depth += ch == "{"
        depth -= ch == "}"
        if depth == 0:
            end = k
            break
    return body[:end]


def main():
    text = open(SRC).read()
    m32 = numbers(table(text, "const uint32_t SobolMatrices32"))
    vdc_block = table(text, "const uint64_t VdCSobolMatrices[]")
    inv_block = table(text, "const uint64_t VdCSobolMatricesInv[]")
    vdc = [numbers(b) for b in re.findall(r"\{([^{}]*)\}", vdc_block)]
    inv = [numbers(b) for b in re.findall(r"\{([^{}]*)\}", inv_block)]

    def interval_to_index(m, frame, px, py):   # pbrt-v3 lowdiscrepancy.h SobolIntervalToIndex
        if m == 0:
            return 0
        index = frame << (2 * m)
        delta, c, f = 0, 0, frame
        while f:
            if f & 1:
                delta ^= vdc[m - 1][c]
            f >>= 1
            c += 1
        b = ((px << m) | py) ^ delta
        c = 0
        while b:
            if b & 1:
                index ^= inv[m - 1][c]
            b >>= 1
            c += 1
        return index

    def sample_dimension(index, dim, res, pix):   # SobolSampler::SampleDimension over SobolSampleFloat
        v, a, i = 0, index, dim * MATRIX_SIZE
        while a:
            if a & 1:
                v ^= m32[i]
            a >>= 1
            i += 1
        s = min(np.float32(v) * np.float32(2.0 ** -32), ONE_MINUS_EPS)
        if dim >= 2:
            return np.float32(s)
        s = np.float32(s * np.float32(res)) + np.float32(0)
        s = np.float32(s - np.float32(pix))
        return np.float32(min(max(s, np.float32(0)), ONE_MINUS_EPS))

    cases = []
    rng = np.random.default_rng(7)
    for (w, h) in [(1920, 1080), (256, 256), (100, 37), (3840, 2160), (1, 1)]:
        res, m = 1, 0
        while res < max(w, h):
            res, m = res * 2, m + 1
        pix = [(0, 0), (w - 1, h - 1), (min(5, w - 1), min(7, h - 1))]
        pix += [(int(rng.integers(w)), int(rng.integers(h))) for _ in range(3)]
        for (px, py) in pix:
            wide = 1 << (32 - 2 * m) if m else 256   # the first sample number whose index needs bit 32
            for frame in (0, 1, 2, 63, 255, wide, wide + 5, 3 * wide + 17):
                idx = interval_to_index(m, frame, px, py)
                d0 = sample_dimension(idx, 0, res, px)
                d1 = sample_dimension(idx, 1, res, py)
                hi = "".join("%08x" % np.float32(sample_dimension(idx, d, res, 0)).view(np.uint32)
                             for d in range(2, HIGH_DIMS))
                cases.append({"raster": [w, h], "pixel": [px, py], "sample": frame, "index": idx,
                              "dim0": "%08x" % np.float32(d0).view(np.uint32),
                              "dim1": "%08x" % np.float32(d1).view(np.uint32),
                              "dims2_127": hi})
    words = np.array(m32[:2 * MATRIX_SIZE], np.uint32).tobytes()
    json.dump({"source": "Sampler/SobolMatrices.cpp (SobolMatrices32, VdCSobolMatrices, VdCSobolMatricesInv) "
                         "through pbrt-v3 SobolIntervalToIndex / SobolSampler::SampleDimension",
               "dims01_sha256": hashlib.sha256(words).hexdigest(),
               "all_sha256": hashlib.sha256(np.array(m32, "<u4").tobytes()).hexdigest(),
               "high_dims": HIGH_DIMS, "cases": cases}, open(OUT, "w"), indent=0)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
