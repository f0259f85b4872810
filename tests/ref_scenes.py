"""Scenes of the reference-output fixtures (tests/golden/ref_fixtures.json) — TEST INFRASTRUCTURE.

tests/golden/make_ref_fixtures.py renders these with the reference itself (oracle/_ref/libpbr_ref.so,
the reference's unmodified sources + oracle/ref/ref_harness.cpp); tests/test_ref_fixtures.py checks
the CPU restatement and the device against what it recorded.  Every case carries a digest of its
descriptors, so a test that rebuilds a scene differently from the generator fails loudly instead
of comparing against the wrong fixture.

Constraints the reference imposes on these scenes: triangle meshes only (its Sphere is a stub, F2),
the Halton sampler (it has no Sobol sampler, F3), fov 90 pinhole cameras (CreatePerspectiveCamera,
Perspective.cpp:84-104), environment maps with .hdr-representable values (scenes.rgbe_roundtrip).
"""
from __future__ import annotations

import ctypes as C
import hashlib

import numpy as np

from pysicalbasedraytracer_amd import capi, scenes

CAM_C = dict(eye=(0.0, 0.55, 2.6), look=(0.0, -0.25, 0.0))


def small_mesh(n=32):
    P, I = scenes.dragon_standin(n=n)
    return P, I, f"standin-{n}"


def halton(rd):
    return scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                              capi.SAMPLER_HALTON)


def uv_patch(n=12, z=-0.6):
    xs = np.linspace(-3.0, 3.0, n + 1, dtype=np.float32)
    P, UV, I = [], [], []
    for j, y in enumerate(xs):
        for i, x in enumerate(xs):
            P.append((x, z + 0.12 * np.sin(2.0 * x) * np.cos(1.5 * y), y))
            UV.append((2.5 * i / n, j / n))
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i, (j + 1) * (n + 1) + i + 1
            I += [(a, d, b), (a, c, d)]
    return np.array(P, np.float32), np.array(I, np.int32), np.array(UV, np.float32)


def box(lo, hi):
    """A closed axis-aligned box, outward-facing triangles."""
    x0, y0, z0 = lo
    x1, y1, z1 = hi
    P = np.array([(x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0),
                  (x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1)], np.float32)
    I = np.array([(0, 2, 1), (0, 3, 2), (4, 5, 6), (4, 6, 7), (0, 1, 5), (0, 5, 4),
                  (3, 6, 2), (3, 7, 6), (0, 4, 7), (0, 7, 3), (1, 2, 6), (1, 6, 5)], np.int32)
    return P, I


def texture_image(w, h, seed):
    """A deterministic RGB image with structure at texel scale (checks + gradients), rows as stbi_loadf
    returns them."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    base = rng.random(3) * 0.6 + 0.2
    img = np.stack([base[0] + 0.3 * ((x // 3 + y // 2) % 2), base[1] * (0.5 + x / w), base[2] * (0.4 + 0.6 * y / h)], -1)
    return (img + rng.random((h, w, 3)) * 0.15).astype(np.float32)


def inf_xform():   # main.cpp's InfinityLightToWorld = RotateX(-90) * RotateY(-0) * RotateZ(-50)
    return scenes.compose(scenes.compose(scenes.rotate_x(-90), scenes.rotate_y(-0.0)), scenes.rotate_z(-50))


def render_cases():
    """name → (scene, render desc) for the per-pixel float + RGBA8 fixtures (ref_render)."""
    m = small_mesh()
    out = {}
    s, rd = scenes.config_c2(48, 27, 8, mesh=m, sky=scenes.procedural_sky(128, 64))
    out["c2_whitted_skybox_mirror"] = (s, rd)

    s = scenes.Scene()
    s.mesh(m[0], m[1], s.matte((0.7, 0.3, 0.2)))
    Pf, If = scenes.quad(-1.12, 6.0)
    s.mesh(Pf, If, s.mirror((0.9, 0.9, 0.9)))
    s.point_light((1.0, 2.0, 1.5), (6.0, 5.0, 4.0))
    s.point_light((-1.5, 1.0, 2.0), (3.0, 3.0, 6.0))
    out["whitted_two_points_mirror"] = (s, scenes.render_desc(scenes.camera(40, 24, **CAM_C), capi.INTEGRATOR_WHITTED, 4, 5))

    s, rd = scenes.config_c3(48, 27, 16, mesh=m)
    out["c3_path_area"] = (s, halton(rd))

    s, rd = scenes.config_c3(40, 24, 8, mesh=m)
    s.point_light((1.5, 1.5, 1.5), (3.0, 3.0, 3.0))
    rd = scenes.render_desc(rd.camera, capi.INTEGRATOR_PATH, 8, 6, 0.8, capi.LIGHTS_POWER, capi.SAMPLER_HALTON)
    out["path_power_strategy"] = (s, rd)

    s, rd = scenes.config_c4(64, 36, 16, mesh=m)
    out["c4_glass_metal_plastic"] = (s, halton(rd))

    s, rd = scenes.config_c5(48, 27, 16, mesh=m)
    out["c5_volpath_medium"] = (s, halton(rd))

    # Oren-Nayar matte, anisotropic metal on a UV mesh (dpdu from the UVs), two-sided area light
    s = scenes.Scene()
    P, I, UV = uv_patch()
    s.mesh(P, I, s.metal(rough=0.3, urough=0.05, vrough=0.4, remap=True), uv=UV)
    s.mesh(m[0], m[1], s.matte((0.5, 0.6, 0.3), sigma=20.0))
    Pl, Il = scenes.quad(1.8, 0.8, flip=True)
    s.area_light_mesh(Pl, Il, (4.0, 4.0, 4.0), s.matte((0.5, 0.5, 0.5)), n_samples=2, two_sided=True)
    s.point_light((-1.0, 1.5, 1.5), (3.0, 3.0, 3.0))
    out["path_oren_nayar_aniso_metal"] = (s, scenes.render_desc(scenes.camera(48, 27, **CAM_C), capi.INTEGRATOR_PATH, 16, 6))

    # InfiniteAreaLight: non-power-of-two map (Lanczos resample), rotated as main.cpp does
    env = scenes.rgbe_roundtrip(scenes.procedural_sky(100, 50, seed=3))
    for integ, name, spp in ((capi.INTEGRATOR_WHITTED, "whitted", 4), (capi.INTEGRATOR_PATH, "path", 8)):
        s = scenes.Scene()
        s.mesh(m[0], m[1], s.plastic())
        Pf, If = scenes.quad(-1.12, 6.0)
        s.mesh(Pf, If, s.matte((0.6, 0.6, 0.6)))
        s.infinite_light(env, L=(1.0, 1.0, 1.0), xform=inf_xform(), n_samples=4)
        out[f"{name}_infinite_area_light"] = (s, scenes.render_desc(scenes.camera(40, 24, **CAM_C), integ, spp, 5))

    # a material-less closed box bounding a medium (pbrt's interface idiom) around a matte dragon
    s = scenes.Scene()
    med = s.homogeneous_medium(0.3, 1.2, 0.4)
    s.mesh(m[0], m[1], s.matte((0.8, 0.5, 0.2)))
    Pb, Ib = box((-1.3, -1.05, -1.3), (1.3, 1.3, 1.3))
    s.mesh(Pb, Ib, -1, medium_inside=med, medium_outside=-1)
    Pf, If = scenes.quad(-1.12, 6.0)
    s.mesh(Pf, If, s.matte((0.7, 0.7, 0.7)))
    Pl, Il = scenes.quad(2.45, 1.4, flip=True)
    s.area_light_mesh(Pl, Il, (6.0, 6.0, 6.0), s.matte((0.5, 0.5, 0.5)), n_samples=2)
    out["volpath_medium_box_interface"] = (s, scenes.render_desc(scenes.camera(40, 24, **CAM_C), capi.INTEGRATOR_VOLPATH, 16, 8))

    # ImageTexture (Texture/ImageTexture.cpp): RGB and float textures, non-power-of-two images
    # (Lanczos resample), the three wrap modes, gamma / scale, UVMapping2D offsets, mesh UVs and the
    # default triangle UVs, and GetTexture's grey substitute for a missing image
    for integ, name, spp, depth in ((capi.INTEGRATOR_WHITTED, "whitted", 4, 5), (capi.INTEGRATOR_PATH, "path", 8, 5)):
        s = scenes.Scene()
        P, I, UV = uv_patch()
        img_a = scenes.rgbe_roundtrip(texture_image(37, 23, seed=1))
        img_b = scenes.rgbe_roundtrip(texture_image(16, 8, seed=2))
        img_c = scenes.rgbe_roundtrip(texture_image(21, 30, seed=3))
        ta = s.image_texture(img_a, wrap=capi.WRAP_REPEAT, mapping=(2.0, 1.5, 0.1, -0.2))
        tb = s.image_texture(img_b, wrap=capi.WRAP_CLAMP, gamma=True, scale=0.8)
        tc = s.image_texture(img_c, wrap=capi.WRAP_BLACK, mapping=(1.3, 1.1, -0.15, 0.05))
        tr = s.image_texture(img_c, is_float=True, scale=0.3, wrap=capi.WRAP_REPEAT, mapping=(3.0, 2.0, 0.0, 0.0))
        ts = s.image_texture(img_b, is_float=True, scale=25.0, wrap=capi.WRAP_CLAMP, trilinear=True)
        tg = s.image_texture(None, scale=1.6, gamma=True)
        floor = s.set_texture(s.matte((0.5, 0.5, 0.5)), capi.TEX_KD, ta)
        s.set_texture(floor, capi.TEX_SIGMA, ts)
        s.mesh(P, I, floor, uv=UV)
        dragon = s.set_texture(s.plastic((0.3, 0.3, 0.3), (0.2, 0.2, 0.2), rough=0.2, remap=True), capi.TEX_KD, tb)
        s.set_texture(dragon, capi.TEX_KS, tc)
        s.set_texture(dragon, capi.TEX_ROUGHNESS, tr)
        s.mesh(m[0], m[1], dragon)
        Pm, Im = scenes.quad(1.9, 4.0, flip=True)
        s.mesh(Pm, Im, s.set_texture(s.mirror((0.9, 0.9, 0.9)), capi.TEX_KR, tc))
        Pg, Ig = box((0.9, -0.9, 0.4), (1.4, -0.2, 0.9))
        glass = s.set_texture(s.glass(eta=1.5, urough=0.0, vrough=0.0), capi.TEX_KT, tg)
        s.mesh(Pg, Ig, s.set_texture(glass, capi.TEX_KR, tb))
        if integ == capi.INTEGRATOR_PATH:
            Pl, Il = scenes.quad(1.8, 0.8, flip=True)
            s.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), s.matte((0.5, 0.5, 0.5)), n_samples=2)
        s.point_light((1.0, 1.5, 1.8), (5.0, 5.0, 5.0))
        out[f"{name}_image_textures"] = (s, scenes.render_desc(scenes.camera(40, 24, **CAM_C), integ, spp, depth))

    # two facing mirrors: deep Whitted recursion (maxDepth 12)
    s = scenes.Scene()
    s.mesh(m[0], m[1], s.matte((0.2, 0.7, 0.9)))
    Pa, Ia = scenes.quad(-1.12, 6.0)
    s.mesh(Pa, Ia, s.mirror((0.95, 0.9, 0.85)))
    Pb, Ib = scenes.quad(1.6, 6.0, flip=True)
    s.mesh(Pb, Ib, s.mirror((0.9, 0.95, 0.9)))
    s.point_light((0.3, 1.2, 1.5), (8.0, 8.0, 8.0))
    out["whitted_facing_mirrors_d12"] = (s, scenes.render_desc(scenes.camera(32, 20, **CAM_C), capi.INTEGRATOR_WHITTED, 4, 12))

    # an ingested mesh: tests/golden/mesh_small.3d through scenes.load_3d — the
    # generator checks that the reference's own reader (plyInfo, Shape/plyRead.h:22-47) returns the
    # same arrays — placed as main.cpp:332-348 does (TriangleMesh with an object-to-world translation)
    import os
    path3d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mesh_small.3d")
    V, F = scenes.load_3d(path3d)
    s = scenes.Scene()
    s.mesh(V, F, s.glass(), xform=scenes.translate(0.0, -0.35, 0.0))
    Pf, If = scenes.quad(-1.12, 6.0)
    s.mesh(Pf, If, s.matte((0.7, 0.7, 0.7)))
    Pl, Il = scenes.quad(2.45, 1.4, flip=True)
    s.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), s.matte((0.5, 0.5, 0.5)), n_samples=2)
    s.info["mesh_3d"] = path3d
    out["path_mesh_small_3d"] = (s, scenes.render_desc(scenes.camera(40, 24, **CAM_C), capi.INTEGRATOR_PATH, 16, 8, 0.8))

    # thin-lens cameras (Perspective.cpp:28-32,49-62): PerspectiveCamera with an aperture, pLens from
    # the sampler's dimensions 3-4 through ConcentricSampleDisk, focused behind / in front of the dragon
    for integ, name, spp, (lr, fd) in ((capi.INTEGRATOR_WHITTED, "whitted", 8, (0.08, 2.7)),
                                       (capi.INTEGRATOR_PATH, "path", 8, (0.15, 1.6))):
        s, rd = scenes.config_c2(40, 24, spp, mesh=m, sky=scenes.procedural_sky(64, 32)) if integ == capi.INTEGRATOR_WHITTED \
            else scenes.config_c3(40, 24, spp, mesh=m)
        cam = rd.camera
        cam.lens_radius, cam.focal_distance = lr, fd
        out[f"{name}_thin_lens"] = (s, scenes.render_desc(cam, integ, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                                                          capi.SAMPLER_HALTON))
    return out


def frame_cases():
    """name → (scene, render desc) rendered through the reference's own Integrator::Render (square)."""
    m = small_mesh(24)
    s, rd = scenes.config_c2(32, 32, 4, mesh=m, sky=scenes.procedural_sky(64, 32))
    out = {"frame_c2_whitted": (s, rd)}
    s, rd = scenes.config_c3(32, 32, 8, mesh=m)
    out["frame_c3_path"] = (s, halton(rd))
    return out


def default_chunk_starts(n_pixels, spp, integrator, max_depth, lanes=3):
    """First packed pixel of every chunk of the default wavefront schedule for a one-tile frame —
    wf_chunks (pysicalbasedraytracer_amd/csrc/pbr_kernels.hip, `WfChunks wf_chunks`): at most 2^25
    samples per Whitted chunk (fewer while levels x 36 B x 2^k > 8 GB), 2^26 for Path/VolPath; 24 or
    more chunks are equalised to a whole number per lane.  Parity tests pick the pixels either side
    of each boundary, where one lane's chunk hands over to the next."""
    if integrator == capi.INTEGRATOR_WHITTED:
        log2 = 25
        while log2 > 20 and max(1, max_depth) * 36.0 * (1 << log2) > 8e9:
            log2 -= 1
    else:
        log2 = 26
    chunk = max(1, (1 << log2) // spp)
    if chunk >= n_pixels:
        return [0]
    n = (n_pixels + chunk - 1) // chunk
    if n >= 24:
        n = max(lanes, n // lanes * lanes)
        chunk = (n_pixels + n - 1) // n
    return list(range(0, n_pixels, chunk))


def fullsize_pixels(width, height, n=1024, seed=0, boundaries=()):
    """n distinct pixels of a width x height raster as one-pixel tiles (x0, y0, x1, y1): the four
    corners, the centre, one on the area light, a jittered 4x4 grid over the whole frame and a
    jittered 6x7 grid over the dragon's part of the frame (x 0.38-0.65, y 0.2-0.62 of the raster,
    where the paths are longest) — the 64 pixels of round 5, kept first — then the two pixels either
    side of every chunk boundary of the default schedule (`boundaries`: packed row-major indices),
    then jittered 16x16 grids over the frame and 24x24 over the dragon until n, seeded."""
    rng = np.random.default_rng(seed)
    px = [(0, 0), (width - 1, 0), (0, height - 1), (width - 1, height - 1), (width // 2, height // 2),
          (width // 2, height // 50)]

    def grid(nx, ny, x0, x1, y0, y1):
        for j in range(ny):
            for i in range(nx):
                x = (x0 + (i + rng.uniform(0.1, 0.9)) * (x1 - x0) / nx) * width
                y = (y0 + (j + rng.uniform(0.1, 0.9)) * (y1 - y0) / ny) * height
                px.append((min(int(x), width - 1), min(int(y), height - 1)))

    grid(4, 4, 0.0, 1.0, 0.0, 1.0)
    grid(6, 7, 0.38, 0.65, 0.2, 0.62)
    for p0 in boundaries:
        for p in (p0 - 1, p0):
            if 0 <= p < width * height:
                px.append((p % width, p // width))
    while len(set(px)) < n:
        grid(16, 16, 0.0, 1.0, 0.0, 1.0)
        grid(24, 24, 0.38, 0.65, 0.2, 0.62)
    out, seen = [], set()
    for p in px:
        if p not in seen:
            seen.add(p)
            out.append(p)
    return [(x, y, x + 1, y + 1) for x, y in out[:n]]


FULLSIZE_PIXELS = 1024


def fullsize_cases():
    """name → (scene, render desc with one-pixel tiles): the BASELINE configs at their real size —
    the 100,352-triangle dragon stand-in, full raster, full spp, full depth — on 1024 pixels each,
    among them both sides of every chunk boundary of the benchmarked schedule.  C3 runs on the Halton
    sampler (the reference has no Sobol sampler, F3); C4 is 3840x2160 at 1024 spp.  The raster and
    spp fix the sample indices, so these are the benchmarked samples."""
    mesh = scenes.dragon_standin()
    mesh = (mesh[0], mesh[1], "standin:displaced-uv-sphere-224")
    out = {}
    for name, fn, seed in (("c2", scenes.config_c2, 2), ("c3_halton", scenes.config_c3, 3),
                           ("c4", scenes.config_c4, 4), ("c5", scenes.config_c5, 5)):
        s, rd = fn(mesh=mesh)
        cam = rd.camera
        starts = default_chunk_starts(cam.width * cam.height, rd.spp, rd.integrator, rd.max_depth)
        tiles = fullsize_pixels(cam.width, cam.height, n=FULLSIZE_PIXELS, seed=seed, boundaries=starts[1:])
        out[name] = (s, scenes.render_desc(cam, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold,
                                           rd.light_strategy, capi.SAMPLER_HALTON, tiles=tiles))
    return out


def bvh_cases():
    """name → scene for BVHAccel's node array and primitive order."""
    out = {}
    s = scenes.Scene()
    m = small_mesh(24)
    s.mesh(m[0], m[1], s.matte((0.5, 0.5, 0.5)))
    out["dragon_1152"] = s
    s4, _ = scenes.config_c4(8, 8, 1, mesh=small_mesh(20))
    out["c4_three_dragons"] = s4
    s = scenes.Scene()
    s.mesh(m[0], m[1], s.matte((0.5, 0.5, 0.5)))
    s.max_prims_in_node = 4
    out["dragon_1152_max4"] = s
    # the other SplitMethods (BVHAccel.cpp:136-158): Middle (std::partition at the centroid midpoint,
    # falling through to EqualCounts when one side is empty) and EqualCounts (std::nth_element);
    # HLBVH builds with SAH.  A grid of duplicated triangles makes Middle fall through.
    for name, split in (("middle", capi.SPLIT_MIDDLE), ("equal_counts", capi.SPLIT_EQUAL_COUNTS), ("hlbvh", capi.SPLIT_HLBVH)):
        s = scenes.Scene()
        s.mesh(m[0], m[1], s.matte((0.5, 0.5, 0.5)))
        Pq, Iq = scenes.quad(-1.2, 2.0)
        for k in range(3):
            s.mesh(Pq, Iq, s.matte((0.5, 0.5, 0.5)))
        s.split_method = split
        out[f"dragon_1152_{name}"] = s
    return out


def intersect_case():
    """A 1152-triangle mesh and 3000 seeded rays: towards random points, exactly at vertices and
    edge midpoints (the double-precision fallback of Triangle::Intersect), and along grazing lines."""
    m = small_mesh(24)
    s = scenes.Scene()
    s.mesh(m[0], m[1], s.matte((0.5, 0.5, 0.5)))
    rng = np.random.default_rng(99)
    P, I = m[0], m[1]
    n = 1000
    org = rng.normal(size=(3 * n, 3)).astype(np.float32)
    org = (org / np.linalg.norm(org, axis=1, keepdims=True) * 3.0).astype(np.float32)
    tgt_rand = rng.uniform(-1.1, 1.1, size=(n, 3)).astype(np.float32)
    tri = rng.integers(0, I.shape[0], n)
    tgt_vert = P[I[tri, rng.integers(0, 3, n)]]
    e0, e1 = rng.integers(0, 3, n), rng.integers(1, 3, n)
    tgt_edge = ((P[I[tri, e0]] + P[I[tri, (e0 + e1) % 3]]) * np.float32(0.5)).astype(np.float32)
    tgt = np.concatenate([tgt_rand, tgt_vert, tgt_edge])
    d = (tgt - org).astype(np.float32)
    tmax = np.full((3 * n, 1), np.inf, np.float32)
    tmax[::7] = 2.5   # some rays end before the surface
    rays = np.concatenate([org, d, tmax], axis=1).astype(np.float32)
    return s, rays


def camera_case():
    rng = np.random.default_rng(5)
    cams = [scenes.camera(48, 27, **CAM_C), scenes.camera(27, 48, (1.0, 2.0, -3.0), (0.2, 0.1, 0.0))]
    pf = [np.stack([rng.uniform(0, c.width, 32), rng.uniform(0, c.height, 32)], 1).astype(np.float32) for c in cams]
    return cams, pf


def canonical_nodes(nodes):
    """LinearBVHNode bytes with the bytes the reference leaves unwritten zeroed: `pad` always, and
    `axis` in leaves (flattenBVHTree sets it only for interior nodes; `new LinearBVHNode[n]` does
    not initialise, BVHAccel.cpp:82,261-283)."""
    a = np.array(nodes, dtype=np.uint8).reshape(-1, 32).copy()
    leaf = a[:, 28:30].copy().view("<u2").ravel() > 0
    a[:, 31] = 0
    a[leaf, 30] = 0
    return a.reshape(-1)


# ---------------------------------------------------------------- descriptor digests
def _arr(ptr, n, ctype):
    if not ptr or n <= 0:
        return b""
    return bytes(C.string_at(C.cast(ptr, C.c_void_p), n * C.sizeof(ctype)))


def _fields(h, st):
    """Hash a ctypes structure's values, skipping pointers (addresses differ run to run)."""
    for name, typ in st._fields_:
        v = getattr(st, name)
        if isinstance(typ, type) and issubclass(typ, (C._Pointer, C.c_void_p, C.c_char_p)) or typ is C.c_void_p:
            continue
        if name in ("n_bvh_nodes", "level0", "use_raster_to_camera") and v == 0:
            continue   # added after the fixtures were digested; hashed only when set
        if name == "raster_to_camera" and not st.use_raster_to_camera:
            continue
        if name == "abi_version":
            # the descriptor layout the fixtures were digested with: ABI v4 added an entry point
            # (pbr_hip_set_schedule), v5 fields that are hashed only when set, so scene digests
            # stay comparable
            v = 3
        if isinstance(v, C.Structure):
            _fields(h, v)
        elif isinstance(v, C.Array):
            h.update(bytes(memoryview(v)))
        else:
            h.update(f"{name}={v!r};".encode())


def scene_digest(scene, rd=None):
    """SHA-256 over everything the descriptors hand to a renderer (arrays included)."""
    h = hashlib.sha256()
    d = scene.desc()
    _fields(h, d)
    for i in range(d.n_shapes):
        sd = d.shapes[i]
        _fields(h, sd)
        h.update(_arr(sd.indices, 3 * sd.n_triangles, C.c_int32))
        h.update(_arr(sd.P, 3 * sd.n_vertices, C.c_float))
        h.update(_arr(sd.N, 3 * sd.n_vertices, C.c_float))
        h.update(_arr(sd.UV, 2 * sd.n_vertices, C.c_float))
    for i in range(d.n_materials):
        _fields(h, d.materials[i])
    for i in range(d.n_lights):
        ld = d.lights[i]
        _fields(h, ld)
        h.update(_arr(ld.env_data, ld.env_width * ld.env_height * ld.env_components, C.c_float))
    for i in range(d.n_media):
        _fields(h, d.media[i])
    for i in range(d.n_textures):
        td = d.textures[i]
        _fields(h, td)
        h.update(_arr(td.data, td.width * td.height * td.components, C.c_float))
    if rd is not None:
        for f in ("integrator", "spp", "max_depth", "rr_threshold", "light_strategy", "sampler"):
            h.update(f"{f}={getattr(rd, f)!r};".encode())
        _fields(h, rd.camera)
    return h.hexdigest()
