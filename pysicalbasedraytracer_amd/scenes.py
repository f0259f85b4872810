"""Scene descriptions for the BASELINE configs (C1..C5), built as the reference's `main.cpp` builds
them: a list of shapes (in `prims` order), materials, lights and media, flattened into the C-ABI
descriptor of include/pbr_hip.h.

Assets: the reference ships no Stanford Dragon and no .hdr.  `dragon_standin()` is
the deterministic ~100k-triangle displaced sphere of SURVEY §8(d) and `procedural_sky()` a
deterministic equirect HDR; `load_ply()` / `load_3d()` read the real Dragon when a file exists.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import struct

import numpy as np

from . import capi

f32 = np.float32


# ----------------------------------------------------------------------------- transforms
def identity():
    m = np.eye(4, dtype=f32)
    return m, m.copy()


def translate(dx, dy, dz):
    """Translate (Core/Transform.cpp:156-163): exact m and mInv."""
    m = np.eye(4, dtype=f32)
    mi = np.eye(4, dtype=f32)
    m[0, 3], m[1, 3], m[2, 3] = f32(dx), f32(dy), f32(dz)
    mi[0, 3], mi[1, 3], mi[2, 3] = -f32(dx), -f32(dy), -f32(dz)
    return m, mi


def scale(sx, sy, sz):
    """Scale (Core/Transform.cpp:164-169): mInv holds float reciprocals."""
    m = np.diag([f32(sx), f32(sy), f32(sz), f32(1)]).astype(f32)
    mi = np.diag([f32(1) / f32(sx), f32(1) / f32(sy), f32(1) / f32(sz), f32(1)]).astype(f32)
    return m, mi


def _rotate(axis, theta):
    """RotateX/Y/Z (Core/Transform.cpp): sin/cos of Radians(theta) in float (correctly rounded,
    pbr_math.h convention), mInv = Transpose(m)."""
    rad = f32(f32(f32(math.pi) / f32(180)) * f32(theta))   # Radians (PBR.h)
    st, ct = f32(math.sin(float(rad))), f32(math.cos(float(rad)))
    m = np.eye(4, dtype=f32)
    i, j = {"x": (1, 2), "y": (2, 0), "z": (0, 1)}[axis]
    m[i, i], m[i, j], m[j, i], m[j, j] = ct, -st, st, ct
    return m, np.ascontiguousarray(m.T)


def rotate_x(theta):
    return _rotate("x", theta)


def rotate_y(theta):
    return _rotate("y", theta)


def rotate_z(theta):
    return _rotate("z", theta)


def _mul(a, b):
    r = np.zeros((4, 4), dtype=f32)
    for i in range(4):
        for j in range(4):
            acc = f32(a[i, 0]) * f32(b[0, j])
            acc = f32(acc + f32(a[i, 1]) * f32(b[1, j]))
            acc = f32(acc + f32(a[i, 2]) * f32(b[2, j]))
            acc = f32(acc + f32(a[i, 3]) * f32(b[3, j]))
            r[i, j] = acc
    return r


def compose(t1, t2):
    """Transform::operator* (Transform.cpp:151-154)."""
    return _mul(t1[0], t2[0]), _mul(t2[1], t1[1])


def _xf(t):
    x = capi.Transform()
    for i in range(16):
        x.m[i] = float(t[0].flat[i])
        x.m_inv[i] = float(t[1].flat[i])
    return x


# ----------------------------------------------------------------------------- geometry
def dragon_standin(n=224, center=(0.0, 0.0, 0.0), radius=1.0):
    """Deterministic displaced UV sphere, (n+1) latitude rows × n longitudes → 2·n·n triangles
    (100,352 at n=224), SURVEY §8(d): r = 1 + 0.08·sin7θ·cos9φ + 0.03·sin(31θ+17φ)."""
    rows = n + 1
    th = np.linspace(0.0, math.pi, rows, dtype=np.float64)
    ph = np.linspace(0.0, 2 * math.pi, n + 1, dtype=np.float64)[:-1]
    T, Pp = np.meshgrid(th, ph, indexing="ij")
    r = radius * (1.0 + 0.08 * np.sin(7 * T) * np.cos(9 * Pp) + 0.03 * np.sin(31 * T + 17 * Pp))
    x = r * np.sin(T) * np.cos(Pp)
    y = r * np.cos(T)
    z = r * np.sin(T) * np.sin(Pp)
    P = np.stack([x + center[0], y + center[1], z + center[2]], axis=-1).reshape(-1, 3).astype(f32)
    idx = []
    for i in range(rows - 1):
        a = i * n + np.arange(n)
        b = i * n + (np.arange(n) + 1) % n
        c = (i + 1) * n + np.arange(n)
        d = (i + 1) * n + (np.arange(n) + 1) % n
        idx.append(np.stack([a, c, b], axis=1))
        idx.append(np.stack([b, c, d], axis=1))
    I = np.concatenate(idx, axis=0).astype(np.int32)
    # interleave to keep neighbouring triangles adjacent in prims order
    I = I.reshape(rows - 1, 2, n, 3).transpose(0, 2, 1, 3).reshape(-1, 3)
    return P, np.ascontiguousarray(I)


def quad(y, half, x0=0.0, z0=0.0, flip=False):
    """Two triangles in the plane y = const (Main/main.cpp:262-270 layout)."""
    P = np.array([[x0 - half, y, z0 + half], [x0 + half, y, z0 + half], [x0 - half, y, z0 - half],
                  [x0 + half, y, z0 + half], [x0 + half, y, z0 - half], [x0 - half, y, z0 - half]], dtype=f32)
    I = np.arange(6, dtype=np.int32).reshape(2, 3)
    if flip:
        I = I[:, ::-1].copy()
    return P, I


def load_3d(path):
    """The reference's `.3d` text mesh ("vertex N face M"; vertices ×20), Shape/plyRead.h:17-50."""
    toks = open(path).read().split()
    pos = 0
    nv = nf = 0
    for _ in range(2):
        key = toks[pos]; pos += 1
        if key == "vertex":
            nv = int(toks[pos]); pos += 1
        elif key == "face":
            nf = int(toks[pos]); pos += 1
    V = np.array(toks[pos:pos + 3 * nv], dtype=f32).reshape(nv, 3) * f32(20)
    pos += 3 * nv
    F = np.array(toks[pos:pos + 4 * nf], dtype=np.int64).reshape(nf, 4)[:, 1:].astype(np.int32)
    return V, F


def load_ply(path):
    """Minimal PLY reader (ascii and binary_little_endian; vertex x,y,z + triangle faces)."""
    with open(path, "rb") as fh:
        header = []
        while True:
            line = fh.readline().decode("ascii", "replace").strip()
            header.append(line)
            if line == "end_header":
                break
        fmt = [h for h in header if h.startswith("format")][0].split()[1]
        elements, cur = [], None
        for h in header:
            p = h.split()
            if not p:
                continue
            if p[0] == "element":
                cur = [p[1], int(p[2]), []]
                elements.append(cur)
            elif p[0] == "property" and cur is not None:
                cur[2].append(p[1:])
        tsize = {"char": "b", "uchar": "B", "int8": "b", "uint8": "B", "short": "h", "ushort": "H", "int16": "h",
                 "uint16": "H", "int": "i", "uint": "I", "int32": "i", "uint32": "I", "float": "f", "float32": "f",
                 "double": "d", "float64": "d"}
        V = F = None
        if fmt == "ascii":
            body = fh.read().decode("ascii").split()
            pos = 0
            for name, count, props in elements:
                if name == "vertex":
                    k = len(props)
                    arr = np.array(body[pos:pos + k * count], dtype=np.float64).reshape(count, k)
                    names = [p[-1] for p in props]
                    V = arr[:, [names.index("x"), names.index("y"), names.index("z")]].astype(f32)
                    pos += k * count
                elif name == "face":
                    faces = []
                    for _ in range(count):
                        nvtx = int(body[pos]); pos += 1
                        faces.append([int(t) for t in body[pos:pos + nvtx]]); pos += nvtx
                    F = _triangulate(faces)
                else:
                    pos += len(props) * count
        elif fmt == "binary_little_endian":
            for name, count, props in elements:
                if name == "vertex":
                    dt = np.dtype([(p[-1], "<" + tsize[p[0]]) for p in props])
                    arr = np.frombuffer(fh.read(dt.itemsize * count), dtype=dt)
                    V = np.stack([arr["x"], arr["y"], arr["z"]], axis=1).astype(f32)
                elif name == "face":
                    lp = props[0]
                    cnt_fmt, idx_fmt = "<" + tsize[lp[1]], "<" + tsize[lp[2]]
                    cs, isz = struct.calcsize(cnt_fmt), struct.calcsize(idx_fmt)
                    faces = []
                    for _ in range(count):
                        nvtx = struct.unpack(cnt_fmt, fh.read(cs))[0]
                        faces.append(list(struct.unpack("<" + idx_fmt[1:] * nvtx, fh.read(isz * nvtx))))
                    F = _triangulate(faces)
                else:
                    raise ValueError("unsupported PLY element " + name)
        else:
            raise ValueError("unsupported PLY format " + fmt)
    return V, F


def _triangulate(faces):
    tris = []
    for f in faces:
        for k in range(1, len(f) - 1):
            tris.append([f[0], f[k], f[k + 1]])
    return np.array(tris, dtype=np.int32)


def find_dragon():
    """Returns (P, I, source) for the real Stanford Dragon if a file is present, else the stand-in."""
    for env in ("PBR_DRAGON_PLY",):
        p = os.environ.get(env)
        if p and os.path.exists(p):
            V, F = load_ply(p) if p.endswith(".ply") else load_3d(p)
            return V, F, p
    P, I = dragon_standin()
    return P, I, "standin:displaced-uv-sphere-224"


def rgbe_roundtrip(img):
    """What stbi_loadf returns for `img` written with stbi_write_hdr: each pixel in the .hdr
    format's shared-exponent RGBE bytes (stb_image_write's stbiw__linear_to_rgbe: frexp of the
    largest component, channels scaled by mantissa·256/max and truncated) decoded as byte·2^(E−136)
    (stb_image's stbi__hdr_convert).  The reference reads environment maps only from .hdr files
    (SkyBoxLight.cpp:19-24, InfiniteAreaLight.cpp:14-21), so a map it can see has these values; they
    survive another write/read unchanged."""
    img = np.asarray(img, dtype=f32)
    e = img.reshape(-1, img.shape[-1])
    mx = e[:, :3].max(axis=1)
    out = np.zeros_like(e)
    ok = mx >= f32(1e-32)
    mant, ex = np.frexp(mx[ok])
    norm = (mant.astype(f32) * f32(256.0) / mx[ok]).astype(f32)
    b = np.floor((e[ok, :3] * norm[:, None]).astype(f32)).astype(np.float64)
    out[ok, :3] = (b * np.ldexp(1.0, ex - 8)[:, None]).astype(f32)
    return np.ascontiguousarray(out.reshape(img.shape))


def procedural_sky(width=2048, height=1024, seed=7):
    """Deterministic equirect HDR (sky gradient + sun + cloud noise), rows bottom-up as
    stbi_loadf returns them after stbi_set_flip_vertically_on_load(true) (SkyBoxLight.cpp:20), with
    the values an .hdr file can hold (rgbe_roundtrip)."""
    rng = np.random.default_rng(seed)
    v = (np.arange(height, dtype=np.float64) + 0.5) / height          # 0 bottom .. 1 top
    u = (np.arange(width, dtype=np.float64) + 0.5) / width
    U, Vv = np.meshgrid(u, v)
    elev = (Vv - 0.5) * math.pi
    sky = np.stack([0.25 + 0.35 * Vv, 0.45 + 0.4 * Vv, 0.85 + 0.5 * Vv], axis=-1)
    ground = np.stack([0.25 + 0 * Vv, 0.22 + 0 * Vv, 0.2 + 0 * Vv], axis=-1)
    img = np.where((elev > 0)[..., None], sky, ground)
    # clouds: a few octaves of value noise
    cloud = np.zeros_like(U)
    for octave in range(5):
        f = 4 * 2 ** octave
        g = rng.random((f + 1, 2 * f + 1))
        gy, gx = Vv * f, U * 2 * f
        y0, x0 = np.floor(gy).astype(int), np.floor(gx).astype(int)
        ty, tx = gy - y0, gx - x0
        n = (g[y0, x0] * (1 - tx) * (1 - ty) + g[y0, x0 + 1] * tx * (1 - ty) + g[y0 + 1, x0] * (1 - tx) * ty
             + g[y0 + 1, x0 + 1] * tx * ty)
        cloud += n / 2 ** octave
    cloud = np.clip((cloud / 1.9 - 0.55) * 3.0, 0, 1) * (elev > 0.05)
    img = img * (1 - cloud[..., None]) + cloud[..., None] * np.array([1.4, 1.4, 1.45])
    # sun
    sd = np.hypot((U - 0.3) * 2, (Vv - 0.75))
    img += (np.exp(-(sd / 0.02) ** 2) * 40.0)[..., None] * np.array([1.0, 0.95, 0.85])
    return rgbe_roundtrip(img.astype(f32))


# ----------------------------------------------------------------------------- scene container
class Scene:
    """Reference-shaped scene: shapes are appended in `prims` order (main.cpp:247-348)."""

    def __init__(self):
        self.shapes, self.materials, self.lights, self.media, self.textures = [], [], [], [], []
        self._keep = []
        self.max_prims_in_node = 1
        self.split_method = capi.SPLIT_SAH
        self.info = {}

    # materials (Main/main.cpp:147-239 recipes)
    def matte(self, kd, sigma=0.0):
        m = capi.MaterialDesc(type=capi.MAT_MATTE)
        m.Kd[:] = [float(c) for c in kd]
        m.sigma = sigma
        self.materials.append(m)
        return len(self.materials) - 1

    def mirror(self, kr=(1.0, 1.0, 1.0)):
        m = capi.MaterialDesc(type=capi.MAT_MIRROR)
        m.Kr[:] = [float(c) for c in kr]
        self.materials.append(m)
        return len(self.materials) - 1

    def glass(self, kr=(0.98,) * 3, kt=(0.98,) * 3, eta=1.5, urough=0.1, vrough=0.1, remap=False):
        m = capi.MaterialDesc(type=capi.MAT_GLASS, eta=eta, uroughness=urough, vroughness=vrough,
                              remap_roughness=int(remap))
        m.Kr[:] = list(kr)
        m.Kt[:] = list(kt)
        self.materials.append(m)
        return len(self.materials) - 1

    def metal(self, eta=(0.2, 0.2, 0.8), k=(0.11, 0.11, 0.11), rough=0.15, urough=0.15, vrough=0.15, remap=False):
        m = capi.MaterialDesc(type=capi.MAT_METAL, roughness=rough, uroughness=urough, vroughness=vrough,
                              has_uv_roughness=1, remap_roughness=int(remap))
        m.metal_eta[:] = list(eta)
        m.metal_k[:] = list(k)
        self.materials.append(m)
        return len(self.materials) - 1

    def plastic(self, kd=(0.35, 0.12, 0.48), ks=None, rough=0.1, remap=True):
        if ks is None:
            ks = [float(f32(1) - f32(c)) for c in kd]
        m = capi.MaterialDesc(type=capi.MAT_PLASTIC, roughness=rough, remap_roughness=int(remap))
        m.Kd[:] = list(kd)
        m.Ks[:] = list(ks)
        self.materials.append(m)
        return len(self.materials) - 1

    def image_texture(self, image=None, is_float=False, scale=1.0, gamma=False, wrap=capi.WRAP_REPEAT,
                      trilinear=False, max_aniso=8.0, mapping=(1.0, 1.0, 0.0, 0.0)):
        """ImageTexture<RGBSpectrum, Spectrum> (or <float, float>) with UVMapping2D(su, sv, du, dv)
        (Texture/ImageTexture.h:43-91): `image` [h, w, c>=3] float32 as loadImage's stbi_loadf
        returns it (rows bottom-up), None → the 0.5 grey image GetTexture substitutes.  Returns its
        index for set_texture()."""
        t = capi.TextureDesc(is_float=int(is_float), scale=scale, gamma=int(gamma), wrap=wrap,
                             trilinear=int(trilinear), max_aniso=max_aniso)
        t.su, t.sv, t.du, t.dv = mapping
        if image is not None:
            img = np.ascontiguousarray(image, dtype=f32)
            t.height, t.width, t.components = img.shape
            t.data = capi.fptr(img)
            self._keep.append(img)
        self.textures.append(t)
        return len(self.textures) - 1

    def set_texture(self, material, slot, texture):
        """Make a material parameter (capi.TEX_KD / KS / KR / KT / SIGMA / ROUGHNESS) read an image texture."""
        self.materials[material].tex[slot] = texture + 1
        return material

    def homogeneous_medium(self, sigma_a, sigma_s, g):
        md = capi.MediumDesc(g=g)
        md.sigma_a[:] = [float(sigma_a)] * 3 if np.isscalar(sigma_a) else list(sigma_a)
        md.sigma_s[:] = [float(sigma_s)] * 3 if np.isscalar(sigma_s) else list(sigma_s)
        self.media.append(md)
        return len(self.media) - 1

    # shapes
    def mesh(self, P, I, material, xform=None, reverse=False, area_light_first=-1, uv=None,
             medium_inside=-1, medium_outside=-1):
        P = np.ascontiguousarray(P, dtype=f32)
        I = np.ascontiguousarray(I, dtype=np.int32)
        s = capi.ShapeDesc(type=capi.SHAPE_TRIANGLE_MESH)
        s.object_to_world = _xf(xform or identity())
        s.reverse_orientation = int(reverse)
        s.n_triangles = I.shape[0]
        s.n_vertices = P.shape[0]
        s.indices = capi.iptr(I)
        s.P = capi.fptr(P)
        if uv is not None:
            uv = np.ascontiguousarray(uv, dtype=f32)
            s.UV = capi.fptr(uv)
            self._keep.append(uv)
        s.material = material
        s.area_light_first = area_light_first
        s.medium_inside, s.medium_outside = medium_inside, medium_outside
        self._keep += [P, I]
        self.shapes.append(s)
        return len(self.shapes) - 1

    def sphere(self, center, radius, material, reverse=False, medium_inside=-1, medium_outside=-1):
        s = capi.ShapeDesc(type=capi.SHAPE_SPHERE)
        s.object_to_world = _xf(translate(*center))
        s.reverse_orientation = int(reverse)
        s.radius = radius
        s.material = material
        s.area_light_first = -1
        s.medium_inside, s.medium_outside = medium_inside, medium_outside
        self.shapes.append(s)
        return len(self.shapes) - 1

    # lights
    def point_light(self, pos, I):
        l = capi.LightDesc(type=capi.LIGHT_POINT, n_samples=1, medium_inside=-1, medium_outside=-1)
        l.light_to_world = _xf(translate(*pos))
        l.I[:] = [float(c) for c in I]
        self.lights.append(l)
        return len(self.lights) - 1

    def area_light_mesh(self, P, I, Le, material, n_samples=1, two_sided=False, xform=None):
        """One DiffuseAreaLight per triangle, pushed in order (main.cpp:367-375)."""
        first = len(self.lights)
        shape = self.mesh(P, I, material, xform=xform, area_light_first=first)
        for t in range(np.asarray(I).shape[0]):
            l = capi.LightDesc(type=capi.LIGHT_DIFFUSE_AREA, shape=shape, triangle=t, two_sided=int(two_sided),
                               n_samples=n_samples, medium_inside=-1, medium_outside=-1)
            l.light_to_world = _xf(xform or identity())
            l.Le[:] = [float(c) for c in Le]
            self.lights.append(l)
        return shape

    def skybox(self, env, world_center=(0.0, 0.0, 0.0), world_radius=100.0, n_samples=1):
        env = np.ascontiguousarray(env, dtype=f32)
        l = capi.LightDesc(type=capi.LIGHT_SKYBOX, n_samples=n_samples, medium_inside=-1, medium_outside=-1)
        l.light_to_world = _xf(identity())
        l.world_center[:] = list(world_center)
        l.world_radius = world_radius
        l.env_height, l.env_width, l.env_components = env.shape
        l.env_data = capi.fptr(env)
        self._keep.append(env)
        self.lights.append(l)
        return len(self.lights) - 1

    def infinite_light(self, env=None, L=(1.0, 1.0, 1.0), xform=None, n_samples=1):
        """InfiniteAreaLight(LightToWorld, power L, nSamples, texmap) (Light/InfiniteAreaLight.cpp:7-61):
        env = the image as stbi_loadf returned it (rows × cols × comps float), None → a constant L."""
        l = capi.LightDesc(type=capi.LIGHT_INFINITE_AREA, n_samples=n_samples, medium_inside=-1, medium_outside=-1)
        l.light_to_world = _xf(xform or identity())
        l.Le[:] = [float(c) for c in L]
        if env is not None:
            env = np.ascontiguousarray(env, dtype=f32)
            l.env_height, l.env_width, l.env_components = env.shape
            l.env_data = capi.fptr(env)
            self._keep.append(env)
        self.lights.append(l)
        return len(self.lights) - 1

    def desc(self):
        self._arrays = (
            (capi.ShapeDesc * max(1, len(self.shapes)))(*self.shapes),
            (capi.MaterialDesc * max(1, len(self.materials)))(*self.materials),
            (capi.LightDesc * max(1, len(self.lights)))(*self.lights),
            (capi.MediumDesc * max(1, len(self.media)))(*self.media),
            (capi.TextureDesc * max(1, len(self.textures)))(*self.textures),
        )
        d = capi.SceneDesc(abi_version=capi.ABI_VERSION, n_shapes=len(self.shapes), n_materials=len(self.materials),
                           n_lights=len(self.lights), n_media=len(self.media),
                           max_prims_in_node=self.max_prims_in_node, n_textures=len(self.textures),
                           split_method=self.split_method)
        d.textures = C.cast(self._arrays[4], C.POINTER(capi.TextureDesc))
        d.shapes = C.cast(self._arrays[0], C.POINTER(capi.ShapeDesc))
        d.materials = C.cast(self._arrays[1], C.POINTER(capi.MaterialDesc))
        d.lights = C.cast(self._arrays[2], C.POINTER(capi.LightDesc))
        d.media = C.cast(self._arrays[3], C.POINTER(capi.MediumDesc))
        if getattr(self, "bvh_nodes", None) is not None:   # a caller-built BVHAccel (pbr_scene_desc::bvh_nodes)
            nodes = np.ascontiguousarray(self.bvh_nodes, dtype=np.uint8)
            self._arrays = self._arrays + (nodes,)
            d.bvh_nodes = nodes.ctypes.data
            d.n_bvh_nodes = nodes.size // 32
        return d


def camera(width, height, eye, look, up=(0.0, 1.0, 0.0), fov=90.0):
    c = capi.CameraDesc(width=width, height=height, use_look_at=1, fov=fov, lens_radius=0.0, focal_distance=0.0,
                        medium=-1)
    c.eye[:], c.look[:], c.up[:] = list(eye), list(look), list(up)
    return c


def render_desc(cam, integrator, spp, max_depth, rr_threshold=1.0, light_strategy=capi.LIGHTS_UNIFORM,
                sampler=capi.SAMPLER_HALTON, tiles=None, sobol_matrices=None, sample_table=None):
    """sobol_matrices: optional uint32 array in SobolMatrices32 layout ([dims][52]); None → the
    library's built-in matrices.  sample_table: float32 [height, width, spp, dims] of a caller's
    sampler (capi.SAMPLER_TABLE)."""
    d = capi.RenderDesc(integrator=integrator, max_depth=max_depth, rr_threshold=rr_threshold,
                        light_strategy=light_strategy, sampler=sampler, spp=spp, camera=cam)
    if sample_table is not None:
        arr = np.ascontiguousarray(sample_table, dtype=np.float32)
        d.sample_table = arr.ctypes.data_as(C.POINTER(C.c_float))
        d.table_dims = arr.shape[-1]
        d._table_keep = arr
    if sobol_matrices is not None:
        arr = np.ascontiguousarray(sobol_matrices, dtype=np.uint32)
        d.sobol_matrices = arr.ctypes.data_as(C.POINTER(C.c_uint32))
        d.sobol_dims = arr.size // 52
        d._sobol_keep = arr
    if tiles:
        arr = (capi.Tile * len(tiles))(*[capi.Tile(*t) for t in tiles])
        d.n_tiles = len(tiles)
        d.tiles = C.cast(arr, C.POINTER(capi.Tile))
        d._tiles_keep = arr
    return d


# ----------------------------------------------------------------------------- BASELINE configs
def config_c1(width=256, height=256, spp=4):
    """C1: Whitted d5, 2 matte spheres + point light; background 0.8 grey (F4). SURVEY §8(d)."""
    s = Scene()
    m = s.matte((0.5, 0.5, 0.5))
    s.sphere((-1.0, 0.0, 0.0), 1.0, m)
    s.sphere((1.2, 0.0, -1.0), 1.0, m)
    s.point_light((0.0, 4.0, 4.0), (20.0, 20.0, 20.0))
    cam = camera(width, height, (0.0, 0.0, 5.0), (0.0, 0.0, 0.0))
    return s, render_desc(cam, capi.INTEGRATOR_WHITTED, spp, 5)


def _dragon(s, material, mesh=None, xform=None, **kw):
    P, I, src = mesh if mesh is not None else find_dragon()
    s.info["dragon"] = src
    s.info["triangles"] = int(I.shape[0])
    return s.mesh(P, I, material, xform=xform, **kw)


def config_c2(width=1920, height=1080, spp=64, mesh=None, sky=None):
    """C2: Whitted d5, matte green dragon on a mirror floor under a SkyBox (render_final_parallel.png)."""
    s = Scene()
    green = s.matte((0.0, 1.0, 0.0))
    mirror = s.mirror((1.0, 1.0, 1.0))
    _dragon(s, green, mesh)
    Pf, If = quad(-1.12, 40.0)
    s.mesh(Pf, If, mirror)
    s.skybox(procedural_sky() if sky is None else sky, world_radius=60.0)
    cam = camera(width, height, (0.0, 0.55, 2.6), (0.0, -0.25, 0.0))
    return s, render_desc(cam, capi.INTEGRATOR_WHITTED, spp, 5)


def config_c3(width=1920, height=1080, spp=256, mesh=None):
    """C3: Path d8 rr 0.8 'uniform', dragon + one-sided 2-triangle area light (Lemit 5, nSamples 5)."""
    s = Scene()
    white = s.matte((0.8, 0.8, 0.8))
    green = s.matte((0.0, 1.0, 0.0))
    _dragon(s, green, mesh)
    Pf, If = quad(-1.12, 6.0)
    s.mesh(Pf, If, white)
    Pl, Il = quad(2.45, 1.4, flip=True)
    s.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), white, n_samples=5)
    cam = camera(width, height, (0.0, 0.55, 2.6), (0.0, -0.25, 0.0))
    return s, render_desc(cam, capi.INTEGRATOR_PATH, spp, 8, rr_threshold=0.8, sampler=capi.SAMPLER_SOBOL)


def config_c4(width=3840, height=2160, spp=1024, mesh=None):
    """C4: Path, three dragons (glass / metal / plastic recipes of main.cpp:160-183,228-239)."""
    s = Scene()
    white = s.matte((0.8, 0.8, 0.8))
    glass, metal, plastic = s.glass(), s.metal(), s.plastic()
    for mat, dx in ((glass, -2.3), (metal, 0.0), (plastic, 2.3)):
        _dragon(s, mat, mesh, xform=translate(dx, 0.0, 0.0))
    Pf, If = quad(-1.12, 10.0)
    s.mesh(Pf, If, white)
    Pl, Il = quad(2.9, 1.8, flip=True)
    s.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), white, n_samples=5)
    cam = camera(width, height, (0.0, 1.2, 5.0), (0.0, -0.3, 0.0))
    return s, render_desc(cam, capi.INTEGRATOR_PATH, spp, 8, rr_threshold=0.8)


def config_c5(width=1920, height=1080, spp=512, mesh=None):
    """C5: VolPath d10 rr 1, glass dragon filled with HomogeneousMedium(σa 0.5, σs 4.4, g −0.5)."""
    s = Scene()
    white = s.matte((0.8, 0.8, 0.8))
    glass = s.glass()
    med = s.homogeneous_medium(0.5, 4.4, -0.5)
    _dragon(s, glass, mesh, medium_inside=med, medium_outside=-1)
    Pf, If = quad(-1.12, 6.0)
    s.mesh(Pf, If, white)
    Pl, Il = quad(2.45, 1.4, flip=True)
    s.area_light_mesh(Pl, Il, (5.0, 5.0, 5.0), white, n_samples=5)
    cam = camera(width, height, (0.0, 0.55, 2.6), (0.0, -0.25, 0.0))
    return s, render_desc(cam, capi.INTEGRATOR_VOLPATH, spp, 10, rr_threshold=1.0)


def config_c2_lights(width=1920, height=1080, spp=64, mesh=None):
    """C2 with two extra point lights (three lights): the multi-light Whitted schedule
    (k_wf_shade_ml).  Not a BASELINE config; used to time it against the megakernel."""
    s, rd = config_c2(width, height, spp, mesh)
    s.point_light((1.0, 2.0, 1.5), (6.0, 5.0, 4.0))
    s.point_light((-1.5, 1.0, 2.0), (3.0, 3.0, 6.0))
    return s, rd


CONFIGS = {"C1": config_c1, "C2": config_c2, "C3": config_c3, "C4": config_c4, "C5": config_c5,
           "C2L3": config_c2_lights}
