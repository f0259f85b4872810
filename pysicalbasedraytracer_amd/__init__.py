"""MI355X-native render path for the reference's per-pixel integrator loop.

`HipRenderer` is the Python face of the C-ABI (include/pbr_hip.h): upload a reference-shaped scene
(`scenes.Scene`), then `render()` runs Whitted/Path/VolPath on the GPU — the counterpart of
`Integrator::Render(const Scene&, double&)` (Integrator/Integrator.h:14).  The C++ host mirror of
the reference classes lives in include/pbr/ (see INTEGRATION.md).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import capi, scenes  # noqa: F401

__all__ = ["HipRenderer", "capi", "scenes", "tile_grid", "tiles_for_rank"]


class PbrError(RuntimeError):
    pass


class HipRenderer:
    def __init__(self, device: int = 0):
        self.lib = capi.load_library()
        self.ctx = C.c_void_p()
        rc = self.lib.pbr_hip_create(device, C.byref(self.ctx))
        if rc != capi.PBR_OK:
            raise PbrError(f"pbr_hip_create failed ({rc}); a GPU is required — there is no CPU fallback")

    def _check(self, rc, what):
        if rc != capi.PBR_OK:
            raise PbrError(f"{what} failed ({rc}): {self.lib.pbr_hip_last_error(self.ctx).decode()}")

    def sync(self):
        """Wait for asynchronous frames; raises if one stopped at a safety bound (pbr_hip_sync)."""
        self._check(self.lib.pbr_hip_sync(self.ctx), "sync")

    def close(self):
        if self.ctx:
            self.lib.pbr_hip_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload(self, scene: "scenes.Scene"):
        self._desc = scene.desc()
        self._desc.abi_version = self.lib.pbr_hip_abi_version()   # (an older A/B build: same descriptors)
        self._scene = scene
        self._check(self.lib.pbr_hip_upload_scene(self.ctx, C.byref(self._desc)), "upload_scene")

    @staticmethod
    def n_pixels(rdesc) -> int:
        if rdesc.n_tiles:
            return sum((rdesc.tiles[i].x1 - rdesc.tiles[i].x0) * (rdesc.tiles[i].y1 - rdesc.tiles[i].y0)
                       for i in range(rdesc.n_tiles))
        return rdesc.camera.width * rdesc.camera.height

    def render(self, rdesc, rgb=True, rgba=True, stats=False):
        """Returns (rgb float32 [n,3], rgba uint8 [n,4], RenderStats) in packed tile order."""
        n = self.n_pixels(rdesc)
        out_rgb = np.empty((n, 3), dtype=np.float32) if rgb else None
        out_rgba = np.empty((n, 4), dtype=np.uint8) if rgba else None
        st = capi.RenderStats()
        rdesc.outputs_on_device = 0
        rdesc.collect_stats = int(stats)
        self._check(self.lib.pbr_hip_render(self.ctx, C.byref(rdesc),
                                             out_rgb.ctypes.data if rgb else None,
                                             out_rgba.ctypes.data if rgba else None, C.byref(st)), "render")
        return out_rgb, out_rgba, st

    def render_device(self, rdesc, rgb_ptr: int, rgba_ptr: int, stream: int | None = None, stats=False,
                      sync=True):
        """Render straight into device buffers (e.g. torch tensors' data_ptr()) on `stream`.

        sync=False (and stats=False): the frame is only enqueued on `stream` — the caller
        synchronises — and None is returned; frames then run back to back on the device."""
        rdesc.outputs_on_device = 1
        rdesc.stream = stream
        rdesc.collect_stats = int(stats)
        st = capi.RenderStats() if (sync or stats) else None
        self._check(self.lib.pbr_hip_render(self.ctx, C.byref(rdesc), rgb_ptr or None, rgba_ptr or None,
                                            C.byref(st) if st is not None else None), "render")
        return st

    def render_frames(self, rdesc, rgb_ptrs, rgba_ptrs, stream: int | None = None):
        """n frames of one descriptor into device buffers (pbr_hip_render_frames): their chunks
        continue one rotation over the lanes with no join between frames.  Asynchronous; `stream`
        reaches its tail when every frame is done; wait_frame orders another stream after one."""
        rgb_ptrs, rgba_ptrs = list(rgb_ptrs or []), list(rgba_ptrs or [])
        if rgb_ptrs and rgba_ptrs and len(rgb_ptrs) != len(rgba_ptrs):
            raise ValueError(f"render_frames: {len(rgb_ptrs)} float outputs but {len(rgba_ptrs)} RGBA8 outputs")
        n = max(len(rgb_ptrs), len(rgba_ptrs))
        if n == 0:
            raise ValueError("render_frames: no output buffers")
        rgb = (C.c_void_p * n)(*[p or None for p in rgb_ptrs]) if rgb_ptrs else None
        rgba = (C.c_void_p * n)(*[p or None for p in rgba_ptrs]) if rgba_ptrs else None
        # the caller's descriptor is left as it was: the batch's settings go on a copy (its tile
        # pointer still refers to the caller's arrays, which rdesc keeps alive for this call)
        d = type(rdesc).from_buffer_copy(rdesc)
        d.outputs_on_device = 1
        d.stream = stream
        d.collect_stats = 0
        self._check(self.lib.pbr_hip_render_frames(self.ctx, C.byref(d), n, rgb, rgba), "render_frames")

    def wait_frame(self, stream: int | None, f: int):
        """Make `stream` wait for frame f of the last render_frames call (pbr_hip_wait_frame)."""
        self._check(self.lib.pbr_hip_wait_frame(self.ctx, stream, f), "wait_frame")

    def set_schedule(self, kernels=capi.KERNELS_AUTO, chunk_log2=0, lanes=0, fuse_camera=capi.FUSE_AUTO, serial=False):
        """How later frames are cut into launches (pbr_hip_set_schedule); no arguments = the measured
        default; serial=True runs every launch on the caller's stream in turn (measurement).  Results
        are the same bits under every schedule."""
        s = capi.Schedule(kernels, chunk_log2, lanes, fuse_camera, int(serial))
        self._check(self.lib.pbr_hip_set_schedule(self.ctx, C.byref(s)), "set_schedule")

    def set_profiling(self, on: bool = True):
        """Start (on) or stop a per-kernel measurement window (pbr_hip_set_profiling)."""
        self._check(self.lib.pbr_hip_set_profiling(self.ctx, int(on)), "set_profiling")

    def get_profile(self) -> dict:
        """Per kernel family of the window: launches, summed HIP-event ms, work units, algorithmic
        HBM bytes and raw counters (pbr_hip_get_profile); starts a new window."""
        arr = (capi.KernelProfile * 32)()
        n = C.c_int()
        self._check(self.lib.pbr_hip_get_profile(self.ctx, arr, 32, C.byref(n)), "get_profile")
        return {arr[i].name.decode(): {"launches": arr[i].launches, "ms": arr[i].ms, "units": int(arr[i].units),
                                       "bytes": int(arr[i].bytes), "counts": [int(c) for c in arr[i].counts]}
                for i in range(min(n.value, 32))}

    def get_bvh(self):
        nn, npr = C.c_int(), C.c_int()
        self._check(self.lib.pbr_hip_get_bvh(self.ctx, None, C.byref(nn), None, C.byref(npr)), "get_bvh")
        nodes = np.empty(nn.value * 32, dtype=np.uint8)
        ids = np.empty(npr.value, dtype=np.int32)
        self._check(self.lib.pbr_hip_get_bvh(self.ctx, nodes.ctypes.data, C.byref(nn), capi.iptr(ids), C.byref(npr)),
                    "get_bvh")
        return nodes, ids

    def set_bvh_build(self, where: int):
        """Which SAH builder the next upload runs: capi.BVH_BUILD_DEVICE (default) or BVH_BUILD_HOST."""
        self._check(self.lib.pbr_hip_set_bvh_build(self.ctx, where), "set_bvh_build")

    def bvh_build_info(self) -> dict:
        """The last upload's BVH build: builder, wall ms, device kernel ms (pbr_hip_bvh_build_info)."""
        w, ms, kms = C.c_int(), C.c_double(), C.c_double()
        self._check(self.lib.pbr_hip_bvh_build_info(self.ctx, C.byref(w), C.byref(ms), C.byref(kms)), "bvh_build_info")
        return {"where": "device" if w.value == capi.BVH_BUILD_DEVICE else "host", "ms": ms.value,
                "kernel_ms": kms.value}

    def build_bvh(self, prim_bounds, where=capi.BVH_BUILD_DEVICE, max_prims=1):
        """BVHAccel's SAH build over [n, 6] primitive world bounds (pbr_hip_build_bvh): returns
        (LinearBVHNode bytes [n_nodes*32], ordered prim ids, {"ms", "kernel_ms"})."""
        b = np.ascontiguousarray(prim_bounds, dtype=np.float32).reshape(-1, 6)
        n = b.shape[0]
        nodes = np.zeros(max(1, 2 * n - 1) * 32, dtype=np.uint8)
        ids = np.zeros(max(1, n), dtype=np.int32)
        nn = C.c_int()
        ms = (C.c_double * 2)()
        self._check(self.lib.pbr_hip_build_bvh(self.ctx, where, n, capi.fptr(b), max_prims, nodes.ctypes.data,
                                                C.byref(nn), capi.iptr(ids), ms), "build_bvh")
        return nodes[:nn.value * 32], ids[:n], {"ms": ms[0], "kernel_ms": ms[1]}

    def sampler_values(self, width, height, spp, queries, sampler=capi.SAMPLER_HALTON):
        q = np.ascontiguousarray(queries, dtype=np.int32).reshape(-1, 4)
        out = np.empty(q.shape[0], dtype=np.float32)
        self._check(self.lib.pbr_hip_sampler_values(self.ctx, sampler, width, height, spp, q.shape[0], capi.iptr(q),
                                                    capi.fptr(out)), "sampler_values")
        return out

    def sample_index(self, width, height, spp, px_py_sample, sampler=capi.SAMPLER_HALTON):
        """GlobalSampler::GetIndexForSample on the device: int64 [n]."""
        q = np.ascontiguousarray(px_py_sample, dtype=np.int32).reshape(-1, 3)
        out = np.empty(q.shape[0], dtype=np.int64)
        self._check(self.lib.pbr_hip_sample_index(self.ctx, sampler, width, height, spp, q.shape[0], capi.iptr(q),
                                                  out.ctypes.data_as(C.POINTER(C.c_int64))), "sample_index")
        return out

    def sample_dimensions(self, width, height, index, px_py_dim, sampler=capi.SAMPLER_HALTON):
        """GlobalSampler::SampleDimension(index, dim) on the device (pixel for Sobol's dims 0, 1): float32 [n]."""
        idx = np.ascontiguousarray(index, dtype=np.int64).reshape(-1)
        q = np.ascontiguousarray(px_py_dim, dtype=np.int32).reshape(-1, 3)
        assert idx.shape[0] == q.shape[0]
        out = np.empty(q.shape[0], dtype=np.float32)
        self._check(self.lib.pbr_hip_sample_dimensions(self.ctx, sampler, width, height, q.shape[0],
                                                       idx.ctypes.data_as(C.POINTER(C.c_int64)), capi.iptr(q),
                                                       capi.fptr(out)), "sample_dimensions")
        return out

    def camera_rays(self, cam, pfilm):
        pf = np.ascontiguousarray(pfilm, dtype=np.float32).reshape(-1, 2)
        out = np.empty((pf.shape[0], 6), dtype=np.float32)
        self._check(self.lib.pbr_hip_camera_rays(self.ctx, C.byref(cam), pf.shape[0], capi.fptr(pf), capi.fptr(out)),
                    "camera_rays")
        return out

    def query(self, rays, any_hit=False, prim=-1):
        """Scene::Intersect / IntersectP (prim >= 0: GeometricPrimitive::Intersect of that primitive)
        with the SurfaceInteraction fields of each hit: an array of capi.SurfaceHit."""
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 7)
        out = (capi.SurfaceHit * max(1, r.shape[0]))()
        self._check(self.lib.pbr_hip_query(self.ctx, r.shape[0], capi.fptr(r), int(any_hit), int(prim), out), "query")
        return out[:r.shape[0]]

    def bounds(self, prim=-1):
        """Scene::WorldBound (prim = -1) or GeometricPrimitive::WorldBound: (lo[3], hi[3])."""
        b = np.empty(6, dtype=np.float32)
        self._check(self.lib.pbr_hip_bounds(self.ctx, int(prim), capi.fptr(b)), "bounds")
        return b[:3], b[3:]

    def li(self, rdesc, rays, px_py_sample_dim, depth=0):
        """SamplerIntegrator::Li on the device for caller-given rays: float32 [n, 3]."""
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 7)
        q = np.ascontiguousarray(px_py_sample_dim, dtype=np.int32).reshape(-1, 4)
        assert q.shape[0] == r.shape[0]
        out = np.empty((r.shape[0], 3), dtype=np.float32)
        self._check(self.lib.pbr_hip_li(self.ctx, C.byref(rdesc), r.shape[0], capi.fptr(r), capi.iptr(q), int(depth),
                                        capi.fptr(out)), "li")
        return out

    def intersect(self, rays, any_hit=False):
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 7)
        out = np.empty((r.shape[0], 5), dtype=np.float32)
        self._check(self.lib.pbr_hip_intersect(self.ctx, r.shape[0], capi.fptr(r), capi.fptr(out), int(any_hit)),
                    "intersect")
        return out


# Edge of the multi-GPU tiles.  Per-rank frame of an 8-GPU C2 job (slowest of 8 ranks, one GPU,
# tools/shard_sweep.sh): 64 → 3.14 ms, 32 → 3.07, 16 → 3.02; 32 keeps the tile list short.
TILE = 32


def tile_grid(width, height, tile=TILE):
    """TILE×TILE (32×32) pixel tiles in row-major order (SURVEY §8(e) suggests 64×64; 32×32 measured
    better, see the TILE comment)."""
    return [(x, y, min(x + tile, width), min(y + tile, height))
            for y in range(0, height, tile) for x in range(0, width, tile)]


def tiles_for_rank(width, height, rank, world, tile=TILE):
    """Round-robin tile ownership `tileId mod nGPU` so heavy regions spread over ranks."""
    return [t for i, t in enumerate(tile_grid(width, height, tile)) if i % world == rank]


def assemble(width, height, tiles, packed, channels):
    """Scatter a packed per-tile buffer back into a row-major frame."""
    frame = np.zeros((height, width, channels), dtype=packed.dtype)
    pos = 0
    for (x0, y0, x1, y1) in tiles:
        n = (x1 - x0) * (y1 - y0)
        frame[y0:y1, x0:x1] = packed[pos:pos + n].reshape(y1 - y0, x1 - x0, channels)
        pos += n
    return frame


def span_pixels(width, height, rank, world, tile=TILE):
    """Pixels in rank's packed span (the sum of its tiles' areas)."""
    return sum((t[2] - t[0]) * (t[3] - t[1]) for t in tiles_for_rank(width, height, rank, world, tile))


class FrameGather:
    """Multi-GPU exchange.  Every rank holds its tiles' packed span — float linear
    RGB [npx, 3] (the F7 float buffer) or the RGBA8 FrameBuffer bytes [npx, 4] uint8 (what the
    reference's Render writes, Integrator.cpp:327-344) — as a torch tensor on its device, or on
    the CPU under gloo.  One `gather` brings the spans to rank 0 (RCCL over xGMI under the nccl
    backend), padded to the largest span, and rank 0 scatters them into a row-major
    [height*width, channels] frame on its own device (index_copy_ with per-rank pixel indices
    computed once)."""

    def __init__(self, width, height, world, device, tile=TILE, channels=3, dtype=None):
        import torch
        dtype = torch.float32 if dtype is None else dtype
        self.world = world
        self.npx = [span_pixels(width, height, r, world, tile) for r in range(world)]
        self.max_px = max(self.npx)
        self.index = []
        for r in range(world):
            idx = [y * width + x for (x0, y0, x1, y1) in tiles_for_rank(width, height, r, world, tile)
                   for y in range(y0, y1) for x in range(x0, x1)]
            self.index.append(torch.tensor(idx, dtype=torch.long, device=device))
        self.send = torch.zeros((self.max_px, channels), dtype=dtype, device=device)
        self.recv = [torch.empty_like(self.send) for _ in range(world)]
        self.frame = torch.zeros((height * width, channels), dtype=dtype, device=device)

    def __call__(self, span, rank, group=None):
        import torch.distributed as dist
        self.send[:span.shape[0]].copy_(span)
        dist.gather(self.send, gather_list=self.recv if rank == 0 else None, dst=0, group=group)
        if rank != 0:
            return None
        for r in range(self.world):
            self.frame.index_copy_(0, self.index[r], self.recv[r][:self.npx[r]])
        return self.frame


def gather_frame(span, width, height, rank, world, group=None, tile=TILE):
    """One-shot FrameGather: the assembled [height, width, channels] numpy frame on rank 0, None elsewhere."""
    ch = span.shape[1]
    g = FrameGather(width, height, world, span.device, tile, channels=ch, dtype=span.dtype)
    f = g(span, rank, group)
    return None if f is None else f.cpu().numpy().reshape(height, width, ch)
