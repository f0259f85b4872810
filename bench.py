"""Headline benchmark: Msamples/s of the MI355X render path on BASELINE config C2
(1920×1080, 64 spp, WhittedIntegrator, dragon + mirror floor + SkyBox HDR), with the roofline of the
dominant kernel and the reference's own CPU path timed beside it.

One step = one full frame.  With --gpus N (launched by torch.distributed.run, one rank per GPU)
the frame's 32×32 tiles are dealt round-robin over ranks and rank 0 gathers the per-tile RGBA8
FrameBuffer spans over RCCL — total work is fixed, so scaling is strong.  The gather of frame k
runs on a communication stream while frame k+1 renders into the other of two output buffers.

Measurement windows (all after the warm-up frames):
  1. the timed region: K frames back to back, barrier + synchronize on both sides → `value`;
  2. K more frames with a HIP event pair around every kernel launch, on the stream it runs on
     (pbr_hip_set_profiling(1)) → per-kernel-family launch durations under the default schedule,
     where up to three chunk lanes run kernels concurrently (`roofline.kernels_overlapped`);
  3. one frame with work counters (pbr_hip_set_profiling(2)) → units and algorithmic HBM bytes per
     family (the compulsory queue / record / output bytes of the wavefront design);
  4. windows 2-3 again on the SERIAL schedule (pbr_hip_set_schedule serial: every launch on one
     stream, one after another) → each family's own launch durations (`roofline.kernels`).
`roofline.frame` is the whole frame of window 1: every family's algorithmic (and PMC) bytes per
frame over the frame time.  The roofline's top-level fields name the family with the largest
standalone time per frame: achieved = its algorithmic bytes per launch ÷ its own mean launch
duration (window 4); traffic = rocprofv3 PMC bytes per launch of the same family
(profiles/<config>_traffic.json, used only when measured on the very build that is loaded).
`--serial` runs every window on the serial schedule (the command whose rocprofv3 kernel stats back
the standalone durations, profiles/r4_*_kernel_stats.csv).

The CPU baseline (rank 0, N=1) runs FIRST, in a child process started before this process touches
the GPU: the reference itself (oracle/_ref/libpbr_ref.so, its unmodified sources built by
oracle/ref/Makefile) when that library is present — else the oracle/ restatement — on the physical
cores of socket 0 (lscpu), pinned one thread per core, OMP_PLACES=cores OMP_PROC_BIND=close, over
an evenly spread sample of the frame's rows; plus the reference's as-shipped 4 threads
(Integrator.cpp:282).
"""
import argparse
import json
import re
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E (MI355X_MICROARCH.md)
HBM_COPY_GBS = 6290.0        # measured device-to-device copy rate in the same guide
# The chip's VALU issue rate in wave64 instructions per second: 256 CUs x 4 SIMD-32 units, a wave64
# VALU instruction issues over 2 cycles, 2400 MHz (MI355X_MICROARCH.md, chip table and § Wave scheduling)
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2
# SURVEY §8(d) per-sample model (32 B per node test, 48 per primitive test, 96 per ray, 64 per
# shading event): reported for reference only — it counts cache-served BVH/mesh fetches as HBM
# bytes, so it is not a bound
B_NODE, B_PRIM, B_RAY, B_SHADE = 32, 48, 96, 64


# ------------------------------------------------------------------------------- CPU baseline
def cpu_topology():
    """Socket-0 physical cores (first logical CPU of each), allowed CPUs, cgroup CPU quota."""
    info = {"sockets": None, "physical_cores_socket0": None, "threads_per_core": None}
    cores0 = {}
    try:
        out = subprocess.run(["lscpu", "-p=CPU,CORE,SOCKET"], capture_output=True, text=True, check=True).stdout
        sockets, per_core = set(), {}
        for line in out.splitlines():
            if not line or line.startswith("#"):
                continue
            cpu, core, sock = (int(x) if x else 0 for x in line.split(","))
            sockets.add(sock)
            per_core[(sock, core)] = per_core.get((sock, core), 0) + 1
            if sock == 0:
                cores0.setdefault(core, cpu)
        info["sockets"] = len(sockets)
        info["physical_cores_socket0"] = len(cores0)
        info["threads_per_core"] = max(per_core.values()) if per_core else None
    except (OSError, subprocess.CalledProcessError, ValueError):
        pass
    allowed = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    info["allowed_cpus"] = len(allowed)
    info["cgroup_cpu_quota"] = quota
    pin = [c for c in sorted(cores0.values()) if c in allowed] or allowed
    n = len(pin)
    if quota is not None:
        n = max(1, min(n, int(quota)))
    info["threads"] = n
    info["pinned_cpus"] = pin[:n]
    return info


def cpu_baseline_worker(config, threads, budget_s, kind):
    """Child process: time the CPU render of an evenly spread sample of the frame's rows."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from pysicalbasedraytracer_amd import scenes
    if kind == "reference":
        import ref_lib as lib          # the reference itself (test infrastructure, oracle/_ref)
    else:
        import oracle_lib as lib       # the CPU restatement (test infrastructure, oracle/)
    scene, rd = scenes.CONFIGS[config]()
    if kind == "reference" and rd.sampler != 0:
        # the reference has no SobolSampler (F3): its HaltonSampler, same scene and spp
        rd = scenes.render_desc(rd.camera, rd.integrator, rd.spp, rd.max_depth, rd.rr_threshold, rd.light_strategy, 0)
    W, H, spp = rd.camera.width, rd.camera.height, rd.spp

    def run(rows):
        tiles = [(0, y, W, y + 1) for y in rows]
        rdc = scenes.render_desc(rd.camera, rd.integrator, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                                 rd.sampler, tiles=tiles)
        return lib.render(scene, rdc, threads=threads)[2]

    probe_rows = list(range(H // 2, H, max(1, H // 8)))[:4]
    t = run(probe_rows)
    per_row = max(t / len(probe_rows), 1e-4)
    n = int(max(4, min(H, budget_s / per_row)))
    stride = max(1, H // n)
    rows = list(range(stride // 2, H, stride))[:n]
    secs = run(rows)
    samples = len(rows) * W * spp
    return {"value": samples / secs / 1e6, "seconds": secs, "rows": len(rows), "row_stride": stride,
            "samples": samples}


def cpu_baseline(config, budget_s):
    topo = cpu_topology()
    kind = "reference" if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libpbr_ref.so")) else "port"
    out = {"unit": "Msamples/s", "kind": kind}
    legs = [("socket0", topo["threads"], topo["pinned_cpus"], budget_s), ("as_shipped_4", 4, topo["pinned_cpus"][:4], budget_s / 2)]
    for name, threads, cpus, b in legs:
        env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PLACES="cores", OMP_PROC_BIND="close",
                   OMP_DYNAMIC="false")
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-worker", "--config", config,
               "--threads", str(threads), "--budget", str(b), "--kind", kind]
        p = None
        try:
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=60 + 4 * b,
                               preexec_fn=(lambda c=cpus: os.sched_setaffinity(0, c)) if cpus else None)
            res = json.loads(p.stdout.strip().splitlines()[-1])
        except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
            res = {"error": f"{type(e).__name__}: {(p.stderr or '')[-300:] if p is not None else ''}"}
        res["threads"] = threads
        out[name] = res
    s0 = out["socket0"]
    out["value"] = s0.get("value")
    out["cores"] = topo["threads"]
    out["sockets"] = topo["sockets"]
    out["physical_cores"] = topo["physical_cores_socket0"]
    out["threads"] = topo["threads"]
    out["topology"] = {k: topo[k] for k in ("threads_per_core", "allowed_cpus", "cgroup_cpu_quota")}
    if s0.get("value") and topo["physical_cores_socket0"] and topo["threads"] < topo["physical_cores_socket0"]:
        # the job's CPU share is smaller than socket 0: linear scaling to all its physical cores, an
        # upper bound on what the reference could reach there (labelled, never used as `value`)
        out["socket0_linear_estimate"] = round(s0["value"] * topo["physical_cores_socket0"] / topo["threads"], 3)
    what = ("the reference's own code (oracle/_ref/libpbr_ref.so: its unmodified sources, SamplerIntegrator::"
            "Render's per-pixel body over the sampled rows)" if kind == "reference" else
            "the oracle/ CPU restatement")
    from pysicalbasedraytracer_amd import scenes
    if kind == "reference" and scenes.CONFIGS[config]()[1].sampler != 0:
        what += (", run with the reference's HaltonSampler in place of the Sobol sampler the GPU uses (the "
                 "reference ships the Sobol tables but no SobolSampler, F3); same scene, raster, spp and depth")
    limit = ""
    if topo["physical_cores_socket0"] and topo["threads"] < topo["physical_cores_socket0"]:
        limit = (f"; the job may use {topo['threads']} of socket 0's {topo['physical_cores_socket0']} physical cores "
                 f"(affinity {topo['allowed_cpus']} CPUs, cgroup quota {topo['cgroup_cpu_quota']})")
    out["sample"] = (f"{config}: {s0.get('rows')} rows (every {s0.get('row_stride')}th) × full width × spp = "
                     f"{s0.get('samples')} samples in {s0.get('seconds', 0):.1f} s, {what}, "
                     f"{topo['threads']} threads pinned one per physical core of socket 0, OMP_PLACES=cores "
                     f"OMP_PROC_BIND=close (no numactl in the image: memory is first-touch local){limit}")
    return out


# ------------------------------------------------------------------------------- GPU bench
def pmc_traffic(config, build_info):
    path = os.path.join(ROOT, "profiles", f"{config.lower()}_traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None, f"no PMC summary ({os.path.relpath(path, ROOT)})"
    if not t.get("build") or not build_info.endswith(t["build"]):
        return None, f"{os.path.relpath(path, ROOT)} is for build {t.get('build')}, not this one"
    return t, f"{os.path.relpath(path, ROOT)} ({t['method']})"


def kernel_family(name):
    """The profile family of a rocprof kernel name (template arguments stripped): k_wf_shade's CAMERA
    instances (4th template argument true) are the fused level-0 launches, family k_wf_shade_l0."""
    m = re.search(r"(k_\w+?)(<([^()]*)>)?(\(|$)", name)
    if not m:
        return None
    fam = m.group(1)
    if fam == "k_wf_shade" and m.group(3):
        targs = [a.strip() for a in m.group(3).split(",")]
        if len(targs) >= 4 and targs[3] == "true":
            fam = "k_wf_shade_l0"
    return fam


def family_counts(t, family):
    """SQ / TCC counts per frame of one kernel family (summed over its template instances), or None."""
    keys = ("valu_insts", "waves", "wave_cycles", "wait_any", "wait_inst_any", "active_inst_any", "tcc_hit", "tcc_miss")
    out, hit = dict.fromkeys(keys, 0.0), False
    for k, v in t["per_kernel"].items():
        if kernel_family(k) == family and "valu_insts" in v:
            for c in keys:
                out[c] += v.get(c, 0.0)
            hit = True
    return out if hit else None


def binding_bound(hbm_frac, issue_frac, wait_share):
    """The bound a family sits on: the larger of its HBM and VALU-issue fractions once either passes
    half of its peak; below that, 'latency' when its waves are parked on memory (s_waitcnt) for 40%
    or more of their cycles; else the larger fraction.  Returns (bound, fraction of that bound)."""
    h, i = hbm_frac or 0.0, issue_frac or 0.0
    if max(h, i) >= 0.5:
        return ("hbm", h) if h >= i else ("issue", i)
    if wait_share is not None and wait_share >= 0.4:
        return "latency", wait_share
    return ("hbm", h) if h >= i else ("issue", i)


def family_traffic(t, family):
    """PMC bytes per frame of one kernel family (rocprof names carry template arguments)."""
    rd = wr = 0.0
    hit = False
    for k, v in t["per_kernel"].items():
        if kernel_family(k) == family:
            rd += v["read_bytes"]
            wr += v["write_bytes"]
            hit = True
    return (rd + wr) if hit else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU render for the baseline")
    ap.add_argument("--no-model", action="store_true", help="skip the SURVEY-model counting pass")
    ap.add_argument("--serial", action="store_true", help="every window on the serial (one-stream) schedule")
    ap.add_argument("--per-frame", action="store_true",
                    help="one pbr_hip_render call per frame (a join between frames) instead of one batch per window")
    ap.add_argument("--cpu-baseline-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--threads", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--budget", type=float, default=10.0, help=argparse.SUPPRESS)
    ap.add_argument("--kind", default="reference", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_baseline_worker:
        print(json.dumps(cpu_baseline_worker(args.config, args.threads, args.budget, args.kind)), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline runs before this process initialises the GPU
    cpu = cpu_baseline(args.config, args.cpu_budget) if (world == 1 and not args.no_cpu_baseline) else None

    import numpy as np
    import torch
    import torch.distributed as dist
    from pysicalbasedraytracer_amd import FrameGather, HipRenderer, scenes, tiles_for_rank

    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    scene, rd = scenes.CONFIGS[args.config]()
    W, H, spp = rd.camera.width, rd.camera.height, rd.spp
    tiles = tiles_for_rank(W, H, rank, world) if world > 1 else [(0, 0, W, H)]
    rdr = scenes.render_desc(rd.camera, rd.integrator, spp, rd.max_depth, rd.rr_threshold, rd.light_strategy,
                             rd.sampler, tiles=tiles)
    npx = sum((t[2] - t[0]) * (t[3] - t[1]) for t in tiles)

    r = HipRenderer(local)
    if args.serial:
        r.set_schedule(serial=True)
    build_info = r.lib.pbr_hip_build_info().decode()
    t0 = time.time()
    r.upload(scene)
    upload_s = time.time() - t0

    # a real stream (torch's default one has handle 0, which the C-ABI reads as "context stream")
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    # multi-GPU: rank 0 gathers the packed RGBA8 tile spans (the FrameBuffer the reference's Render
    # fills) over RCCL; double-buffered outputs let the gather of frame k (communication stream)
    # overlap the render of frame k+1 (render stream)
    # one output pair per frame of a window: the frames of a window are one pbr_hip_render_frames
    # batch (their chunks continue one rotation over the lanes, no join between frames), so no frame
    # may overwrite a buffer an earlier frame's gather still reads
    nbuf = max(2 if world > 1 else 1, args.steps)
    rgbs = [torch.empty((npx, 3), dtype=torch.float32, device=dev) for _ in range(nbuf)]
    rgbas = [torch.empty((npx, 4), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    exchange = FrameGather(W, H, world, dev, channels=4, dtype=torch.uint8) if world > 1 else None
    comm = torch.cuda.Stream(dev) if world > 1 else None
    released = [None] * nbuf   # event: the gather that read buffer b has finished
    frame_no = [0]

    def render():
        b = frame_no[0] % nbuf
        frame_no[0] += 1
        if released[b] is not None:
            stream.wait_event(released[b])
        # asynchronous: the frame is enqueued on `stream` and the next one queues behind it
        r.render_device(rdr, rgbs[b].data_ptr(), rgbas[b].data_ptr(), stream=stream.cuda_stream, sync=False)
        if exchange is not None:
            rendered = torch.cuda.Event()
            rendered.record(stream)
            comm.wait_event(rendered)
            with torch.cuda.stream(comm):
                exchange(rgbas[b], rank)
                done = torch.cuda.Event()
                done.record(comm)
            released[b] = done

    def frames(k):
        """k frames as one batch (pbr_hip_render_frames); each frame's gather waits for that frame."""
        r.render_frames(rdr, [rgbs[f].data_ptr() for f in range(k)], [rgbas[f].data_ptr() for f in range(k)],
                        stream=stream.cuda_stream)
        if exchange is not None:
            for f in range(k):
                r.wait_frame(comm.cuda_stream, f)
                with torch.cuda.stream(comm):
                    exchange(rgbas[f], rank)
            stream.wait_stream(comm)

    def window(k):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if args.per_frame:
            for _ in range(k):
                render()
        else:
            frames(k)
        r.sync()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        if rank == 0:   # progress on stderr (the one JSON line is stdout's)
            print(f"[bench] {args.config}: {k} frame(s) in {el * 1e3:.1f} ms", file=sys.stderr, flush=True)
        return el

    for _ in range(args.warmup):
        render()
    r.sync()
    torch.cuda.synchronize(dev)
    # 1. the timed region
    elapsed = window(args.steps)
    # 2. per-kernel launch durations (HIP events on each launch's stream), same K frames
    r.set_profiling(1)
    elapsed_ev = window(args.steps)
    timing = r.get_profile()
    # 3. work counters of one frame (units, algorithmic bytes)
    r.set_profiling(2)
    window(1)
    counts = r.get_profile()
    r.set_profiling(0)
    # 4. the same on the serial schedule: each kernel family's own launch durations
    if args.serial:
        timing_s, counts_s, elapsed_s = timing, counts, elapsed_ev
    else:
        r.set_schedule(serial=True)
        render()
        r.sync()
        r.set_profiling(1)
        elapsed_s = window(args.steps)
        timing_s = r.get_profile()
        r.set_profiling(2)
        window(1)
        counts_s = r.get_profile()
        r.set_profiling(0)
        r.set_schedule()
    # SURVEY §8(d) model counts: the instrumented megakernel pass (binary traversal; same tests)
    model = None
    if not args.no_model:
        st = r.render_device(rdr, rgbs[0].data_ptr(), rgbas[0].data_ptr(), stream=stream.cuda_stream, stats=True)
        torch.cuda.synchronize(dev)
        samples_rank = npx * spp
        mb = B_NODE * st.node_visits + B_PRIM * st.prim_tests + B_RAY * st.rays + B_SHADE * st.shading_events
        model = {"bytes_per_sample": round(mb / samples_rank, 1),
                 "per_sample": {"rays": round(st.rays / samples_rank, 3), "node_tests": round(st.node_visits / samples_rank, 2),
                                "prim_tests": round(st.prim_tests / samples_rank, 3),
                                "shading_events": round(st.shading_events / samples_rank, 3)},
                 "formula": "32*node_tests + 48*prim_tests + 96*rays + 64*shading_events (SURVEY 8(d))",
                 "source": "instrumented megakernel pass (k_render<I,true,1>, binary traversal: the same "
                           "node/primitive tests BVHAccel performs)",
                 "note": "not a bound: counts every BVH-node and triangle fetch as HBM bytes, but the BVH and "
                         "mesh are served by L2 / Infinity Cache / scalar cache"}

    ms_per_step = elapsed / args.steps * 1e3
    value = W * H * spp / (elapsed / args.steps) / 1e6

    if rank == 0:
        pmc, pmc_src = pmc_traffic(args.config, build_info) if world == 1 else (None, "1 GPU only")

        def families(timing, counts):
            kernels = {}
            for fam, tv in timing.items():
                cv = counts.get(fam, {})
                lpf = tv["launches"] / args.steps                     # launches per frame
                avg_ms = tv["ms"] / max(1, tv["launches"])
                cl = cv.get("launches", 0) or 1
                alg_launch = cv.get("bytes", 0) / cl                  # algorithmic bytes per launch
                k = {"launches_per_frame": round(lpf, 2), "ms_per_frame": round(tv["ms"] / args.steps, 3),
                     "avg_launch_us": round(avg_ms * 1e3, 1), "units_per_frame": cv.get("units"),
                     "alg_bytes_per_launch": round(alg_launch), "counts_per_frame": cv.get("counts"),
                     "achieved_gbs": round(alg_launch / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else None}
                k["frac"] = round(k["achieved_gbs"] / HBM_PEAK_GBS, 4) if k["achieved_gbs"] is not None else None
                if pmc is not None:
                    fb = family_traffic(pmc, fam)
                    if fb is not None and lpf > 0:
                        k["traffic_per_launch"] = round(fb / lpf)
                        k["traffic_gbs"] = round(fb / lpf / (avg_ms * 1e-3) / 1e9, 1)
                        k["traffic_frac"] = round(k["traffic_gbs"] / HBM_PEAK_GBS, 4)
                    # the issue side (VALU wave-instructions per frame over this window's time per
                    # frame, against the chip's issue rate), the parked share of wave-cycles and
                    # the L2 hit rate, from the same build's SQ / TCC passes
                    cc = family_counts(pmc, fam)
                    if cc is not None and tv["ms"] > 0:
                        ms_frame = tv["ms"] / args.steps
                        k["valu_insts_per_frame"] = round(cc["valu_insts"])
                        k["valu_issue_frac"] = round(cc["valu_insts"] / (ms_frame * 1e-3) / VALU_ISSUE_PEAK, 4)
                        wc = cc["wave_cycles"] or 1.0
                        k["wait_any_share"] = round(cc["wait_any"] / wc, 3)
                        k["issue_stall_share"] = round(cc["wait_inst_any"] / wc, 3)
                        k["active_share"] = round(cc["active_inst_any"] / wc, 3)
                        if cc["tcc_hit"] + cc["tcc_miss"] > 0:
                            k["l2_hit"] = round(cc["tcc_hit"] / (cc["tcc_hit"] + cc["tcc_miss"]), 3)
                        b, f = binding_bound(k.get("traffic_frac", k["frac"]), k["valu_issue_frac"], k["wait_any_share"])
                        k["bound"] = b
                        k["bound_frac"] = round(f, 4)
                kernels[fam] = k
            return kernels

        kernels = families(timing_s, counts_s)          # standalone (serial schedule)
        overlapped = families(timing, counts)           # default schedule, lanes concurrent
        dom = max(kernels, key=lambda f: kernels[f]["ms_per_frame"]) if kernels else None
        dk = kernels.get(dom, {})
        # The whole frame of the timed schedule: every family's algorithmic (and PMC) bytes per frame
        # over the frame's wall time.
        fr_ms = elapsed / args.steps * 1e3
        alg_frame = sum(k["alg_bytes_per_launch"] * k["launches_per_frame"] for k in overlapped.values())
        frame = {"alg_bytes": round(alg_frame), "achieved_gbs": round(alg_frame / (fr_ms * 1e-3) / 1e9, 1),
                 "frac": round(alg_frame / (fr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "frame_ms": round(fr_ms, 3)}
        if pmc is not None:
            pmc_frame = sum(k.get("traffic_per_launch", 0) * k["launches_per_frame"] for k in overlapped.values())
            frame.update({"traffic": round(pmc_frame), "traffic_gbs": round(pmc_frame / (fr_ms * 1e-3) / 1e9, 1),
                          "traffic_frac": round(pmc_frame / (fr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "traffic_over_alg": round(pmc_frame / alg_frame, 3) if alg_frame else None})
        roofline = {"bound": "hbm", "kernel": dom, "achieved": dk.get("achieved_gbs"), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": dk.get("frac"), "traffic": dk.get("traffic_per_launch"),
                    "frame": frame,
                    "traffic_gbs": dk.get("traffic_gbs"), "traffic_frac": dk.get("traffic_frac"),
                    # what actually binds the dominant family (HBM bytes, VALU issue or memory
                    # latency) and at what fraction: `frac` above prices it against HBM only
                    "binding": ({"bound": dk["bound"], "frac": dk["bound_frac"], "hbm_frac": dk.get("traffic_frac", dk.get("frac")),
                                 "valu_issue_frac": dk.get("valu_issue_frac"), "wait_any_share": dk.get("wait_any_share"),
                                 "issue_stall_share": dk.get("issue_stall_share"), "l2_hit": dk.get("l2_hit"),
                                 "valu_issue_peak": VALU_ISSUE_PEAK,
                                 "rule": "hbm or issue when that fraction of its peak is >= 0.5 (the larger); below, "
                                         "latency when >= 0.4 of the wave-cycles are parked (SQ_WAIT_ANY); else the "
                                         "larger fraction"} if dk.get("bound") else None),
                    "copy_peak_gbs": HBM_COPY_GBS,
                    "frac_of_copy_peak": round(dk["achieved_gbs"] / HBM_COPY_GBS, 4) if dk.get("achieved_gbs") else None,
                    "alg_bytes_per_launch": dk.get("alg_bytes_per_launch"), "avg_launch_us": dk.get("avg_launch_us"),
                    "launches_per_frame": dk.get("launches_per_frame"), "ms_per_frame": dk.get("ms_per_frame"),
                    "definition": "frame = the timed schedule's whole frame: algorithmic HBM bytes per frame (compulsory "
                                  "queue/record/output bytes per counted unit, DESIGN.md 7, counted on the device) / frame "
                                  "time, PMC bytes likewise.  Top level = the kernel family with the most standalone time "
                                  "per frame: its algorithmic bytes per launch / its own mean launch duration (HIP events, "
                                  "serial schedule: one stream, no concurrent kernels); traffic = rocprofv3 PMC bytes per "
                                  "launch (FETCH_SIZE x2 + WRITE_SIZE)",
                    "traffic_source": pmc_src,
                    "serial_frame_ms": round(elapsed_s / args.steps * 1e3, 3),
                    "kernels": kernels,
                    "kernels_overlapped": {"window_ms_per_step": round(elapsed_ev / args.steps * 1e3, 3),
                                           "concurrency": round(sum(k["ms_per_frame"] for k in overlapped.values()) /
                                                                (elapsed_ev / args.steps * 1e3), 2),
                                           "families": overlapped},
                    "survey_model": model, "build": build_info}
        out = {
            "metric": "Msamples/sec (whole node) + wall-clock to 1080p/64spp frame; %HBM roofline",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"{args.config}: {W}x{H}, {spp} spp, "
                                   f"{['Whitted', 'Path', 'VolPath'][rd.integrator]} d{rd.max_depth}"
                                   f"{', Sobol' if rd.sampler == 1 else ''}",
                       "scene": scene.info.get("dragon", ""), "triangles": scene.info.get("triangles"),
                       "parallelism": (f"tiles32x32 round-robin over {world} GPUs, RCCL gather of RGBA8 spans"
                                       if world > 1 else "1 GPU, whole frame (no exchange)"),
                       "schedule": "serial (one stream)" if args.serial else "default (3 chunk lanes)",
                       "frame_ms": round(ms_per_step, 3), "scene_upload_s": round(upload_s, 3)},
            "roofline": roofline,
        }
        if cpu is not None:
            out["cpu_baseline"] = cpu
            if cpu.get("value"):
                out["gpu_over_cpu"] = round(value / cpu["value"], 1)
            if cpu.get("socket0_linear_estimate"):
                out["gpu_over_cpu_socket0_estimate"] = round(value / cpu["socket0_linear_estimate"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
