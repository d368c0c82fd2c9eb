"""Benchmark: Mray/s + ms/frame on bunny-in-Cornell 1920x1080 @1024spp (BASELINE.json configs[2]).

One step = one full frame of the path-tracing hot path (render kernel over all pixels x spp,
every bounce's closest-hit traversal + BSDF scatter) followed, for N > 1, by one RCCL gather
of the ranks' rows to rank 0.  The frame is split into interleaved 8-row stripes across
the N ranks (stripe s -> rank s % N), so the total work is fixed as N grows ("strong").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5] [--spp S]
    torchrun --nproc-per-node N bench.py --gpus N ...

RNG mode (--rng): `sample` (default) draws each pixel-sample from its own XORWOW stream seeded
by Philox, so a frame is a set of independent (pixel, 16-sample block) tasks that persistent
waves take from a counter: every GPU gets an equal share.  `compat` reproduces the reference's
per-pixel curand_init(seed, pixel, 0) streams bit for bit; a pixel's 1024 samples are then one
sequential chain, and the slowest pixels (paths trapped under the bunny, ~40 rays each) bound
the frame at ~1.8 s however many GPUs share it.  At N = 1 the line also carries one compat frame
(`compat_mode`).  Both modes render the same image in distribution (tests/test_oracle.py).

Kernel (--kernel): `wide` (default) traverses the compressed 8-wide SAH tree nearest child
first and keeps the reference's closest hit by (t, the reference's tie order); `wavefront` walks
the binary LBVH in the reference's own order.  Both render the same image bit for bit.

Rank 0 prints one JSON line.  `value` = total closest-hit queries (counted in-kernel, all
ranks) / max-over-ranks wall time of the K timed frames.  `roofline.achieved` = algorithmic
bytes of the traversed tree (per node visit its child boxes and refs -- 56 B
binary, 80 B 8-wide compressed -- + 40 B per triangle test + 20 B per sphere test) / render-kernel
time from HIP events on the render stream, against the L2 ceiling (the tree is L2-resident; the
HBM fraction of the PMC traffic is reported beside it).  PMC-derived fields (traffic, VALU
instructions) come from the committed profiles of the SAME libpt.so build (`build_id`, sha256),
else null.  `cpu_baseline` = the CPU restatement (oracle/) on the host cores, rank 0 at N = 1 only,
on a bounded sample.  `interactive` (N = 1) = frames/s of the progressive interactive mode at
1 / 4 / 16 spp.  Every timed frame is compared with the reference-order kernel's frame (pixels
and rays).  The headline renders one frame at a time at every N, with the host-built wide tree
at every N (the same method for N = 1 and N = 8: the driver divides their ms_per_step).  The
`pipelined` figure beside it repeats the timed sequence with two frames in flight: consecutive
steps alternate between two films on two streams, so a frame's first waves overlap the previous
frame's tail (7 % of a 1/8 share).  (--frames-in-flight 2 makes that the headline; its roofline
launch duration is then taken from a warmup launch that ran alone.)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # first: libpt.so then binds to the HIP runtime torch loaded
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "path-tracer-cuda-opengl_amd", "python"))
import ptamd  # noqa: E402
import ptdist  # noqa: E402

METRIC = "Mray/s + ms/frame, bunny-in-Cornell 1920×1080 @1024spp, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md "HBM": HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0   # MI355X_MICROARCH.md "L2 (per XCD)": 4 MiB per XCD, ~34.5 TB/s aggregate
GATHER_CEILING_GBS = 16000.0   # tools/micro/chase.hip: dependent per-lane gathers of 64-B records, L2-resident
CONFIGS = {
    "c3": ("bunny_cornell", "bunny-in-Cornell (5,000 tris) 1920x1080 @1024spp depth 50 (C3)"),
    "c2": ("cornell", "Cornell box (32 tris) 800x800 @256spp depth 8 (C2)"),
    "c5": ("bunny_field", "1,043,312-tri bunny field 1920x1080 @512spp depth 16 (C5)"),
    "c4": ("bunny_cornell", "bunny-in-Cornell (5,000 tris) 1920x1080 @4096spp depth 50 (C4, the 8-GPU config)"),
    "c5x4": ("bunny_field_x4", "C5 at 4x the triangles: 840 half-size bunnies, 4,173,152 tris 1920x1080 @128spp "
                               "depth 16 (a flattened tree beyond the 256 MB Infinity Cache; not a BASELINE config)"),
    "c5i": ("bunny_field", "bunny field instanced: 5,000 tris stored once, 211 instances (1,043,312 tris placed) "
                           "1920x1080 @512spp depth 16 (C5, two-level tree)"),
}
INSTANCED = {"c5i"}
CONFIG_SPP = {"c4": 4096}
STRIPE = 8


def cpu_facts() -> dict:
    """The host the CPU baseline ran on: nproc (os.cpu_count(): every CPU of the machine), the CPUs
    this process may run on (affinity mask), the cgroup CPU quota if one is set, OMP_NUM_THREADS,
    and the CPU model (/proc/cpuinfo).  On the GPU pool a 1-GPU box is a share of a larger machine:
    os.cpu_count() counts the whole machine, the share (affinity / quota / OMP_NUM_THREADS) is what
    a process may use."""
    nproc = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):   # cgroup v2: "<quota> <period>" or "max <period>"
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
        except (OSError, ValueError):
            pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = allowed if quota is None else max(1, min(allowed, int(quota)))
    # the pool's per-box CPU share (a 1-GPU box gets 16 of its machine's CPUs; OMP_NUM_THREADS
    # says so there): one thread per CPU of that share
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp > 0:
        usable = min(usable, omp)
    return {"nproc": nproc, "cpus_allowed": allowed, "cgroup_cpu_quota": quota, "omp_num_threads": omp or None,
            "cpu_model": model, "usable_cpus": usable}


def cpu_baseline(preset, budget_s: float = 12.0, gpu_ref=None, spp: int = 0, legs=None) -> dict:
    """Oracle (scalar C++ port of the reference path, std::thread over rows) on a bounded sample:
    the full frame at 1 spp per pass, passes repeated until `budget_s` of CPU work.  One thread per
    CPU this process may use (the affinity mask / cgroup quota: on the GPU pool the box's share of
    its machine, whose nproc is larger -- both are recorded); the host's timing in the reference is
    std::clock around render (main.cu:469-476).  BASELINE.md section 4 asks for ms/frame at the
    config's sample count: `ms_per_frame_extrapolated` = the measured time of one 1-spp pass x spp
    (a pass is the whole frame at 1 spp; samples are independent, so time is linear in spp).
    Beside the rate: the CPU traversal's node visits and primitive tests per ray (binary LBVH, the
    reference's order) and the GPU's counts for the same scene (reference-order kernel and the wide
    kernel).  `legs`: {config: (preset, spp, budget_s)} -- the same measurement, shorter, on other
    BASELINE configurations."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    facts = cpu_facts()
    threads = int(os.environ.get("PT_CPU_THREADS", "0")) or facts["usable_cpus"]

    def leg(p, budget, spp_full):
        w, h = p.width, p.height
        nodes = oracle.build_lbvh(p.objects, oracle.morton_keys(p.objects), tight=True)
        rows = np.arange(h, dtype=np.int32)
        states = oracle.film_states(1, w, rows)
        cam = ptamd.camera_to_array(p.camera)
        rays = visits = tris = sphs = 0
        passes, t0 = 0, time.perf_counter()
        while True:
            _, st = oracle.render(p.objects, p.materials, nodes, cam, w, h, rows, 1, p.max_depth, states,
                                  nthreads=threads)
            rays += st.rays
            visits += st.node_visits
            tris += st.tri_tests
            sphs += st.sphere_tests
            passes += 1
            el = time.perf_counter() - t0
            if el >= budget:
                break
        return {"value": rays / el / 1e6, "unit": "Mray/s",
                "ms_per_frame_extrapolated": el / passes * spp_full * 1e3, "spp": spp_full,
                "sample": f"{p.name} {w}x{h}, {passes} pass(es) of 1 spp depth {p.max_depth} "
                          f"({rays} rays, {el:.1f} s), oracle/ scalar C++ on {threads} threads",
                "per_ray": {"cpu_node_visits": visits / max(rays, 1), "cpu_prim_tests": (tris + sphs) / max(rays, 1)}}

    out = leg(preset, budget_s, spp or preset.spp)
    out.update({"cores": threads, "threads": threads, "kind": "port",
                "ms_per_frame_note": "time of one 1-spp pass over the whole frame x the config's spp (the "
                                     "reference's own timing is std::clock around render, main.cu:469-476)"})
    out.update(facts)
    if gpu_ref:
        out["per_ray"].update(gpu_ref)
    if legs:
        out["legs"] = {k: leg(p, b, s) for k, (p, s, b) in legs.items()}
    return out


def build_id() -> str:
    """sha256 (16 hex digits) of the libpt.so this process loaded: the committed PMC profiles carry
    the id of the build they measured, and their counters are reported only for that build."""
    import hashlib
    with open(ptamd.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_entry(name: str, workload: str, spp: int, rng: str, kernel: str, build: str):
    """The committed rocprofv3 PMC figures (profiles/<name>.json, written by tools/collect_profile.py:
    one entry per workload) for exactly this workload, sample count, RNG mode, kernel AND library
    build; None otherwise -- counters of another build are never paired with this build's times."""
    try:
        entries = json.load(open(os.path.join(REPO, "profiles", name + ".json")))
    except (OSError, ValueError):
        return None
    for e in entries.get("entries", []):
        if (e.get("workload") == workload and e.get("spp") == spp and e.get("rng") == rng and
                e.get("kernel") == kernel and e.get("build_id") == build):
            return e
    return None


# VALU issue ceiling: 256 CUs x 4 SIMDs, each issuing one wave64 VALU instruction per 2 cycles
# (MI355X_MICROARCH.md: 32 lanes/cycle x 2) at the 2.4 GHz maximum clock
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2.0


def interactive(scene, preset, dev, stream, local, frames=(30, 20, 10), spps=(1, 4, 16)) -> dict:
    """The reference's second product mode (renderToGL, main.cu:489-528: camera movement via
    camera::processKeyboard, camera.h:41-56, then a frame rendered into an RGBA8 surface),
    made progressive: per display frame one camera move, the accumulation restarted
    (pt_film_clear), `spp` samples accumulated and converted to RGBA8 on the device
    (PT_OUT_RGBA8_SURFACE).  Frames are enqueued without host synchronisation (pt_render_ex
    without pt_stats); frames/s = frames / wall time from the first enqueue to the last frame
    done.  `fps_2_streams`: the same frames alternating between two films (double-buffered
    surfaces) on two streams, so that a frame's first waves start while the previous frame's
    last paths finish (throughput; each frame's latency stays `ms_per_frame`)."""
    w, h = preset.width, preset.height
    films = [ptamd.Film(w, h, 1, device=local), ptamd.Film(w, h, 1, device=local)]
    bufs = [torch.empty((w * h * 4,), dtype=torch.uint8, device=dev) for _ in range(2)]
    streams = [stream, torch.cuda.Stream(dev)]
    cam = ptamd.Camera.from_buffer_copy(bytes(preset.camera))
    out = {}
    for spp, n in zip(spps, frames):
        res = {}
        for pipes in (1, 2):
            for it in range(2):   # warm (tile order, allocations), then timed
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for k in range(n):
                    j = k % pipes
                    ptamd.camera_move(cam, (0, 2, 1, 3)[k % 4], 0.01)   # forward, left, back, right
                    films[j].clear(streams[j].cuda_stream)
                    ptamd.render(scene, films[j], cam, spp, preset.max_depth, out=bufs[j].data_ptr(),
                                 stream=streams[j].cuda_stream, rng=ptamd.RNG_SAMPLE, accumulate=True,
                                 out_format=ptamd.OUT_RGBA8_SURFACE, wait=False)
                torch.cuda.synchronize(dev)
                res[pipes] = time.perf_counter() - t0
            if pipes == 1:
                st = films[0].stats()   # (the sequential frames' counters and kernel time)
        out[f"{spp}spp"] = {"fps": n / res[1], "ms_per_frame": res[1] / n * 1e3, "frames": n,
                            "rays_per_frame": st.rays, "kernel_ms": st.kernel_ms, "fps_2_streams": n / res[2]}
    for f in films:
        f.close()
    return out


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--spp", type=int, default=0, help="override samples per pixel (0 = the config's)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--leaf-batch", type=int, default=0, help="wavefront LEAF threshold (0 = library default)")
    ap.add_argument("--shade-batch", type=int, default=0, help="wavefront SHADE threshold (0 = library default)")
    ap.add_argument("--rng", default="sample", choices=["compat", "sample"],
                    help="sample (default): a XORWOW stream per pixel-sample seeded by Philox, (pixel, block) "
                         "tasks on persistent waves -- the frame splits over any number of GPUs; compat: the "
                         "reference's per-pixel cuRAND-XORWOW streams (a pixel's 1024 samples are sequential)")
    ap.add_argument("--chunk", type=int, default=0, help="sample mode: summation block (0 = library default)")
    ap.add_argument("--no-compat", action="store_true", help="skip the compat-mode reference frame (N = 1)")
    ap.add_argument("--no-interactive", action="store_true",
                    help="skip the interactive-mode frames/s at 1 / 4 / 16 spp (N = 1)")
    ap.add_argument("--output", default="rgba8", choices=["rgba8", "f32"],
                    help="frame format rendered and gathered: rgba8 (default: quantised on the device like "
                         "PngImage::saveColor, 4 B/pixel on the wire) or f32 (linear-sqrt RGB, 12 B/pixel)")
    ap.add_argument("--png", default="", help="rank 0 writes the last (assembled) frame to this PNG")
    ap.add_argument("--frames-in-flight", type=int, default=0, choices=[0, 1, 2],
                    help="frames rendered concurrently on two streams for the headline (0 = 1 at every N)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the `pipelined` figure (the timed sequence again with two frames in flight)")
    ap.add_argument("--kernel", default="wide", choices=["wide", "wavefront"],
                    help="wide (default): the compressed 8-wide SAH tree, nearest child first; wavefront: the "
                         "binary LBVH in the reference's visiting order.  Same image either way")
    return ap


def main() -> None:
    args = make_parser().parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # nccl = RCCL over xGMI.  PT_DIST_BACKEND=gloo only rehearses the multi-rank flow (e.g. two
    # ranks sharing one GPU, frames gathered through host memory); it never produces a reported number.
    backend = os.environ.get("PT_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # PT_DIST_FORCE=1: the multi-rank path (process group, gather, barriers, reductions) even for
    # one rank -- a one-GPU box can run the RCCL gather of a real frame (never a reported number)
    dist_on = world > 1 or os.environ.get("PT_DIST_FORCE") == "1"
    if dist_on:
        # every collective times out (PT_DIST_TIMEOUT, default 120 s) and a rank that spends longer
        # than PT_BENCH_WATCHDOG s (default 600 for N > 1) in one phase dumps its stacks and exits
        ptdist.init(backend, rank, world, device=dev if backend == "nccl" else None,
                    timeout_s=float(os.environ.get("PT_DIST_TIMEOUT", "120")),
                    watchdog_s=float(os.environ.get("PT_BENCH_WATCHDOG", "600" if world > 1 else "0")))
        with ptdist.guarded():   # any failure on a rank ends it at once, naming rank and phase
            run(args, world, rank, local, backend, dev, dist_on)
    else:
        run(args, world, rank, local, backend, dev, dist_on)


def injected(rank: int, where: str) -> str:
    """Test hook (tests/test_gpu_zz_ranks.py): PT_BENCH_INJECT=<rank>:<where>:<kind> makes that
    rank fail at that point -- kind `raise` (an exception), `mismatch` (a frame check that fails) or
    `hang` (stops responding) -- to show that every rank then exits non-zero within the timeout."""
    spec = os.environ.get("PT_BENCH_INJECT", "")
    if not spec:
        return ""
    r, w, kind = spec.split(":")
    if int(r) != rank or w != where:
        return ""
    if kind == "raise":
        raise RuntimeError(f"injected failure on rank {rank} at {where}")
    if kind == "hang":
        time.sleep(10 ** 6)
    return kind


def run_settings(args, world: int) -> dict:
    """The method of a run, identical at every N unless a flag or knob says otherwise (the driver
    divides the N = 1 and N = 8 lines' ms_per_step; both must measure the same thing): one frame at
    a time, the wide tree from the host SAH build.  tests/test_host.py checks it for N = 1, 2, 8."""
    return {"frames_in_flight": args.frames_in_flight or 1,
            "wide_tree": "device" if os.environ.get("PT_BENCH_WIDE_DEVICE", "0") == "1" else "host"}


def run(args, world: int, rank: int, local: int, backend: str, dev, dist_on: bool) -> None:
    phase = ptdist.phase
    settings = run_settings(args, world)

    if world > 1 and "PT_BUILD_THREADS" not in os.environ:
        # the ranks of a node share its host cores: each rank's host wide-tree build (before the
        # timed frames) takes its share of them instead of 16 threads each
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        os.environ["PT_BUILD_THREADS"] = str(max(1, cpu_facts()["usable_cpus"] // max(1, local_world)))
    phase("scene build")
    name, workload = CONFIGS[args.config]
    instanced = args.config in INSTANCED
    if instanced and args.kernel != "wide":
        raise SystemExit("instanced scenes render with the wide kernel")
    preset = ptamd.InstancedPreset(name) if instanced else ptamd.Preset(name)
    spp = args.spp or CONFIG_SPP.get(args.config, preset.spp)
    w, h, depth = preset.width, preset.height, preset.max_depth
    if instanced:
        scene = ptamd.Scene.instanced(preset.objects, preset.mesh_first, preset.mesh_count, preset.instances,
                                      preset.materials, device=local)
        scene.build_bvh()
        scene_build = {"two_level_tree_host_ms": scene.build_ms, "device_bytes": scene.bvh_info()["device_bytes"]}
    else:
        # The same tree builder at every N (the driver's 1 -> 8 ratio compares one method): the host
        # SAH build (before the timed frames; with N > 1 each rank takes its share of the host cores,
        # PT_BUILD_THREADS).  PT_BENCH_WIDE_DEVICE=1 builds it on each rank's device instead (top-down
        # SAH of the host build's quality, C5 7 ms); the frames are the same either way (closest hits
        # do not depend on the tree).
        wide_dev = settings["wide_tree"] == "device"
        flags = ptamd.PT_BVH_ORIGIN_BOUNDS | (ptamd.PT_BVH_WIDE_DEVICE if wide_dev else 0)
        scene = ptamd.Scene(preset.objects, preset.materials, device=local, flags=flags)
        scene.build_bvh(flags)   # again: the first build in a process also pays one-time module loading
        scene_build = {"lbvh_device_ms" if not wide_dev else "lbvh_plus_wide_tree_device_ms": scene.build_ms}
    # Frames in flight (--frames-in-flight, default 1 at every N): with 2, consecutive steps
    # alternate between two films (and output buffers) on two streams, so a frame's first waves
    # start while the previous frame's last paths finish -- the launch's tail, 7 % of a 1/8 share of
    # C3 but 0.2 % of the whole frame (tools/pipe_frames.py).  The headline renders one frame at a
    # time at every N (one method for the driver's ratio; the render kernel's launches run alone, so
    # their HIP-event and rocprof durations are the frame's); the `pipelined` figure beside it is the
    # same sequence with two frames in flight.  Every frame is still rendered in full and checked
    # against the reference-order frame.
    films = [ptamd.Film(w, h, args.seed, device=local, stripe_height=STRIPE, n_parts=world, part=rank) for _ in range(2)]
    max_rows = ptdist.max_rows(h, STRIPE, world)
    rgba8 = args.output == "rgba8"
    chans, tdt = (4, torch.uint8) if rgba8 else (3, torch.float32)
    out_format = ptamd.OUT_RGBA8 if rgba8 else ptamd.OUT_RGB32F
    local_bufs = [torch.zeros((max_rows * w * chans,), dtype=tdt, device=dev) for _ in range(2)]
    ref_buf = torch.zeros_like(local_bufs[0])   # the reference-order kernel's frame (warmup step 1)
    gathered = [torch.empty((world * max_rows * w * chans,), dtype=tdt, device=dev) if dist_on and rank == 0 else None
                for _ in range(2)]
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    film, local_buf, stream = films[0], local_bufs[0], streams[0]   # (single-frame uses below)

    sample = args.rng == "sample"

    kernel_id = ptamd.KERNEL_WIDE if args.kernel == "wide" else ptamd.KERNEL_WAVEFRONT
    gather_ev = []   # (start, end) HIP events around each timed frame's gather (nccl), read after the loop
    gather_host_ms = [0.0]   # gloo rehearsal: host time of the gathers

    def frame(j, kernel=kernel_id, wait=False, timed=False):
        # every step renders the SAME frame: streams back to curand_init(seed, pixel, 0)
        # (sample mode is stateless: a pure function of seed, pixel and sample).  Film j, its
        # buffer and stream; wait=False enqueues it (films[j].stats() waits for it).
        f, buf, s = films[j], local_bufs[j], streams[j]
        if not sample:
            f.reset(s.cuda_stream)
        _, st = ptamd.render(scene, f, preset.camera, spp, depth, out=buf.data_ptr(),
                             stream=s.cuda_stream, kernel=kernel, leaf_batch=args.leaf_batch,
                             shade_batch=args.shade_batch, rng=ptamd.RNG_SAMPLE if sample else ptamd.RNG_COMPAT,
                             chunk=args.chunk, out_format=out_format, wait=wait)
        if dist_on:   # the frame's stripes to rank 0 (one gather; SURVEY 8(e) ncclGather), after it on its stream
            with torch.cuda.stream(s):
                if backend == "nccl":
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else None
                    if ev:
                        ev[0].record(s)
                    ptdist.gather_to_root(buf, world, rank, gathered[j])
                    if ev:
                        ev[1].record(s)
                        gather_ev.append(ev)
                else:   # (gloo: host staging; the gather's own time, not the render it waits for)
                    host = buf.cpu()
                    tg0 = time.perf_counter()
                    g = ptdist.gather_to_root(host, world, rank)
                    if rank == 0:
                        gathered[j].copy_(g)
                    if timed:
                        gather_host_ms[0] += (time.perf_counter() - tg0) * 1e3
        return st

    # Warmup 1 uses the ray-synchronous kernel, whose traversal follows the reference's node
    # order exactly: its counters give the frame's ALGORITHMIC bytes (the wavefront kernel may
    # visit a few extra nodes speculatively; those are not counted as useful work).  Both
    # kernels produce the identical frame (same rays, same primitive tests, same pixels).
    # (An instanced scene has only the wide kernel: its first frame is the one later frames equal.)
    phase("reference-order frame")
    ref_st = frame(0, ptamd.KERNEL_WIDE if instanced else ptamd.KERNEL_SIMPLE, wait=True)
    ref_buf.copy_(local_bufs[0])
    failed = []   # this rank's frames that differ from the reference-order frame

    def check(st, j, where):
        # every frame: this rank's pixels and ray count equal the reference-order frame's.  A
        # mismatch is recorded, not raised: all ranks learn of it together (agree) and exit with it.
        with torch.cuda.stream(streams[j]):
            same = torch.equal(local_bufs[j], ref_buf)
        if injected(rank, where) == "mismatch":
            same = False
        if st.rays != ref_st.rays or not same or (
                args.kernel == "wavefront" and (st.tri_tests != ref_st.tri_tests or
                                                st.sphere_tests != ref_st.sphere_tests)):
            failed.append(where)

    def agree(where):
        # every rank's checks so far; any failure ends EVERY rank with status 3 (N = 1: this rank)
        bad = ptdist.agree(not failed, dev if backend == "nccl" else "cpu") if dist_on else ([rank] if failed else [])
        if bad:
            raise SystemExit(f"frame differs from the reference-order frame on rank(s) {bad} ({where}; "
                             f"this rank: {failed or 'ok'})")

    def finish(j, where="timed frames"):
        st = films[j].stats()   # (waits for film j's frame)
        check(st, j, where)
        return st

    check(ref_st, 0, "reference-order frame")   # (also loads torch's comparison kernels before the timed region)
    fif = settings["frames_in_flight"]
    warm_kms = ref_st.kernel_ms
    phase("warmup frames")
    if fif == 2:
        st1 = frame(1, wait=True)   # (film 1's first launch: its tile costs for the launch order)
        check(st1, 1, "warmup frames")
        warm_kms = st1.kernel_ms
    # (the reference-order frame above counts as one warmup step; the benchmarked kernel gets at least
    # one warmup frame of its own, so its first use -- the wide tree's host build, module loading --
    # never falls into the timed region)
    for k in range(max(1, args.warmup - 1) if args.warmup > 0 else 0):
        stw = frame(k % fif, wait=True)
        check(stw, k % fif, "warmup frames")
        warm_kms = stw.kernel_ms
    if args.kernel == "wide" and not instanced and "lbvh_plus_wide_tree_device_ms" not in scene_build:
        scene_build["wide_tree_host_ms"] = scene.wide_info()["build_ms"]   # built at the first wide render (host SAH)
    agree("warmup")
    phase("timed frames")
    injected(rank, "timed")
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rays = kbytes = 0
    kms = 0.0
    spec_visits = 0
    inflight = []

    last_st = ref_st

    def account(st):
        nonlocal rays, kbytes, kms, spec_visits, last_st
        last_st = st
        rays += st.rays
        # algorithmic bytes of the tree the kernel traverses: the wide kernel's own visits; the
        # binary kernel's reference-order visits (its speculative extra visits are not work)
        kbytes += st.algo_bytes if args.kernel == "wide" else ref_st.algo_bytes
        spec_visits += st.node_visits
        kms += st.kernel_ms

    for k in range(args.steps):
        if len(inflight) == fif:   # film k % fif is free once frame k - fif is done (and checked)
            account(finish(inflight.pop(0)))
        frame(k % fif, timed=True)
        inflight.append(k % fif)
    for j in inflight:
        account(finish(j))
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    last = (args.steps - 1) % fif if args.steps > 0 else 0
    st = last_st   # (the last timed frame's counters)
    phase("reduce")
    agree("timed frames")

    tdev = dev if backend == "nccl" else "cpu"
    gather_ms = sum(a.elapsed_time(b) for a, b in gather_ev) if gather_ev else gather_host_ms[0]
    t = torch.tensor([elapsed, float(rays)], dtype=torch.float64, device=tdev)
    per_rank = single_frame_ms = None
    if dist_on:
        mx = t[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t[1:].clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, total_rays = float(mx.item()), float(sm.item())
        # per rank: render-kernel ms and gather ms per timed frame (HIP events on the frame's
        # stream; gloo: host time), rays per frame, wall ms per frame
        mine = torch.tensor([kms / max(args.steps, 1), gather_ms / max(args.steps, 1), rays / max(args.steps, 1),
                             t[0].item() / max(args.steps, 1) * 1e3],
                            dtype=torch.float64, device=tdev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [{"rank": r, "kernel_ms": float(v[0]), "gather_ms": float(v[1]), "rays_per_frame": float(v[2]),
                     "wall_ms_per_frame": float(v[3])} for r, v in enumerate(torch.stack(allr).cpu().tolist())]
    else:
        total_rays = float(rays)
    if fif > 1 and args.steps > 0:
        # one frame alone (no frame in flight beside it): its latency, max over ranks, beside the
        # pipelined ms_per_step
        phase("single frame")
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        frame(0)
        finish(0, "single frame")
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier()
        sf = torch.tensor([(time.perf_counter() - t1) * 1e3], dtype=torch.float64, device=tdev)
        if dist_on:
            dist.all_reduce(sf, op=dist.ReduceOp.MAX)
        single_frame_ms = float(sf.item())
        agree("single frame")
    pipelined = None
    if args.steps > 0 and fif == 1 and not args.no_pipelined:
        # The same timed sequence with two frames in flight (films 0 / 1 on two streams, each frame
        # still rendered in full, gathered and checked): the launches' tails overlap the next frame's
        # first waves.  Reported beside the one-frame-at-a-time headline, never instead of it.
        phase("pipelined frames")
        check(frame(1, wait=True), 1, "pipelined frames")   # film 1's first launch: its tile order
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize(dev)
        tp = time.perf_counter()
        prays, infl = 0, []
        for k in range(args.steps):
            if len(infl) == 2:
                prays += finish(infl.pop(0), "pipelined frames").rays
            frame(k % 2)
            infl.append(k % 2)
        for j in infl:
            prays += finish(j, "pipelined frames").rays
        torch.cuda.synchronize(dev)
        if dist_on:
            dist.barrier()
        pt_ = torch.tensor([time.perf_counter() - tp, float(prays)], dtype=torch.float64, device=tdev)
        if dist_on:
            pmx, psm = pt_[:1].clone(), pt_[1:].clone()
            dist.all_reduce(pmx, op=dist.ReduceOp.MAX)
            dist.all_reduce(psm, op=dist.ReduceOp.SUM)
            pel, ptot = float(pmx.item()), float(psm.item())
        else:
            pel, ptot = float(pt_[0].item()), float(pt_[1].item())
        agree("pipelined frames")
        pipelined = {"frames_in_flight": 2, "steps": args.steps, "ms_per_step": pel / args.steps * 1e3,
                     "value": ptot / pel / 1e6, "unit": "Mray/s",
                     "note": "the timed sequence again with two frames in flight (two films on two streams: a "
                             "frame's first waves overlap the previous frame's tail), max over ranks; the headline "
                             "renders one frame at a time at every N"}
    phase("report")

    compat = None
    if sample and world == 1 and not args.no_compat:
        # the reference's RNG semantics on the same frame, for comparison (2 frames: the first
        # measures tile costs for the longest-first launch order, the second is timed)
        for it in range(2):
            film.reset(stream.cuda_stream)
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            _, cst = ptamd.render(scene, film, preset.camera, spp, depth, out=local_buf.data_ptr(),
                                  stream=stream.cuda_stream, rng=ptamd.RNG_COMPAT, out_format=out_format,
                                  kernel=kernel_id)
            torch.cuda.synchronize(dev)
            el1 = time.perf_counter() - t1
        compat = {"value": cst.rays / el1 / 1e6, "unit": "Mray/s", "ms_per_step": el1 * 1e3,
                  "kernel_ms": cst.kernel_ms, "rays_per_frame": cst.rays,
                  "note": "compat RNG mode (per-pixel curand_init(seed, pixel, 0) streams, bit-exact with "
                          "oracle/), one frame after one warmup"}

    if rank == 0:
        if dist_on:   # un-permute the stripes of the last frame (rank 0 holds the full image)
            img = ptdist.assemble(gathered[last], h, w, STRIPE, world, chans)
            torch.cuda.synchronize(dev)
        else:
            img = local_bufs[last][: h * w * chans]
        if args.png:
            a = img.reshape(-1).cpu().numpy()
            if rgba8:
                ptamd.write_png_rgba8(args.png, a, w, h)
            else:
                ptamd.write_png(args.png, a, w, h)
        if fif > 1 and args.steps > 0:   # overlapped launches: the launch time of one that ran alone
            kms = warm_kms * args.steps
        achieved = (kbytes / 1e9) / (kms / 1e3) if kms > 0 else 0.0
        rng_desc = (("sample mode: XORWOW per pixel-sample seeded by Philox4x32-10, summation "
                     f"block {args.chunk or max(16, -(-spp // 64))}") if sample else
                    "cuRAND-XORWOW semantics, curand_init(seed, pixel, 0)")
        bid = build_id()
        te = pmc_entry("traffic", workload, spp, rng_desc, args.kernel, bid)
        ve = pmc_entry("valu", workload, spp, rng_desc, args.kernel, bid)
        traffic, traffic_src = (te["traffic_bytes_per_launch"], te["source"]) if te else (None, None)
        valu, valu_src = (ve["valu_wave_instructions_per_launch"], ve["source"]) if ve else (None, None)
        kernel_s = kms / 1e3 / args.steps if kms > 0 else 0.0
        hbm_gbs = traffic / kernel_s / 1e9 if (traffic and kernel_s > 0) else None
        out = {
            "metric": METRIC,
            "value": total_rays / elapsed / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: scene assembled from the reference's bundled OBJ models (models/), fixed seed",
            "config": {"workload": workload, "width": w, "height": h, "spp": spp, "max_depth": depth,
                       "stripe_rows": STRIPE, "parallelism": f"rows{world}", "frames_in_flight": fif,
                       "wide_tree": settings["wide_tree"] if not instanced else "host two-level",
                       "output": ("rgba8: quantised on the device like PngImage::saveColor, gathered at 4 B/pixel"
                                  if rgba8 else "f32 RGB, gathered at 12 B/pixel"),
                       "rays_per_frame": total_rays / args.steps,
                       "rng": ("sample mode: XORWOW per pixel-sample seeded by Philox4x32-10, summation "
                               f"block {args.chunk or max(16, -(-spp // 64))}") if sample else
                              "cuRAND-XORWOW semantics, curand_init(seed, pixel, 0)"},
            # The traversal's working set (tree + primitive + shading records: 0.5 MB for C3) is
            # L2-resident: its bytes come from L2 and L1, HBM traffic is the per-task block sums
            # (`hbm`, PMC).  The applicable memory ceiling is L2 bandwidth; the measured ceiling of
            # this access pattern (dependent per-lane gathers) is `gather_ceiling`.
            # (the memory level whose ceiling `achieved` is held against; the resource that binds
            # the kernel is VALU issue with partly idle lanes -- `limiter`, `valu_issue`)
            "roofline": {"bound": "l2", "limiter": "valu_issue", "achieved": achieved, "peak": L2_PEAK_GBS,
                         "unit": "GB/s",
                         "frac": achieved / L2_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "hbm": {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS,
                                 "frac": hbm_gbs / HBM_PEAK_GBS if hbm_gbs is not None else None,
                                 "note": "traffic past L2 (PMC; Infinity-Cache hits included): an upper "
                                         "bound of the HBM traffic (profiles/r04_fetch_calib)"},
                         "gather_ceiling": {"peak": GATHER_CEILING_GBS, "frac": achieved / GATHER_CEILING_GBS,
                                            "source": "tools/micro/chase.hip, DESIGN.md section 6"},
                         "kernel": "renderKernelWF<STACK, SAMPLE, WIDE=%s>" % ("true" if args.kernel == "wide" else "false"),
                         "kernel_ms_per_launch": kms / args.steps,
                         "algo_bytes_per_launch": kbytes / args.steps,
                         "algo_bytes_source": ("the wide kernel's own counts: 80 B per 8-wide node visit + 40 B per "
                                               "triangle test + 20 B per sphere test" if args.kernel == "wide" else
                                               "reference-order traversal counts of the same frame (ray-synchronous "
                                               "kernel, warmup step 1): 56 B per binary node visit + 40 B per "
                                               "triangle test + 20 B per sphere test"),
                         "node_visits_reference": ref_st.node_visits,
                         "node_visits_kernel": spec_visits / args.steps,
                         # the kernel's binding resource: VALU instruction
                         # issue, its wave-instructions per launch (PMC) / kernel time vs the ceiling
                         "valu_issue": {"achieved": (valu / kernel_s / 1e9) if (valu and kernel_s > 0) else None,
                                        "peak": VALU_PEAK_GINST, "unit": "G wave-instructions/s",
                                        "frac": (valu / kernel_s / 1e9 / VALU_PEAK_GINST)
                                        if (valu and kernel_s > 0) else None,
                                        "wave_instructions_per_launch": valu, "source": valu_src}},
        }
        out["build_id"] = bid
        if per_rank is not None:
            out["per_rank"] = per_rank
        if single_frame_ms is not None:
            out["single_frame_ms"] = single_frame_ms
            out["single_frame_note"] = ("one frame rendered alone after the timed frames (no frame in flight beside "
                                        "it), max over ranks; ms_per_step is the pipelined rate with "
                                        f"frames_in_flight {fif}")
        if pipelined is not None:
            out["pipelined"] = pipelined
        if compat:
            out["compat_mode"] = compat
        if world == 1 and not args.no_interactive:
            out["interactive"] = interactive(scene, preset, dev, stream, local)
        if world == 1 and not instanced:   # a dynamic scene's per-frame rebuild: LBVH + wide tree on the device
            dyn = ptamd.Scene(preset.objects, preset.materials, device=local,
                              flags=ptamd.PT_BVH_ORIGIN_BOUNDS | ptamd.PT_BVH_WIDE_DEVICE)
            dyn.build_bvh(ptamd.PT_BVH_ORIGIN_BOUNDS | ptamd.PT_BVH_WIDE_DEVICE)   # a rebuild: buffers reused
            scene_build["lbvh_plus_wide_tree_device_ms"] = dyn.build_ms
            del dyn
        out["scene_build"] = scene_build
        if world == 1 and not args.no_cpu_baseline:
            gpu_ref = None if instanced else {
                "gpu_reference_order_node_visits": ref_st.node_visits / max(ref_st.rays, 1),
                "gpu_reference_order_prim_tests": (ref_st.tri_tests + ref_st.sphere_tests) / max(ref_st.rays, 1),
                "gpu_wide_node_visits": st.node_visits / max(st.rays, 1),
                "gpu_wide_prim_tests": (st.tri_tests + st.sphere_tests) / max(st.rays, 1),
                "note": "node visits: binary LBVH nodes (CPU, reference-order GPU kernel) vs compressed 8-wide "
                        "nodes (wide kernel); CPU at 1 spp (bounded sample), GPU over the whole frame"}
            # short legs on the other single-GPU BASELINE configurations (C2, C5; C3 when the bench
            # ran another one), BASELINE.md section 4 (PT_CPU_LEGS=0: none)
            legs = {}
            if os.environ.get("PT_CPU_LEGS", "1") != "0":
                for cfg in ("c2", "c3", "c5"):
                    if CONFIGS[cfg][0] != name:
                        lp = ptamd.Preset(CONFIGS[cfg][0])
                        legs[cfg] = (lp, CONFIG_SPP.get(cfg, lp.spp), 3.0)
            out["cpu_baseline"] = cpu_baseline(ptamd.Preset(name) if instanced else preset, gpu_ref=gpu_ref,
                                               spp=spp, legs=legs)
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
