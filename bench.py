#!/usr/bin/env python3
"""bench.py — Msamples/s (rays x bounces per second) of the HIP path-tracing megakernel.

Workload (BASELINE.json configs[1], the default): Cornell-34 scene, 1920x1080, 64 spp, 8 bounces.
One step = the whole workload once: 64 frames of every pixel (running-average accumulation,
frames 0..63) through libhippt's C ABI.  --preset configN selects another BASELINE workload
(config2 = the default, config3 blob70k 1080p, config4 blob70k 3840x2160 256 spp — the 8-GPU
row-tiled job —, config5 the blob70k wavefront A/B).

With N GPUs (torchrun, one process per GPU) rank r renders rows r, r+N, r+2N, ... (interleaved:
contiguous bands differ in cost by up to 1.6x) and the image is bit-identical for any N.
--scaling strong (default): the SAME job at every N (each rank a 1/N share of the image's rows;
the north star's "tile scaling" of a fixed image); --scaling weak: the step renders spp*N frames
(every rank traces as many samples as one GPU does alone).  No collective touches the data path —
ranks only meet at the barriers, the max-over-ranks of the timed interval and the untimed
bookkeeping after it (gloo, CPU).  For N > 1 the line carries `ranks`: each rank's kernel time
and wall time per step and the max/mean kernel-time imbalance.

value = segments traced by all ranks in the K timed steps / max-over-ranks wall time, in
millions per second; the segment count is the exact count the kernel accumulates (one per
closest-hit query), so nothing is estimated.

Also reported on rank 0:
  roofline      FP32 VALU roofline of the mesh kernel (bound "valu": the path is branchy scalar
                FP32 over a cache-resident scene, neither HBM- nor MFMA-bound): algorithmic
                FLOP per launch from a counted (untimed) pass of the same step (20 per child-box
                slab test, 55 per primitive test, 100 per shading step) / the kernel's mean
                launch time (HIP events on the library's stream, timed region), vs 157.3
                TFLOP/s.  From this workload's PMC summary under profiles/ (when present):
                traffic = HBM bytes per launch, hbm = traffic / launch time vs 8 TB/s,
                valu_issue / ta_busy, and `limiter` = the busiest of VALU issue, TA and HBM.
                algorithmic_bytes = the SURVEY.md 8(d) node/primitive/shading bytes (served by
                LDS/L2/MALL, not HBM).
  cpu_baseline  the reference CPU path tracer (RayTracer.h + Qt-free RenderWorker, built as
                oracle/_ref/ref_harness) timed on this box's host cores over a bounded sample
                of whole rows of the same workload: the median of 5 runs at the box's CPU share,
                a 1-thread rate and the projection to the affinity mask, with the host's CPU
                facts (nproc, the affinity mask's size, lscpu's model name, OMP_NUM_THREADS).  If the
                harness is missing the object says so (value null, an error string) instead of
                timing a different program; --cpu-baseline port times the FP32 oracle port.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))

METRIC = "Msamples/s (rays×bounces/s) at 1920×1080, 8 bounces; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0
BYTES_NODE, BYTES_TRI, BYTES_SHADE, BYTES_SAMPLE = 64, 48, 32, 12
BYTES_NODE4 = 112  # 4-wide node: 4 child boxes + 4 child codes
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector (= FP32 MFMA) peak
FLOP_NODE, FLOP_TRI, FLOP_SHADE = 40, 55, 100  # SURVEY.md §8(d) secondary figure

# BASELINE.json configs[k] as bench workloads (configs[0] is the CPU-only plumbing case)
PRESETS = {
    "config2": dict(scene="cornell34", width=1920, height=1080, spp=64, depth=8, path_mode="megakernel"),
    "config3": dict(scene="blob70k", width=1920, height=1080, spp=64, depth=8, path_mode="megakernel"),
    "config4": dict(scene="blob70k", width=3840, height=2160, spp=256, depth=8, path_mode="megakernel"),
    "config5": dict(scene="blob70k", width=1920, height=1080, spp=64, depth=8, path_mode="wavefront"),
}


def baseline_config_index(args) -> int | None:
    """k of the BASELINE.json configs[k] this run's workload is (None: none of them)."""
    w = dict(scene=args.scene, width=args.width, height=args.height, spp=args.spp, depth=args.depth,
             path_mode=args.path_mode)
    for name, p in PRESETS.items():
        if p == w:
            return int(name[-1]) - 1
    return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=1)
    # the driver's round-end run is 20 timed steps; with chained batches (up to 8 whole images per
    # launch) fewer steps weigh the run's first and last launch more (10 steps: 55.4 G, r6ba)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--prewarm-ms", type=float, default=200.0,
                   help="untimed GPU clock warm-up before the warmup steps: whole steps for this many ms")
    p.add_argument("--scene", default="cornell34",
                   choices=["cornell34", "blob70k", "random_scene", "cornell_mixed"])
    p.add_argument("--path-mode", default="megakernel", choices=["megakernel", "wavefront"],
                   help="BASELINE configs[4] A/B: persistent megakernel or wavefront kernels")
    p.add_argument("--wavefront-slots", type=int, default=None)
    p.add_argument("--preset", default=None, choices=sorted(PRESETS),
                   help="a BASELINE.json workload (overrides --scene/--width/--height/--spp/--depth/--path-mode)")
    p.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                   help="N GPUs render spp frames of the image (strong: a fixed job, the default) or "
                        "N*spp frames (weak: fixed work per GPU)")
    p.add_argument("--split", default="interleave", choices=["interleave", "bands"],
                   help="rows per rank for N>1: interleaved (rank r: rows r, r+N, ...) or contiguous bands")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=64)
    p.add_argument("--depth", type=int, default=8)
    p.add_argument("--wave-threshold", type=int, default=None)
    p.add_argument("--chunk", type=int, default=None)
    p.add_argument("--scratch-mb", type=int, default=None)
    p.add_argument("--bvh-width", type=int, default=None, choices=[0, 2, 4],
                   help="megakernel BVH width (HIPPT_OPT_BVH_WIDTH; default automatic)")
    p.add_argument("--cpu-baseline", default="auto", choices=["auto", "reference", "port", "off"])
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="target duration of one CPU sample run")
    p.add_argument("--cpu-runs", type=int, default=5, help="CPU sample runs (the median is reported)")
    p.add_argument("--cpu-threads", type=int, default=None)
    p.add_argument("--option", action="append", default=[], metavar="NAME=V",
                   help="any library option by its hippt.h name without HIPPT_OPT_ (e.g. BVH_QUANT=3); "
                        "recorded in config.options")
    p.add_argument("--pmc", default=None, help="PMC summary JSON for roofline.traffic")
    a = p.parse_args()
    if a.preset:
        for k, v in PRESETS[a.preset].items():
            setattr(a, k, v)
    return a


def host_cpu_facts() -> dict:
    """What the CPU baseline ran on: nproc (os.cpu_count, the whole machine), the affinity mask's
    size, OMP_NUM_THREADS (the GPU box sets it to the box's CPU share, 16 per GPU) and lscpu's
    model name (read from /proc/cpuinfo, as lscpu does)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    # the cgroup's CPU bandwidth limit (cgroup v2 cpu.max: "quota period" or "max period"), in cores
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": affinity, "omp_num_threads": omp or None, "model": model,
            "cgroup_cpu_quota_cores": quota}


def cpu_threads(args, facts) -> tuple[int, str]:
    """Threads for the CPU baseline and the rule that chose them: --cpu-threads, else the
    affinity mask's size, capped by OMP_NUM_THREADS when set (on the GPU box the mask and nproc
    cover the whole machine while the box's CPU share is OMP_NUM_THREADS = 16 per GPU)."""
    if args.cpu_threads:
        return args.cpu_threads, "--cpu-threads"
    if facts["omp_num_threads"] and facts["omp_num_threads"] < facts["affinity"]:
        return facts["omp_num_threads"], "OMP_NUM_THREADS (the host's CPU share; below the affinity mask)"
    return facts["affinity"], "affinity mask"


def cpu_baseline(args, scene) -> dict | None:
    """Reference CPU tracer on a bounded sample of rows of the same workload: the median of
    --cpu-runs runs."""
    if args.cpu_baseline == "off":
        return None
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle  # checker / baseline only
    from hippt import scenes as sc_mod
    facts = host_cpu_facts()
    threads, rule = cpu_threads(args, facts)
    kind = args.cpu_baseline
    if kind == "auto":
        if not os.path.exists(pyoracle.REF_HARNESS):
            # never a silent substitute: the reference build is missing, say so
            log("cpu_baseline: oracle/_ref/ref_harness is missing (make -C oracle ref, needs /root/reference)")
            return {"value": None, "unit": "Msamples/s", "cores": threads, "kind": "reference",
                    "error": "oracle/_ref/ref_harness missing: the reference CPU tracer was not built "
                             "(make -C oracle ref in the development container); not timed", "host": facts}
        kind = "reference"
    runs = max(1, args.cpu_runs)
    if kind == "reference":
        with tempfile.TemporaryDirectory() as tmp:
            path = os.path.join(tmp, "scene.bin")
            sc_mod.write_scene_file(scene, path)

            def sample(n_threads, seconds, n_runs):
                # probe on every 64th line, then pick the line stride that takes ~seconds
                probe = run_t(64, n_threads)
                per_line = probe["seconds"] / max(1, probe["rows"])
                lines = max(1, min(args.height, int(seconds / max(per_line, 1e-6))))
                stride = max(1, -(-args.height // lines))
                return stride, sorted((run_t(stride, n_threads) for _ in range(n_runs)),
                                      key=lambda r: r["msamples_per_s"])

            def run_t(stride, n_threads):
                out = subprocess.run([pyoracle.REF_HARNESS, "bench", path, str(args.width), str(args.height),
                                      str(stride), str(args.spp), str(args.depth), str(n_threads)],
                                     capture_output=True, text=True, check=True, timeout=900).stdout
                return json.loads(out.strip().splitlines()[-1])

            stride, rs = sample(threads, args.cpu_seconds, runs)
            # per-thread rate (1 thread, fewer lines) and the parallel efficiency of the share, for the
            # projection to the whole affinity mask (the reference uses hardware_concurrency() threads,
            # RayTracerFboItem.cpp:75; the GPU box's CPU share is OMP_NUM_THREADS = 16 per GPU and a run
            # must not use more, so the mask-wide figure is projected, not timed)
            one = procs = None
            if threads > 1 and facts["affinity"] > threads and args.cpu_runs > 1:
                _, r1 = sample(1, args.cpu_seconds / 2, 3)
                one = r1[len(r1) // 2]
                # the timed sample's lines split over `threads` separate 1-thread processes at once: the
                # reference's threads share its materials' shared_ptr control blocks (HitRecord::mat_ptr,
                # RayTracer.h:211, copied on every closer hit, :311 and :348), processes do not
                def run_procs():
                    ps_ = [subprocess.Popen([pyoracle.REF_HARNESS, "bench", path, str(args.width), str(args.height),
                                             str(stride), str(args.spp), str(args.depth), "1", str(k), str(threads)],
                                            stdout=subprocess.PIPE, text=True) for k in range(threads)]
                    outs = [json.loads(p_.communicate(timeout=900)[0].strip().splitlines()[-1]) for p_ in ps_]
                    return sum(o["segments"] for o in outs) / max(o["seconds"] for o in outs) / 1e6

                pr = sorted(run_procs() for _ in range(3))
                procs = {"value": round(pr[1], 4), "processes": threads, "threads_each": 1,
                         "runs": [round(v, 4) for v in pr],
                         "rule": "the timed sample's lines dealt round-robin to the processes, all started at "
                                 "once; total segments / the slowest process's render time; median of 3"}
        r = rs[len(rs) // 2]
        out = {"value": round(r["msamples_per_s"], 4), "unit": "Msamples/s", "cores": threads,
               "kind": "reference",
               "sample": f"every {stride}th line ({r['rows']} whole lines) of {args.width}x{args.height}, {args.spp} spp, "
                         f"depth {args.depth}, "
                         f"{scene.name}; RayTracer.h ray_color + RenderWorker tile pool (tile {r['tile']}), "
                         f"{r['segments']} segments in {r['seconds']:.2f} s; median of {runs} runs",
               "runs": [round(x["msamples_per_s"], 4) for x in rs],
               "threads_rule": rule, "host": facts,
               "mpixel_samples_per_s": round(r["mpixel_samples_per_s"], 4)}
        if one:
            eff = r["msamples_per_s"] / (threads * one["msamples_per_s"])
            out["per_thread"] = {"value": round(one["msamples_per_s"], 4), "threads": 1,
                                 "parallel_efficiency_at_cores": round(eff, 3)}
            # the whole mask's rate is at most the 1-thread rate times its threads (the tile pool,
            # RayTracerFboItem.cpp:75-90, has no serial part; its threads contend on the materials'
            # reference counts instead, which `independent_processes` shows)
            out["full_affinity_upper_bound"] = {
                "value": round(one["msamples_per_s"] * facts["affinity"], 2), "threads": facts["affinity"],
                "rule": "1-thread rate x affinity-mask threads (linear scaling, an upper bound: not timed at the "
                        "mask's size, which the box's CPU share does not allow)"}
        if procs:
            out["independent_processes"] = procs
        return out
    ms = pyoracle.MeshScene(scene, args.width, args.height, accel=1)
    t0 = time.perf_counter()
    _, _, segs, ps = ms.frames(0, args.spp, args.depth, y0=0, y1=2, nthreads=threads)
    rate = segs / max(time.perf_counter() - t0, 1e-6)
    rows = max(1, min(args.height, int(args.cpu_seconds * rate / max(segs / 2, 1))))
    vals = []
    for _ in range(runs):
        t0 = time.perf_counter()
        _, _, segs, ps = ms.frames(0, args.spp, args.depth, y0=0, y1=rows, nthreads=threads)
        vals.append(segs / (time.perf_counter() - t0) / 1e6)
    vals.sort()
    return {"value": round(vals[len(vals) // 2], 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"rows 0..{rows - 1}, {args.spp} spp, depth {args.depth}, {scene.name}; FP32 oracle port; "
                      f"median of {runs} runs",
            "runs": [round(v, 4) for v in vals], "threads_rule": rule, "host": facts}


def load_pmc(args, workload: str) -> list:
    """The PMC summaries of this exact workload (tools/profile.sh + tools/prof_summary.py), most
    recent first: --pmc, else profiles/pmc_summary.json (the default workload), then this round's
    and older rounds' profiles/**/<name>_pmc.json, the archive last.  check_pmc picks the first that
    describes this run."""
    prof = os.path.join(REPO, "profiles")
    paths = [args.pmc] if args.pmc else (
        [os.path.join(prof, "pmc_summary.json")]
        + sorted(glob.glob(os.path.join(prof, "round*", "*_pmc.json")), reverse=True)
        + sorted(glob.glob(os.path.join(prof, "*_pmc.json")), reverse=True)
        + sorted(glob.glob(os.path.join(prof, "archive", "*_pmc.json")), reverse=True))
    found = []
    for path in paths:
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            d["source"] = os.path.relpath(path, REPO)
            found.append(d)
    return found


def lib_sha256(path: str) -> str | None:
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return None


def check_pmc(pmc, image_crc, lib_sha, world: int):
    """A PMC summary of this workload only where it describes this run: the
    same image (the summary's image_crc32 = this run's) traced by the same kernels (the summary's
    lib_sha256 = the loaded libhippt.so's).  Its bytes are per step, so a profile taken on a slower
    box still states this run's traffic; the line's HBM rate divides them by this run's kernel time.
    `pmc`: one summary or load_pmc's list (the first that passes).  Otherwise (None, reason):
    roofline.traffic is null and says why (the first candidate's reason)."""
    if isinstance(pmc, list):
        first = None
        for d in pmc:
            ok, why = check_pmc(d, image_crc, lib_sha, world)
            if ok:
                return ok, None
            first = first or why
        return None, first
    if not pmc:
        return None, None
    if world > 1:
        return None, "the PMC summaries are single-GPU profiles of the whole image"
    if pmc.get("image_crc32") is None:
        return None, f"{pmc.get('source')}: no image_crc32 recorded (profile predates the check)"
    if image_crc is not None and int(pmc["image_crc32"]) != int(image_crc):
        return None, f"{pmc.get('source')}: image CRC {pmc['image_crc32']} is not this run's {image_crc}"
    if not pmc.get("lib_sha256") or pmc["lib_sha256"] != lib_sha:
        return None, f"{pmc.get('source')}: profiled libhippt.so {str(pmc.get('lib_sha256'))[:12]} is not this run's {str(lib_sha)[:12]}"
    if not pmc.get("hbm_bytes_per_step"):
        return None, f"{pmc.get('source')}: no per-step byte count (profile predates round 5)"
    return pmc, None


def make_roofline(args, pmc, traffic, kernel_ms_step, launches, alg_bytes_step, flops_step, counted,
                  alg_gbs, mean_launch_ms) -> dict:
    """Roofline of the dominant kernel.  This path is branchy scalar FP32 over a cache-resident
    scene: neither HBM nor MFMA bounds it.  The headline roofline is the FP32 VALU one
    (algorithmic FLOP per step from the counted pass / the mesh kernel's live time per step, HIP
    events on the library's stream, vs the FP32 vector peak).  Per step, not per launch: chained
    batches (HIPPT_OPT_CHAIN) spread a run's steps over fewer tracing launches, so a launch's
    duration is not a step's.  `limiter` names the busiest unit in this workload's PMC profile (VALU
    issue, the vector-memory texture addresser TA, or HBM), and the HBM fraction is computed from the
    PMC-measured DRAM bytes per step (calibrated, tools/micro/pmc_bytes.hip), not from the modelled
    node/primitive bytes (those are served by LDS/L2/MALL; reported as algorithmic_bytes)."""
    s = kernel_ms_step * 1e-3
    tflops = flops_step / s / 1e12 if s > 0 else 0.0
    r = {"bound": "valu", "achieved": round(tflops, 3), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
         "frac": round(tflops / FP32_PEAK_TFLOPS, 4), "traffic": traffic,
         "kernel": "mesh_kernel" if args.path_mode == "megakernel" else "wf_extend+wf_shade+wf_generate",
         "kernel_ms_per_step": round(kernel_ms_step, 4), "launches_per_step": launches,
         "mean_launch_ms": round(mean_launch_ms, 4),
         "flop_per_step": int(flops_step),
         "model": "20 FLOP per child-box slab test (2 per 2-wide, 4 per 4-wide node visit), 55 per primitive "
                  "test, 100 per shading step",
         "node_visits_per_step": counted["nodeVisits"], "tri_tests_per_step": counted["triTests"],
         "algorithmic_bytes": {"per_step": int(alg_bytes_step), "achieved_gbs": round(alg_gbs, 2),
                               "note": "node/primitive/shading bytes of the traversal (SURVEY.md 8d), served "
                                       "from LDS/L2/MALL; not HBM traffic"}}
    if pmc:
        hbm = traffic / s / 1e9 if traffic and s > 0 else None
        busy = {"valu_issue": pmc.get("valu_issue_busy") or 0.0, "ta": pmc.get("ta_busy") or 0.0,
                "hbm": (hbm or 0.0) / HBM_PEAK_GBS}
        r["limiter"] = max(busy, key=busy.get)
        r["valu_issue"] = {"busy": pmc.get("valu_issue_busy"), "lane_utilization": pmc.get("valu_lane_utilization"),
                           "note": "fraction of cycles a VALU instruction issues (wave64 = 2 cycles), PMC"}
        r["ta_busy"] = pmc.get("ta_busy")
        r["hbm"] = {"achieved": round(hbm, 2) if hbm is not None else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(hbm / HBM_PEAK_GBS, 4) if hbm is not None else None,
                    "note": "PMC DRAM bytes per step (FETCH_SIZE and WRITE_SIZE with the calibrated factors of "
                            "traffic_model) / this run's kernel time per step"}
        r["traffic_model"] = pmc.get("traffic_model")
        r["pmc_source"] = pmc.get("source")
    else:
        r["limiter"] = None
    return r


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv: list, gpus: int, env) -> list | None:
    """How `bench.py --gpus N` must run (never a silent one-GPU run).
    None: this process is the run (N == 1, or a rank of a launcher whose WORLD_SIZE is N).  A list:
    N > 1 without a launcher, so bench.py starts `torch.distributed.run` with N ranks on 127.0.0.1
    as a child (before anything touches the GPU) and exits with its code.  A WORLD_SIZE that
    disagrees with --gpus raises SystemExit (non-zero)."""
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher's WORLD_SIZE is {world}")
        return None
    if gpus <= 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *argv]


def main():
    args = parse()
    cmd = launcher_command(sys.argv[1:], args.gpus, os.environ)
    if cmd is not None:
        log("bench.py: --gpus", args.gpus, "without a launcher: starting", " ".join(cmd[1:6]), "...")
        raise SystemExit(subprocess.run(cmd).returncode)
    import torch  # noqa: F401  (torch.distributed for the rank barrier / max-over-ranks)
    import torch.distributed as dist
    import hippt
    from hippt import distributed as hd
    from hippt import scenes

    rank, local_rank, world = hd.env_rank()
    if world > 1:
        # gloo prints its peer-connection notice on stdout; keep stdout to the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    lib = hippt.load_library()
    ndev = lib.hipptDeviceCount()
    if ndev < 1:
        raise SystemExit("no HIP device visible")
    device = local_rank % ndev

    def barrier():
        if world > 1:
            dist.barrier()

    def device_sync(pt):
        if not pt.synchronize():
            raise SystemExit(pt.lastError())
        if torch.cuda.is_available():
            torch.cuda.set_device(device)
            torch.cuda.synchronize()

    scene = scenes.get_scene(args.scene)
    pt = hippt.PathTracer()
    pt.setDevices([device])
    if args.split == "interleave":
        my_rows = hd.interleaved_rows(rank, world, args.height)
        pt.setRowInterleave(rank, world)
    else:
        y0, y1 = hd.row_band(rank, world, args.height)
        my_rows = np.arange(y0, y1)
        pt.setRowRange(y0, y1)
    if args.wave_threshold is not None:
        pt.setOption(hippt.OPT_WAVE_THRESHOLD, args.wave_threshold)
    if args.chunk is not None:
        pt.setOption(hippt.OPT_CHUNK, args.chunk)
    if args.scratch_mb is not None:
        pt.setOption(hippt.OPT_SCRATCH_MB, args.scratch_mb)
    if args.bvh_width is not None:
        pt.setOption(hippt.OPT_BVH_WIDTH, args.bvh_width)
    pt.setOption(hippt.OPT_PATH_MODE, 1 if args.path_mode == "wavefront" else 0)
    if args.wavefront_slots is not None:
        pt.setOption(hippt.OPT_WAVEFRONT_SLOTS, args.wavefront_slots)
    # the item order's run-cost estimate on the first call (not on a host thread while the first
    # steps run in image order, HIPPT_OPT_ITEM_ORDER's automatic mode): the timed steps are the
    # steady state of a fixed camera either way
    pt.setOption(hippt.OPT_ITEM_ORDER, 1)
    options = {}
    for kv in args.option:
        name, _, v = kv.partition("=")
        key = getattr(hippt, "OPT_" + name.upper(), None)
        if key is None or not v.lstrip("-").isdigit():
            raise SystemExit(f"--option {kv}: unknown option")
        try:
            pt.setOption(key, int(v))
        except hippt.HipptError as e:
            raise SystemExit(f"--option {kv}: {e}") from None
        options[name.upper()] = int(v)
    pt.uploadMesh(scene)
    if not pt.initialize(args.width, args.height):
        raise SystemExit(pt.lastError())

    frames = args.spp * world if args.scaling == "weak" else args.spp

    def step():
        # frames 0..frames-1: frame 0 overwrites the accumulation (acc*0 + L), so every step is
        # the identical full workload
        if not pt._lib.hipptRenderFramesAsync(0, frames, args.depth, None):
            raise SystemExit(hippt.load_library().hipptLastError().decode())

    # counted pass (untimed): traversal counters for the roofline's algorithmic bytes
    pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 1)
    pt.resetStats()
    step()
    device_sync(pt)
    counted = pt.stats()
    bvh_width = pt._lib.hipptActiveBvhWidth()  # the tree nodeVisits count (2- or 4-wide)
    pt.setOption(hippt.OPT_COUNT_TRAVERSAL, 0)

    # GPU clock warm-up (untimed, before the W warmup steps): the first ~20 ms of GPU work after an
    # idle period run slow (the whole image's first three launches 7.69 / 7.49 / 7.17 ms, then
    # 7.14–7.16; a 1/8 share's first 4-batch groups 4.10 / 4.05 / 3.91 / 3.84 ms, then 3.73–3.76:
    # DESIGN_LOG.md §A.R6, r6q), which W steps of a 1/N share (W ms at N = 8) do not cover.  Every
    # rank, at every N, runs whole steps until --prewarm-ms of wall time have passed.
    t_warm = time.perf_counter()
    prewarm_steps = 0
    while (time.perf_counter() - t_warm) * 1e3 < args.prewarm_ms:
        step()
        prewarm_steps += 1
        if prewarm_steps % 4 == 0:
            device_sync(pt)
    for _ in range(args.warmup):
        step()
    device_sync(pt)
    pt.resetStats()

    barrier()
    device_sync(pt)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    device_sync(pt)
    barrier()
    elapsed = time.perf_counter() - t0

    st = pt.stats()
    # per-rank kernel and wall time per step (untimed bookkeeping: the load balance of the split)
    per_rank = hd.gather_floats((st["traceMs"] / args.steps, elapsed * 1e3 / args.steps), dist)
    elapsed_max = hd.max_over_ranks(elapsed, dist)
    segments = hd.sum_over_ranks(st["segments"], dist)
    samples = hd.sum_over_ranks(st["pixelSamples"], dist)
    value = segments / elapsed_max / 1e6

    # output image of the last step: gathered bands (untimed), checksum on rank 0 (below, with the
    # PMC summary's check)

    # roofline of the dominant (mesh) kernel, from this rank's counted pass and live events
    launches = round(st["traceLaunches"] / max(1, args.steps), 3)
    bytes_node = BYTES_NODE if bvh_width != 4 else BYTES_NODE4
    flop_node = FLOP_NODE if bvh_width != 4 else 2 * FLOP_NODE
    alg_bytes_step = (bytes_node * counted["nodeVisits"] + BYTES_TRI * counted["triTests"]
                      + BYTES_SHADE * (counted["segments"] - counted["pixelSamples"])
                      + BYTES_SAMPLE * counted["pixelSamples"])
    flops_step = (flop_node * counted["nodeVisits"] + FLOP_TRI * counted["triTests"]
                  + FLOP_SHADE * counted["segments"])
    kernel_ms_step = st["traceMs"] / max(1, args.steps)
    mean_launch_ms = st["traceMs"] / max(1, st["traceLaunches"])
    achieved = alg_bytes_step / (kernel_ms_step * 1e-3) / 1e9 if kernel_ms_step > 0 else 0.0
    workload = f"{args.scene} {args.width}x{args.height} {frames}spp depth{args.depth}"
    if args.path_mode == "wavefront":
        workload += " wavefront"
    pmc = load_pmc(args, workload)
    px = pt.readback()[0][my_rows]
    full = (hd.gather_interleaved(px, args.height, dist) if args.split == "interleave"
            else hd.gather_bands(px, args.height, dist))
    import zlib
    image_crc = zlib.crc32(full.tobytes()) & 0xFFFFFFFF if full is not None else None
    pmc, pmc_refused = check_pmc(pmc, image_crc, lib_sha256(os.environ.get("HIPPT_LIB") or hippt.LIB_PATH), world)
    traffic = pmc.get("hbm_bytes_per_step") if pmc else None

    roofline = make_roofline(args, pmc, traffic, kernel_ms_step, launches, alg_bytes_step, flops_step,
                             counted, achieved, mean_launch_ms)
    if pmc_refused:
        roofline["pmc_refused"] = pmc_refused

    k = baseline_config_index(args)
    workload_label = workload
    if k is not None:
        workload_label += (f" (BASELINE configs[{k}])" if world == 1 or args.scaling == "strong"
                           else f" (BASELINE configs[{k}] per GPU)")
    if rank == 0:
        cpu = cpu_baseline(args, scene) if world == 1 else None
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm": {"ms": args.prewarm_ms, "steps": prewarm_steps},
            "ms_per_step": round(elapsed_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": workload_label,
                "scene": args.scene, "triangles": scene.num_tris, "spheres": scene.num_spheres,
                "path_mode": args.path_mode, "width": args.width, "height": args.height,
                "spp": frames, "spp_per_gpu_share": args.spp, "max_depth": args.depth,
                "parallelism": f"{'interleaved-rows' if args.split == 'interleave' else 'row-bands'} x{world}",
                "segments_per_step": segments // max(1, args.steps),
                "pixel_samples_per_step": samples // max(1, args.steps),
                "mpixel_samples_per_s": round(samples / elapsed_max / 1e6, 3),
                "trace_ms_per_step": round(st["traceMs"] / args.steps, 4),
                "combine_ms_per_step": round(st["combineMs"] / args.steps, 4),
                "bvh_nodes": st["bvhNodes"], "bvh_depth": st["bvhDepth"], "bvh_width": bvh_width,
                "wave_threshold": pt._lib.hipptGetOption(hippt.OPT_WAVE_THRESHOLD),
                "chunk": {"option": pt._lib.hipptGetOption(hippt.OPT_CHUNK),
                          "applied": pt._lib.hipptGetOption(hippt.INFO_CHUNK)},
                "image_crc32": image_crc,
                # the library default is -1 (automatic: the estimate on a host thread, batches queued
                # meanwhile in image order); bench.py forces it
                "chain": {"option": pt._lib.hipptGetOption(hippt.OPT_CHAIN),
                          "applied_cap": pt._lib.hipptGetOption(hippt.INFO_CHAIN_CAP),
                          "note": "HIPPT_OPT_CHAIN (default -1, automatic: chained for batches of at most "
                                  "2^26 samples, trees in global memory and the general kernel): a launch "
                                  "whose batch is "
                                  "drained goes on with the steps posted behind it (ring of batches, "
                                  "hippt_trace.h), a later launch combines them, and steps that arrive before "
                                  "the run's last launch has started are launched together as one group; every "
                                  "step's frames are traced and combined inside the timed region"},
                "item_order": {"option": 1, "library_default": -1,
                               "note": "run-cost estimate computed on the first (counted, untimed) call, "
                                       "before the timed region: the timed steps are a fixed camera's "
                                       "steady state"},
                **({"options": options} if options else {}),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if world > 1:
            kms = [r[0] for r in per_rank]
            line["ranks"] = {"trace_ms_per_step": [round(x, 4) for x in kms],
                             "wall_ms_per_step": [round(r[1], 4) for r in per_rank],
                             "imbalance_max_over_mean": round(max(kms) / max(sum(kms) / len(kms), 1e-9), 4),
                             "note": "each rank's kernel time (HIP events) and wall time per step; "
                                     "imbalance = slowest rank's kernel time / the mean"}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
