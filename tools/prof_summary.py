#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_summary.md and profiles/pmc_summary.json.

Launch order of bench.py: a counted pass (mesh_kernel<true>), then the warmup steps and the timed
steps (mesh_kernel<false>; with chained batches a launch may trace several steps, another only
combine, and a step may have no launch of its own).  rocprofv3 -T truncates the template instances
to "mesh_kernel", so the timed launches are the last launches_per_step x steps mesh_kernel
dispatches (the bench line's count); every figure is per STEP (their sum / steps), not per launch.

HBM bytes follow MI355X_MICROARCH.md §HBM with this kernel's own access widths calibrated on a known
byte count (tools/micro/pmc_bytes.hip, profiles/round5/pmc_bytes_factors.json): FETCH_SIZE and
WRITE_SIZE are KiB, multiplied by the factor of the access width that carries the workload's DRAM
traffic (traffic_model in the summary says which).
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def load_json_line(path):
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{"):
                return json.loads(line)
    raise ValueError(f"no JSON line in {path}")


def dispatches(path, name="mesh_kernel"):
    rows = [r for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(name)]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id")))
    return rows


def counters(path, last, steps):
    """Per-step sums of each counter over the last `last` mesh_kernel dispatches (the timed launches of
    `steps` steps)."""
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("mesh_kernel"):
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)[-last:]
    out = defaultdict(float)
    for i in ids:
        for k, v in per[i].items():
            out[k] += v
    return {k: v / steps for k, v in out.items()}, len(ids)


FACTORS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "round5",
                       "pmc_bytes_factors.json")


def traffic_model(scene: str):
    """(fetch factor, write factor, description) for the workload's DRAM traffic: the LDS-resident
    scene's DRAM bytes are the 12-B/lane radiance stores and the combine's 12-B/lane loads; a tree in
    global memory adds scattered 16-B node and triangle rows (128-B lines), which dominate its
    reads.  Uncalibrated (no factors file): the guide's 16-B/lane factors (2 x FETCH, 1 x WRITE)."""
    try:
        with open(FACTORS) as f:
            cal = json.load(f)
    except OSError:
        return 2.0, 1.0, "uncalibrated: MI355X_MICROARCH.md 16-B/lane factors (2 x FETCH_SIZE, 1 x WRITE_SIZE)"
    wr = cal["st_f3"]["write_factor"]
    if scene == "cornell34":
        rd = cal["ld_f3_fr"]["fetch_factor"]
        return rd, wr, (f"FETCH_SIZE x {rd} (12-B/lane combine loads, ld_f3_fr) + WRITE_SIZE x {wr} "
                        f"(12-B/lane radiance stores, st_f3); {os.path.relpath(FACTORS, os.path.dirname(FACTORS) + '/../..')}")
    rd = cal["ld_row"]["fetch_factor"]
    return rd, wr, (f"FETCH_SIZE x {rd} (scattered 16-B node/triangle rows, ld_row) + WRITE_SIZE x {wr} "
                    f"(12-B/lane radiance stores, st_f3); {os.path.relpath(FACTORS, os.path.dirname(FACTORS) + '/../..')}")


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("tag", help="profile.sh tag (reads gpurun_out/prof_TAG unless --root)")
    ap.add_argument("--root", default=None)
    ap.add_argument("--out", default="profiles", help="directory (repo-relative) for the summary files")
    ap.add_argument("--name", default=None, help="file stem of the summaries (default: the tag)")
    a = ap.parse_args()
    tag = a.tag
    root = a.root or os.path.join("gpurun_out", f"prof_{tag}")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bench = load_json_line(os.path.join(root, "kt_bench.json"))
    steps = bench["steps"]
    # the timed launches: one per step, or fewer with chained batches (a step posted before the run's
    # last launch started has none; bench.py's launches_per_step counts them)
    launches = int(round(bench["roofline"].get("launches_per_step", 1.0) * steps))
    kt = dispatches(os.path.join(root, "kt", "run_kernel_trace.csv"))
    timed = kt[-launches:]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
    mean_ms = sum(durs) / steps  # kernel time per step
    c = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_ta"):
        p = os.path.join(root, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            vals, n = counters(p, launches, steps)
            c.update(vals)
    cfg = bench["config"]
    f_fetch, f_write, model = traffic_model(cfg["scene"])
    try:
        with open(FACTORS) as f:
            cal = {k: {m: v[m] for m in ("fetch_factor", "write_factor") if m in v} for k, v in json.load(f).items()}
    except OSError:
        cal = None
    fetch_raw = c.get("FETCH_SIZE", 0.0) * 1024
    write_raw = c.get("WRITE_SIZE", 0.0) * 1024
    hbm = f_fetch * fetch_raw + f_write * write_raw
    write = f_write * write_raw
    lib_sha = None
    if os.path.exists(os.path.join(root, "lib.sha256")):
        lib_sha = open(os.path.join(root, "lib.sha256")).read().split()[0]
    workload = f"{cfg['scene']} {cfg['width']}x{cfg['height']} {cfg['spp']}spp depth{cfg['max_depth']}"
    lane_util = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]) if c.get("SQ_ACTIVE_INST_VALU") else None
    clock = c["GRBM_GUI_ACTIVE"] / 8 / (mean_ms * 1e-3) / 1e9 if c.get("GRBM_GUI_ACTIVE") else None
    cus = 256
    valu_busy = (c["SQ_INSTS_VALU"] * 2 / (4 * cus)) / (mean_ms * 1e-3 * clock * 1e9) if clock else None
    summary = {
        "tag": tag, "workload": workload, "kernel": "mesh_kernel",
        "timed_steps": steps, "timed_launches": len(timed),
        "launch_ms_rocprof": [round(d, 4) for d in durs],
        "kernel_ms_per_step_rocprof": round(mean_ms, 4),
        "kernel_ms_per_step_bench_events": bench["roofline"].get("kernel_ms_per_step"),
        "hbm_bytes_per_step": int(hbm), "fetch_bytes_raw_per_step": int(fetch_raw),
        "write_bytes_raw_per_step": int(write_raw), "write_bytes_per_step": int(write),
        "traffic_model": model,
        # per access width: bytes moved / counter bytes, measured on known byte counts (pmc_bytes.hip)
        "pmc_factors": cal,
        "alg_bytes_per_step": bench["roofline"]["algorithmic_bytes"].get("per_step"),
        "flop_per_step": bench["roofline"].get("flop_per_step"),
        "lib_sha256": lib_sha,
        "hbm_gbs": round(hbm / (mean_ms * 1e-3) / 1e9, 2),
        "waves_per_launch": c.get("SQ_WAVES"), "valu_insts_per_launch": c.get("SQ_INSTS_VALU"),
        "salu_insts_per_launch": c.get("SQ_INSTS_SALU"), "vmem_rd_insts_per_launch": c.get("SQ_INSTS_VMEM_RD"),
        "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
        "valu_lane_utilization": round(lane_util, 4) if lane_util else None,
        "clock_ghz": round(clock, 3) if clock else None,
        "valu_issue_busy": round(valu_busy, 4) if valu_busy else None,
        "wait_inst_any_frac": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4) if c.get("SQ_WAVE_CYCLES") else None,
        "active_inst_any_frac": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        if c.get("SQ_WAVE_CYCLES") and c.get("SQ_ACTIVE_INST_ANY") else None,
        # texture-addresser (vector-memory address unit) busy fraction per CU: the limiter of
        # global-memory BVH traversal (every lane's node/triangle load passes through it)
        "ta_busy": round(c["TA_BUSY_avr"] / (c["GRBM_GUI_ACTIVE"] / 8), 4)
        if c.get("TA_BUSY_avr") and c.get("GRBM_GUI_ACTIVE") else None,
        "ta_cycles_per_vmem_wave": round(c["TA_BUSY_avr"] * cus / c["TA_FLAT_READ_WAVEFRONTS_sum"], 2)
        if c.get("TA_BUSY_avr") and c.get("TA_FLAT_READ_WAVEFRONTS_sum") else None,
        "bench_value_msamples_s": bench["value"],
        "bench_ms_per_step": bench["ms_per_step"],
        # the profiled run's image: bench.py uses these counters only for a run of the same image
        "image_crc32": cfg.get("image_crc32"),
        # the kernel-trace run's own step time: the rocprof kernel time per step may not exceed it
        "rocprof_kernel_le_ms_per_step": bool(mean_ms <= bench["ms_per_step"] * 1.0005),
    }
    prof_dir = os.path.join(repo, a.out)
    name = a.name or tag
    os.makedirs(prof_dir, exist_ok=True)
    # bench.py reads profiles/pmc_summary.json for roofline.traffic of its default workload
    # (Cornell); every workload also keeps its counters beside its summary (<name>_pmc.json, which
    # bench.py finds by workload)
    default = workload.startswith("cornell34 1920x1080 64spp depth8") and "wavefront" not in workload
    if default:
        with open(os.path.join(repo, "profiles", "pmc_summary.json"), "w") as f:
            json.dump(summary, f, indent=1)
    with open(os.path.join(prof_dir, f"{name}_pmc.json"), "w") as f:
        json.dump(summary, f, indent=1)
    stats_csv = open(os.path.join(root, "kt", "run_kernel_stats.csv")).read()
    with open(os.path.join(prof_dir, f"{name}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary `{tag}` — {workload}\n\n")
        f.write("Command: `bash tools/profile.sh` (bench.py --steps 20 --warmup 5 under rocprofv3 "
                "--kernel-trace --stats, then separate --pmc passes; figures per step).\n\n")
        f.write("## rocprofv3 --kernel-trace --stats (all dispatches, incl. the counted pass)\n\n```\n")
        f.write(stats_csv)
        f.write("```\n\n## mesh_kernel, the timed steps' launches, per step\n\n```\n")
        f.write(json.dumps(summary, indent=1))
        f.write("\n```\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
