#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>_summary.md and profiles/pmc_summary.json.

Launch order of bench.py: a counted pass (mesh_kernel<true>, `launches_per_step` launches),
then warmup + timed steps (mesh_kernel<false>).  rocprofv3 -T truncates both template
instances to "mesh_kernel", so the counted launches are identified by dispatch order.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reads half the bytes of a wide coalesced stream, so the corrected read bytes are
2 x FETCH_SIZE x 1024 (the raw figure is kept alongside: this kernel's reads are not wide
streams, the correction is an upper bound).
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


def counters(path, skip):
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("mesh_kernel"):
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)[skip:]
    out = defaultdict(list)
    for i in ids:
        for k, v in per[i].items():
            out[k].append(v)
    return {k: statistics.mean(v) for k, v in out.items()}, len(ids)


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
    lps = bench["roofline"]["launches_per_step"]
    kt = dispatches(os.path.join(root, "kt", "run_kernel_trace.csv"))
    timed = kt[lps:]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
    mean_ms = statistics.mean(durs)
    c = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_ta"):
        p = os.path.join(root, sub, "run_counter_collection.csv")
        if os.path.exists(p):
            vals, n = counters(p, lps)
            c.update(vals)
    fetch_raw = c.get("FETCH_SIZE", 0.0) * 1024
    write = c.get("WRITE_SIZE", 0.0) * 1024
    hbm = 2 * fetch_raw + write
    cfg = bench["config"]
    workload = f"{cfg['scene']} {cfg['width']}x{cfg['height']} {cfg['spp']}spp depth{cfg['max_depth']}"
    lane_util = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]) if c.get("SQ_ACTIVE_INST_VALU") else None
    clock = c["GRBM_GUI_ACTIVE"] / 8 / (mean_ms * 1e-3) / 1e9 if c.get("GRBM_GUI_ACTIVE") else None
    cus = 256
    valu_busy = (c["SQ_INSTS_VALU"] * 2 / (4 * cus)) / (mean_ms * 1e-3 * clock * 1e9) if clock else None
    summary = {
        "tag": tag, "workload": workload, "kernel": "mesh_kernel",
        "timed_launches": len(timed), "mean_launch_ms_rocprof": round(mean_ms, 4),
        "mean_launch_ms_bench_events": bench["roofline"]["mean_launch_ms"],
        "hbm_bytes_per_launch": int(hbm), "fetch_bytes_raw_per_launch": int(fetch_raw),
        "write_bytes_per_launch": int(write),
        "alg_bytes_per_launch": bench["roofline"].get("alg_bytes_per_launch")
        or bench["roofline"]["algorithmic_bytes"]["per_launch"],
        "flop_per_launch": bench["roofline"].get("flop_per_launch"),
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
        # the kernel-trace run's own step time: the rocprof mean may not exceed it (same tree,
        # same speed)
        "rocprof_mean_le_ms_per_step": bool(mean_ms <= bench["ms_per_step"] * lps * 1.0005),
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
        f.write("Command: `bash tools/profile.sh` (bench.py --steps 3 --warmup 1 under rocprofv3 "
                "--kernel-trace --stats, then separate --pmc passes).\n\n")
        f.write("## rocprofv3 --kernel-trace --stats (all dispatches, incl. the counted pass)\n\n```\n")
        f.write(stats_csv)
        f.write("```\n\n## mesh_kernel, timed launches only\n\n```\n")
        f.write(json.dumps(summary, indent=1))
        f.write("\n```\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
