#!/usr/bin/env python3
"""BASELINE configs[0] on the reference CPU path tracer itself: Cornell-34, 256x256, 4 spp, 4 bounces,
the whole image, through oracle/_ref/ref_harness bench (the unmodified RayTracer.h ray_color + a
Qt-free copy of RenderWorker::render's tile pool, RayTracerFboItem.cpp:46-144,397-427), median of
--runs runs at each thread count: the box's CPU share (OMP_NUM_THREADS, 16 on the GPU box) and the
whole affinity mask.  One JSON line per thread count.

usage: python tools/ref_cpu_config0.py [--runs 3] [--threads 16,256]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "qt-raytracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)
import pyoracle  # noqa: E402  (baseline tooling: the reference harness's path)
from bench import host_cpu_facts  # noqa: E402
from hippt import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--threads", default="")
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--depth", type=int, default=4)
    a = ap.parse_args()
    facts = host_cpu_facts()
    counts = [int(t) for t in a.threads.split(",") if t] or sorted(
        {t for t in (facts["omp_num_threads"], facts["affinity"]) if t})
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "cornell34.bin")
        scenes.write_scene_file(scenes.cornell34(), path)
        for n in counts:
            rs = []
            for _ in range(a.runs):
                out = subprocess.run([pyoracle.REF_HARNESS, "bench", path, str(a.width), str(a.height), "1",
                                      str(a.spp), str(a.depth), str(n)], capture_output=True, text=True,
                                     check=True, timeout=600).stdout
                rs.append(json.loads(out.strip().splitlines()[-1]))
            rs.sort(key=lambda r: r["msamples_per_s"])
            m = rs[len(rs) // 2]
            print(json.dumps({"config": "configs[0] cornell34 256x256 4spp depth4 (whole image)", "threads": n,
                              "msamples_per_s": round(m["msamples_per_s"], 3),
                              "mpixel_samples_per_s": round(m["mpixel_samples_per_s"], 3),
                              "seconds": round(m["seconds"], 4), "segments": m["segments"],
                              "runs_msamples_per_s": [round(r["msamples_per_s"], 3) for r in rs],
                              "tile": m["tile"], "host": facts}), flush=True)


if __name__ == "__main__":
    main()
