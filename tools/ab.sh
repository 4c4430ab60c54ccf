#!/bin/bash
# tools/ab.sh SCENE STEPS VARIANT... — on the GPU box: tools/sweep.py once per experiment
# variant library (qt-raytracer_amd/libv_VARIANT.so), twice in alternating order to expose drift.
set -uo pipefail
scene=$1; steps=$2; shift 2
for pass in 1 2; do
    for v in "$@"; do
        printf '%s pass%s ' "$v" "$pass"
        HIPPT_LIB=qt-raytracer_amd/libv_$v.so timeout -k 10 120 python tools/sweep.py --scene "$scene" --steps "$steps" || exit 1
    done
done
