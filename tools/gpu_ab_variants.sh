#!/bin/bash
# Interleaved A/B of trace-kernel variants $V (default 30) on generated_scene 1080p and cornell 512^2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
V="${V:-30}"
timeout -k 10 300 python tools/ab_variants.py --variants $V --rounds ${ROUNDS:-5} > gpurun_out/abv.log 2>&1 || { echo "FATAL $?"; cat gpurun_out/abv.log | tail; exit 1; }
tail -1 gpurun_out/abv.log
timeout -k 10 300 python tools/ab_variants.py --variants $V --rounds ${ROUNDS:-5} --scene scenes/cornell_box.scene.json --width 512 --height 512 > gpurun_out/abvc.log 2>&1 || { echo "FATAL $?"; exit 1; }
tail -1 gpurun_out/abvc.log
