#!/bin/bash
# Round 3: tile-schedule sweep (tools/sched_probe.py: issue priority, CU-masked split launches) on
# C3 (N = 1 and rank shares at N = 2, 4), the C4 rank share at N = 8 and C2; A/B of the build without
# SLP vectorisation.  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/r03e"; mkdir -p "$O"; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
run() { name=$1; shift; echo "== $name"; timeout -k 10 300 python tools/sched_probe.py "$@" > "$O/$name.json" 2> "$O/$name.err"; rc=$?; cut -c1-600 "$O/$name.json"; fatal $rc $name; }
echo "== parity (schedule knobs)"; timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "schedule_knobs or persistent or tile_schedule" --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?; tail -2 "$O/pytest.log"; fatal $rc pytest
S="p0,p64,p256,p1024,r16w1,r32w1,r32w2,r64w2"
run c3_n1 --scheds $S
run c3_n2 --n 2 --scheds $S
run c3_n4 --n 4 --scheds $S
run c4_n8 --width 3840 --height 2160 --spp 4096 --n 8 --scheds $S --rounds 2
run c2 --scene scenes/cornell_box.scene.json --width 512 --height 512 --spp 64 --scheds p0,p64,p256,r16w1
echo "== sweep done"
echo "== ab noslp"; TAG=r03e/ab SIDES=". _snap/noslp" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh; fatal $? ab
echo "== done"
