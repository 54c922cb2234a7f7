#!/bin/bash
# Companion scheduling (pt_set_companion) against the shipped schedule, with launch timelines:
# C3 1080p, its N = 2 share, the C4 N = 8 share.  Results are checked bit-identical per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03z; mkdir -p $O
run() { local name=$1; shift
  timeout -k 10 240 python tools/sched_probe.py --spans "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 4; }
  tail -1 $O/$name.log | cut -c1-3000; }
run c3 --scheds a,c1_256,c1_1024,c2_256,c2_64 --rounds 3
run c3n2 --n 2 --scheds a,c1_256,c1_1024,c2_256 --rounds 3
run c4n8 --n 8 --width 3840 --height 2160 --spp 4096 --scheds a,c1_256,c2_256 --rounds 2
echo "== done"
