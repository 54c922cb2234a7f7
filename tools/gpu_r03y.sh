#!/bin/bash
# Tile-time statistics of the shipped schedule (max tile, top 1 %, mean -> sum / slots) on the C3
# image, its N = 2 share and the C4 N = 8 share: how close each launch is to its longest tile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 150 python tools/sched_probe.py --scheds a,o --rounds 3 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 4; }
tail -1 $O/c3.log
timeout -k 10 150 python tools/sched_probe.py --scheds a,o --rounds 3 --n 2 > $O/c3n2.log 2>&1 || { tail -5 $O/c3n2.log; exit 4; }
tail -1 $O/c3n2.log
timeout -k 10 300 python tools/sched_probe.py --scheds a --rounds 2 --n 8 --width 3840 --height 2160 --spp 4096 > $O/c4n8.log 2>&1 || { tail -5 $O/c4n8.log; exit 4; }
tail -1 $O/c4n8.log
echo "== done"
