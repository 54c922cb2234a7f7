#!/bin/bash
# Strong-scaling projections with the round-3 kernel and schedule (refined cost order, graded
# priority): every rank's exact share rendered on one MI355X (tools/scale_sim.py), C3 with sample
# groups automatic and off, and C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${OUT:-r03m}; mkdir -p $O
timeout -k 10 300 python tools/scale_sim.py --width 1920 --height 1080 --spp 1024 --partitions bands:8 --ssg 0 > $O/c3_ssg_auto.log 2>&1 || { echo FATAL c3; tail -3 $O/c3_ssg_auto.log; exit 5; }
tail -1 $O/c3_ssg_auto.log | cut -c1-900
timeout -k 10 300 python tools/scale_sim.py --width 1920 --height 1080 --spp 1024 --partitions bands:8 --ssg 1 --ns 4,8 > $O/c3_ssg_off.log 2>&1 || { echo FATAL c3off; exit 5; }
tail -1 $O/c3_ssg_off.log | cut -c1-900
timeout -k 10 500 python tools/scale_sim.py --partitions bands:8 --ssg 0 > $O/c4.log 2>&1 || { echo FATAL c4; tail -3 $O/c4.log; exit 5; }
tail -1 $O/c4.log | cut -c1-900
