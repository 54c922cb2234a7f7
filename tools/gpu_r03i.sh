#!/bin/bash
# Does raised issue priority shorten the heaviest tiles?  Per-schedule tile times (max, top-1 % mean,
# mean) on C3 at 256 and 1024 spp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03i; mkdir -p $O
for spp in 256 1024; do
  timeout -k 10 300 python tools/sched_probe.py --spp $spp --scheds p0,p64,p256,p1024,p4096 --rounds 3 > $O/prio_$spp.json 2> $O/prio_$spp.err || { echo FATAL; tail -3 $O/prio_$spp.err; exit 5; }
  cut -c1-2000 $O/prio_$spp.json
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; exit $rc
