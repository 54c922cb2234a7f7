#!/bin/bash
# Bench with the refined cost order, then issue priority on top of it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03k; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --secondary 0 --cpu-baseline 0 --steps 5 > $O/bench_$i.json 2> $O/bench_$i.err || { echo FATAL bench; tail -3 $O/bench_$i.err; exit 5; }
  python -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'],d['ms_per_step'])"
done
timeout -k 10 300 python tools/sched_probe.py --scheds p0,p256,p1024,p4096 --rounds 4 > $O/prio.json 2> $O/prio.err || { echo FATAL; exit 5; }
cut -c1-1500 $O/prio.json
timeout -k 10 300 python tools/sched_probe.py --n 2 --scheds p0,p256,p1024,p4096 --rounds 4 > $O/prio_n2.json 2> $O/prio_n2.err || { echo FATAL; exit 5; }
cut -c1-1500 $O/prio_n2.json
