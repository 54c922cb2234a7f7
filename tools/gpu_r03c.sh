#!/bin/bash
# Round 3: which register-pressure change costs time -- same-box A/B of base (round-2 kernel),
# noguard (packed order + float extents + store recompute, if/else range guards) and the working
# tree (+ fast-always range guards); VALU/SALU counts of one C3 launch each; group vs single bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/r03c"; mkdir -p "$O"; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== ab"; TAG=r03c/ab SIDES=". _snap/base _snap/noguard" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh; fatal $? ab
for side in . _snap/base _snap/noguard; do
  t=${side//[\/.]/x}
  echo "== insts $t"
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$O/pmc_$t" -o run --output-format csv -- python3 $R/$side/tools/one_launch.py --spp 1024) > "$O/pmc_$t.log" 2>&1
  rc=$?; tail -1 "$O/pmc_$t.log"; fatal $rc "pmc $t"
done
for m in 0 1 0 1; do
  echo "== bench group=$m"; timeout -k 10 200 python bench.py --secondary 0 --cpu-baseline 0 --steps 5 --group $m > "$O/bench_g$m.json" 2> "$O/bench_g$m.err"
  rc=$?; python -c "import json;d=json.load(open('$O/bench_g$m.json'));print(d['value'],d['ms_per_step'],d.get('group_timing'))"; fatal $rc "bench $m"
done
echo "== done"
