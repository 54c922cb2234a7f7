#!/bin/bash
# Full GPU pass: parity tests, smoke, default bench, rocprofv3 kernel trace + PMC traffic of the
# bench command, C5 stress-scene timing.  Each GPU step has its own limit; fatal exits stop here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== pytest -m gpu"; timeout -k 10 1200 python -m pytest tests -m gpu -q -rf --maxfail=10 > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -15 "$O/pytest_gpu.log"; stop_if_fatal $rc pytest
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; stop_if_fatal $rc smoke
echo "== bench"; timeout -k 10 600 python bench.py > "$O/bench.log" 2>&1
rc=$?; tail -2 "$O/bench.log"; stop_if_fatal $rc bench
BENCH="$R/bench.py --steps 1 --warmup 0 --cpu-baseline 0"
echo "== rocprofv3 kernel trace"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_bench" -o run --output-format csv -- python3 $BENCH) > "$O/prof_bench.log" 2>&1
rc=$?; tail -1 "$O/prof_bench.log"; stop_if_fatal $rc rocprof
i=0
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1)); echo "== pmc $i: $grp"
  (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $grp --kernel-trace -d "$O/pmc_bench/p$i" -o run --output-format csv -- python3 $BENCH) > "$O/pmc_bench_p$i.log" 2>&1
  rc=$?; tail -1 "$O/pmc_bench_p$i.log"; stop_if_fatal $rc "pmc $i"
done
echo "== stress scene"; python tools/make_stress_scene.py /tmp/stress_100k.json > /dev/null && \
  timeout -k 10 600 python tools/ab_variants.py --scene /tmp/stress_100k.json --spp 32 --rounds 3 --variants ${STRESS_VARIANTS:-3,4} > "$O/ab_stress.log" 2>&1
rc=$?; tail -1 "$O/ab_stress.log"; stop_if_fatal $rc stress
echo "== done"
