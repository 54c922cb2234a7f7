#!/bin/bash
# One GPU pass, steps chosen by $STEPS (space-separated): env tests smoke bench scale prof pmc pmc_c2 stress.
# Every GPU step has its own time limit; a crash / abort / timeout stops the script (no retries).
# Output: gpurun_out/$TAG/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/${TAG:-pass}"; mkdir -p "$O"
export TMPDIR=/tmp
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
BENCH="$R/bench.py --steps 1 --warmup 0 --cpu-baseline 0 --secondary 0"
for step in ${STEPS:-tests smoke bench}; do
  echo "== $step $(date +%T)"
  case $step in
  env)
    { nproc; python3 -c 'import os;print("affinity",len(os.sched_getaffinity(0)))'; cat /sys/fs/cgroup/cpu.max 2>&1;
      grep -m1 "model name" /proc/cpuinfo; rocm-smi --showclocks 2>&1 | head -20; } > "$O/env.txt" 2>&1; cat "$O/env.txt";;
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$O/pytest_gpu.log" 2>&1
    rc=$?; grep -E "PASSED|FAILED|ERROR" "$O/pytest_gpu.log" | tail -60; tail -5 "$O/pytest_gpu.log"; stop_if_fatal $rc pytest;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
    rc=$?; tail -2 "$O/smoke.log"; stop_if_fatal $rc smoke;;
  bench)
    timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1
    rc=$?; tail -3 "$O/bench.log"; stop_if_fatal $rc bench;;
  scale)
    timeout -k 10 600 python tools/scale_sim.py ${SCALE_ARGS:-} > "$O/scale_sim.log" 2>&1
    rc=$?; tail -1 "$O/scale_sim.log"; stop_if_fatal $rc scale;;
  prof)
    (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 $BENCH ${PROF_ARGS:-}) > "$O/prof.log" 2>&1
    rc=$?; tail -2 "$O/prof.log"; stop_if_fatal $rc rocprof;;
  pmc|pmc_c2)
    EXTRA=""; [ "$step" = pmc_c2 ] && EXTRA="--config C2 --steps 3"
    i=0
    for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
      i=$((i+1)); echo "-- $step $i: $grp"
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d "$O/$step/p$i" -o run --output-format csv -- python3 $BENCH $EXTRA) > "$O/${step}_p$i.log" 2>&1
      rc=$?; tail -1 "$O/${step}_p$i.log"; stop_if_fatal $rc "$step $i"
    done;;
  stress)
    timeout -k 10 600 python bench.py --config C5 --spp ${STRESS_SPP:-256} --steps 2 --warmup 1 --cpu-baseline 0 --secondary 0 > "$O/stress.log" 2>&1
    rc=$?; tail -1 "$O/stress.log"; stop_if_fatal $rc stress;;
  esac
done
echo "== done $(date +%T)"
