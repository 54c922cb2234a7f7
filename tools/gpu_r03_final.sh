#!/bin/bash
# Round-3 measurement pass: parity suite, smoke, bench (C3 + C2 + C5 records with CPU baselines),
# rocprofv3 kernel-trace stats of the bench, PMC passes of the C3, C2 and C5 timed launches.  Each
# GPU step has its own limit; a fatal exit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/${OUT:-r03f}"; mkdir -p "$O"; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
SHA=$(python3 -c "import bench; print(bench.kernel_source_sha())")
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -2 "$O/pytest_gpu.log"; fatal $rc pytest
  echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
  rc=$?; tail -1 "$O/smoke.log"; fatal $rc smoke
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
echo "== bench"; timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; tail -c 300 "$O/bench.json"; echo; fatal $rc bench
echo "== rocprofv3 kernel trace"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_bench" -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 --extra '') > "$O/prof_bench.log" 2>&1
rc=$?; tail -1 "$O/prof_bench.log"; fatal $rc rocprof
fi
[ "${SKIP_PMC:-0}" = "1" ] && { echo "== done"; exit 0; }
i=0
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  for w in c3 c2 c5; do
    case $w in
      c3) cmd="$R/bench.py --steps 1 --warmup 0 --cpu-baseline 0 --secondary 0";;
      c2) cmd="$R/tools/one_launch.py --scene cornell_box --width 512 --height 512 --spp 64";;
      c5) cmd="$R/bench.py --config C5 --steps 1 --warmup 0 --cpu-baseline 0 --secondary 0";;
    esac
    mkdir -p "$O/pmc_$w"; echo "$SHA" > "$O/pmc_$w/kernel_sha.txt"
    echo "== pmc $w $i: $grp"
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d "$O/pmc_$w/p$i" -o run --output-format csv -- python3 $cmd) > "$O/pmc_${w}_p$i.log" 2>&1
    rc=$?; tail -1 "$O/pmc_${w}_p$i.log"; fatal $rc "pmc $w $i"
  done
done
echo "== done"
