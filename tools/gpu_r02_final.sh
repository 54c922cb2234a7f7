#!/bin/bash
# Round-2 measurement pass after a kernel change: parity suite, sample-group A/B (deferral on/off),
# smoke, bench, rocprofv3 kernel trace of the bench, PMC passes of the bench (C3) and of one C2
# launch.  Each GPU step has its own limit; a fatal exit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== pytest -m gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; fatal $rc pytest
for n in 8 4; do
  echo "== ssg ab n=$n"; timeout -k 10 200 python tools/ab_variants.py --spp 1024 --n $n --rank 0 --groups 0 --variants 39,40 --rounds 3 > "$O/ssg_ab_n$n.log" 2>&1
  rc=$?; tail -1 "$O/ssg_ab_n$n.log"; fatal $rc "ssg ab $n"
done
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -1 "$O/smoke.log"; fatal $rc smoke
echo "== bench"; timeout -k 10 400 python bench.py > "$O/bench.log" 2>&1
rc=$?; tail -1 "$O/bench.log" | cut -c1-300; fatal $rc bench
BENCH="$R/bench.py --steps 1 --warmup 0 --cpu-baseline 0 --secondary 0"
C2="$R/tools/one_launch.py --scene cornell_box --width 512 --height 512 --spp 64"
echo "== rocprofv3 kernel trace"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_bench" -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0) > "$O/prof_bench.log" 2>&1
rc=$?; tail -1 "$O/prof_bench.log"; fatal $rc rocprof
i=0
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  for w in bench c2; do
    cmd=$BENCH; [ $w = c2 ] && cmd=$C2
    echo "== pmc $w $i: $grp"
    (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-trace -d "$O/pmc_$w/p$i" -o run --output-format csv -- python3 $cmd) > "$O/pmc_${w}_p$i.log" 2>&1
    rc=$?; tail -1 "$O/pmc_${w}_p$i.log"; fatal $rc "pmc $w $i"
  done
done
echo "== done"
