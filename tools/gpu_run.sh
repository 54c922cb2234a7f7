#!/bin/bash
# One runner for every GPU measurement (replaces round 3's single-use gpu_r03*.sh scripts, which
# are in git history at commit 1b0d322).  Usage, from the repository root on the GPU box:
#   OUT=<dir under gpurun_out> tools/gpu_run.sh <step> [<step> ...]
# Steps (each under its own time limit; the script stops at the first failing step):
#   tests        pytest -m gpu (thread timeouts, one process)
#   smoke        __graft_entry__.smoke()
#   bench        python bench.py $BENCH_ARGS                      -> $O/bench.json
#   kprof        rocprofv3 --kernel-trace --stats of the bench (headline + C2 only, so the
#                headline kernel's average is its timed launches') -> $O/prof_bench/
#   pmc          rocprofv3 --pmc passes (one counter group per run) of the timed launches of the
#                workloads in $PMC (default "c3 c2 c5")            -> $O/pmc_<w>/p<i>/
#   ab           same-box A/B of the working tree against the snapshot $SNAP (tools/snap_rev.sh),
#                $PAIRS alternating process pairs of tools/ab_variants.py $AB_ARGS
#   py:<args>    python <args> (a tools/ probe), output -> $O/py_<n>.log, last line echoed
# Environment: OUT (default "run"), LIMIT (seconds per py: step, default 300).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/${OUT:-run}"; mkdir -p "$O"; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
SHA=$(python3 -c "import bench; print(bench.kernel_source_sha())")
n=0
for step in "$@"; do
  n=$((n+1))
  case "$step" in
    tests)
      echo "== pytest -m gpu"
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
      rc=$?; tail -2 "$O/pytest_gpu.log"; fatal $rc pytest;;
    smoke)
      echo "== smoke"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      rc=$?; tail -1 "$O/smoke.log"; fatal $rc smoke;;
    bench)
      echo "== bench ${BENCH_ARGS:-}"
      timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err"
      rc=$?; tail -c 400 "$O/bench.json"; echo; fatal $rc bench;;
    kprof)
      echo "== rocprofv3 kernel trace"
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_bench" -o run --output-format csv -- python3 "$R/bench.py" --cpu-baseline 0 --call-loop 0 --cold 0 --extra '') > "$O/prof_bench.log" 2>&1
      rc=$?; tail -1 "$O/prof_bench.log"; fatal $rc rocprof;;
    pmc)
      i=0
      for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
        i=$((i+1))
        for w in ${PMC:-c3 c2 c5}; do
          case $w in
            c3) cmd="$R/bench.py --steps 1 --warmup 1 --cpu-baseline 0 --secondary 0";;
            c2) cmd="$R/tools/one_launch.py --scene cornell_box --width 512 --height 512 --spp 64 --reps 2";;
            c5) cmd="$R/bench.py --config C5 --steps 1 --warmup 1 --cpu-baseline 0 --secondary 0";;
          esac
          mkdir -p "$O/pmc_$w"; echo "$SHA" > "$O/pmc_$w/kernel_sha.txt"
          echo "== pmc $w $i: $grp"
          (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-trace -d "$O/pmc_$w/p$i" -o run --output-format csv -- python3 $cmd) > "$O/pmc_${w}_p$i.log" 2>&1
          rc=$?; tail -1 "$O/pmc_${w}_p$i.log"; fatal $rc "pmc $w $i"
        done
      done;;
    ab)
      for i in $(seq 1 ${PAIRS:-3}); do
        for side in . "${SNAP:-_snap/base}"; do
          tag=$(echo "$side" | tr '/.' 'xx')
          (cd "$side" && timeout -k 10 300 python tools/ab_variants.py --variants 0 --rounds ${ROUNDS:-3} --spp ${SPP:-512} ${AB_ARGS:-} \
              > "$O/ab_${tag}_$i.log" 2>&1) || { echo "FATAL ab $side $i"; tail -5 "$O/ab_${tag}_$i.log"; exit 5; }
        done
      done
      grep -o '"Msamples_s": [0-9.]*' "$O"/ab_*.log;;
    abbench)
      # same-box A/B of whole bench runs (C3 headline only): working tree vs $SNAP, alternating
      for i in $(seq 1 ${PAIRS:-3}); do
        for side in . "${SNAP:-_snap/base}"; do
          tag=$(echo "$side" | tr '/.' 'xx')
          (cd "$side" && timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 2 --secondary 0 --cpu-baseline 0 \
              > "$O/abb_${tag}_$i.json" 2> "$O/abb_${tag}_$i.err") || { echo "FATAL abbench $side $i"; tail -5 "$O/abb_${tag}_$i.err"; exit 5; }
          echo "$side $i $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" "$O/abb_${tag}_$i.json")"
        done
      done;;
    py:*)
      args="${step#py:}"
      echo "== python $args"
      timeout -k 10 ${LIMIT:-300} python -u $args > "$O/py_$n.log" 2>&1
      rc=$?; tail -1 "$O/py_$n.log" | cut -c1-1500; fatal $rc "py $args";;
    *) echo "unknown step $step"; exit 2;;
  esac
done
echo "== done"
