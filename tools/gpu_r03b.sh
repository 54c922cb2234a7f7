#!/bin/bash
# Round 3: parity suite on the register-pressure build, same-box A/B vs _snap/base, WRITE_SIZE of
# one C3 launch on both sides, bench plain vs in-process group (N = 1).  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/r03b"; mkdir -p "$O"; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== pytest"; timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; fatal $rc pytest
echo "== ab"; TAG=r03b/ab SIDES=". _snap/base" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh; fatal $? ab
for side in . _snap/base; do
  t=${side//[\/.]/x}
  echo "== write_size $t"
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_$t" -o run --output-format csv -- python3 $R/$side/tools/one_launch.py --spp 1024) > "$O/pmc_$t.log" 2>&1
  rc=$?; tail -2 "$O/pmc_$t.log"; fatal $rc "pmc $t"
done
for m in 0 1; do
  echo "== bench group=$m"; timeout -k 10 200 python -X faulthandler bench.py --secondary 0 --cpu-baseline 0 --steps 5 --group $m > "$O/bench_g$m.json" 2> "$O/bench_g$m.err"
  rc=$?; tail -c 400 "$O/bench_g$m.json"; echo; fatal $rc "bench $m"
done
echo "== done"
