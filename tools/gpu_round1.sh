#!/bin/bash
# First GPU pass: smoke, GPU parity tests, a short bench, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash / timeout stops the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit code, $2 = step; pytest's 1 (= failed tests) is not fatal
    if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi
}
echo "== smoke"; timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; cat gpurun_out/smoke.log | tail -5; stop_if_fatal $rc smoke
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -rf --maxfail=6 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
echo "== bench"; timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; stop_if_fatal $rc bench
echo "== rocprofv3"; cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --cpu-baseline 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?; tail -5 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; stop_if_fatal $rc rocprof
echo "== done"
