#!/bin/bash
# Quick GPU pass: parity tests, smoke, default bench.  Each step has its own limit; a fatal exit stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out"; mkdir -p "$O"
export TMPDIR=/tmp
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=5 --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -8 "$O/pytest_gpu.log"; stop_if_fatal $rc pytest
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
rc=$?; tail -2 "$O/smoke.log"; stop_if_fatal $rc smoke
echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.log" 2>&1
rc=$?; tail -1 "$O/bench.log"; stop_if_fatal $rc bench
echo "== done"
