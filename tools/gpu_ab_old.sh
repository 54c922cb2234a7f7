#!/bin/bash
# Same-box A/B of the working tree against the snapshot in _ab_old/ (tools/ab_compare.sh), then
# the exhaustive FP check and the GPU parity suite.  Each GPU step time-limited; stops on failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== ab"; timeout -k 10 600 bash tools/ab_compare.sh > gpurun_out/abcmp.log 2>&1; rc=$?; cat gpurun_out/abcmp.log | tail -8
[ $rc -eq 0 ] || { echo "FATAL ab rc=$rc"; exit $rc; }
if [ "${RUN_TESTS:-1}" = "1" ]; then
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; exit $rc
fi
