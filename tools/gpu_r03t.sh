#!/bin/bash
# Leaf loop fetching the next position's primitive record while testing the current one: GPU parity
# suite, then same-box A/B against HEAD's build (_snap/base).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
TAG=r03t/ab SIDES=". _snap/base" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh || exit 5
echo "== done"
