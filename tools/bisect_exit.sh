#!/bin/bash
# Runs groups of GPU parity tests in separate processes and reports each process's exit status
# (a heap corruption shows as 134 at interpreter exit).  Usage on the GPU box:
#   OUT=<dir> tools/bisect_exit.sh <pytest -k expr> [<expr> ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${OUT:-bisect}"; mkdir -p "$O"
i=0
for k in "$@"; do
  i=$((i+1))
  MALLOC_CHECK_=3 timeout -k 10 300 python -u -m pytest -x -q tests/test_gpu_parity.py --timeout 200 -k "$k" > "$O/b_$i.log" 2>&1
  rc=$?
  echo "[$k] rc=$rc $(tail -1 "$O/b_$i.log")"
  if [ $rc -ne 0 ] && [ $rc -ne 134 ] && [ $rc -ne 1 ]; then echo "stop"; exit $rc; fi
done
