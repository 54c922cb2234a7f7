#!/bin/bash
# Runs GPU parity tests one process per test and reports each process's exit status (a heap
# corruption shows as 134 at interpreter exit).  Usage on the GPU box:
#   OUT=<dir> tools/bisect_exit.sh [<pytest -k expr>]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="gpurun_out/${OUT:-bisect}"; mkdir -p "$O"
python -m pytest -q --collect-only tests/test_gpu_parity.py -k "${1:-gpu or not gpu}" 2>/dev/null | grep "::" > "$O/ids.txt"
i=0
while read -r id; do
  i=$((i+1))
  MALLOC_CHECK_=3 timeout -k 10 200 python -u -m pytest -x -q "$id" --timeout 150 > "$O/b_$i.log" 2>&1
  rc=$?
  echo "rc=$rc $id"
  if [ $rc -ne 0 ] && [ $rc -ne 134 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "stop"; exit $rc; fi
done < "$O/ids.txt"
