#!/bin/bash
# Experiment runner: each line of $EXP is one ab_variants.py argument list, run under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "== $i: $line"
  timeout -k 10 ${STEP_LIMIT:-240} python tools/ab_variants.py $line > gpurun_out/exp_$i.log 2>&1
  rc=$?; tail -1 gpurun_out/exp_$i.log
  [ $rc -ne 0 ] && { echo "FATAL step $i rc=$rc"; tail -5 gpurun_out/exp_$i.log; exit $rc; }
done < "${1:-tools/exp.txt}"
echo "== done"
