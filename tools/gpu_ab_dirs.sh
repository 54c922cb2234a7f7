#!/bin/bash
# Same-box A/B over several prebuilt trees (DIRS="_snap/a _snap/b ." ...), alternating, 3 rounds;
# ARGS are tools/ab_variants.py arguments.  Each run time-limited; a failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
R=$PWD
for i in 1 2 3; do
  for d in $DIRS; do
    tag=$(echo "$d" | tr '/.' '__')
    (cd "$d" && timeout -k 10 200 python tools/ab_variants.py $ARGS > "$R/gpurun_out/abd_${tag}_$i.log" 2>&1) \
      || { echo "FATAL $d $i"; tail -5 "$R/gpurun_out/abd_${tag}_$i.log"; exit 5; }
    echo "$d $i $(grep -o '"Msamples_s": [0-9.]*' "$R/gpurun_out/abd_${tag}_$i.log" | tr '\n' ' ')"
  done
done
