#!/bin/bash
# Cost order refined from long launches: one_launch.py (8-spp first launch, then 1024-spp launches)
# on the working tree and on the previous commit (_snap/always), alternating; C3 and the N = 2 share.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r03j; mkdir -p $O
for i in 1 2; do
  for side in . _snap/always; do
    t=${side//[\/.]/x}
    (cd $side && timeout -k 10 200 python tools/one_launch.py --reps 8 > $O/c3_${t}_$i.log 2>&1) || { echo FATAL; exit 5; }
    echo "$t $i: $(grep -o '"ms": [0-9.]*' $O/c3_${t}_$i.log | tr '\n' ' ')"
  done
done
