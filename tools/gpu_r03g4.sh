#!/bin/bash
# Grouped (sample-group) launches compiled for 4 waves per SIMD (variant 47's walk, no spill) against
# the shipped 5-wave grouped kernel (variant 39) on the C3 rank shares at N = 8 and N = 4, in the
# snapshot _snap/g4 (tools/snap_rev.sh with the two edits); results cross-checked bit-identical.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r03g4"; mkdir -p $O
cd _snap/g4
for n in 8 4; do
  timeout -k 10 200 python tools/ab_variants.py --variants 39,47 --groups 0 --n $n --spp 1024 --rounds 4 > $O/n$n.log 2>&1 || { tail -5 $O/n$n.log; exit 4; }
  tail -1 $O/n$n.log
done
echo "== done"
