#!/bin/bash
# C2 (cornell 512x512x64): which variant for the small grid (automatic = 48 since round 2) after the
# round-3 schedule changes; in-process alternating A/B, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03v; mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python tools/ab_variants.py --variants 0,39,40,47,48 --rounds 6 --spp 64 --width 512 --height 512 --scene scenes/cornell_box.scene.json > $O/ab_c2_$i.log 2>&1 || { tail -5 $O/ab_c2_$i.log; exit 4; }
  tail -1 $O/ab_c2_$i.log
done
echo "== done"
