#!/bin/bash
# Variant 49 (6 waves/SIMD) against the default, then the round-3 measurement pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 300 python tools/ab_variants.py --variants 40,41,49 --rounds 3 --spp 1024 > $O/ab_c3.log 2>&1 || { echo FATAL ab; tail -5 $O/ab_c3.log; exit 5; }
tail -3 $O/ab_c3.log | cut -c1-600
bash tools/gpu_r03_final.sh
