#!/bin/bash
# Leaf-round counters of the default kernel (instrumented variant 40 / 41): lanes and pairs per leaf
# round, family-path executions as run, with a whole-wave compaction and with one over the round's
# lanes; phase cycle shares.  C3 at 8 and 64 spp, C2, C5's scene.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 120 python tools/simd_eff.py --spp 8 > $O/c3_8.json 2> $O/c3_8.err || exit 3
timeout -k 10 120 python tools/simd_eff.py --spp 8 --chunks 8 > $O/c3_64.json 2> $O/c3_64.err || exit 3
timeout -k 10 120 python tools/simd_eff.py --scene scenes/cornell_box.scene.json --width 512 --height 512 --spp 8 --chunks 8 --variants 40,48 > $O/c2.json 2> $O/c2.err || exit 3
python -c "import bench; print(bench.scene_path('stress_100k'))" > $O/c5_path.txt || exit 4
timeout -k 10 240 python tools/simd_eff.py --scene /tmp/pt_stress_100k.json --spp 8 --variants 41 > $O/c5.json 2> $O/c5.err || exit 3
echo "== done"
