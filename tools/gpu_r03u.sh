#!/bin/bash
# Leaf compaction (variant 50): GPU parity suite, in-process A/B against variant 40 on C3 and C5's
# scene, leaf-round counters of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/ab_variants.py --variants 40,50 --rounds 4 --spp 512 > $O/ab_c3.log 2>&1 || { tail -5 $O/ab_c3.log; exit 4; }
tail -3 $O/ab_c3.log
timeout -k 10 120 python tools/simd_eff.py --spp 8 --variants 40,50 > $O/eff_c3.json 2> $O/eff_c3.err || exit 5
python -c "import bench; print(bench.scene_path('stress_100k'))" > /dev/null || exit 6
timeout -k 10 300 python tools/ab_variants.py --variants 41,51 --rounds 3 --spp 64 --scene /tmp/pt_stress_100k.json > $O/ab_c5.log 2>&1 || { tail -5 $O/ab_c5.log; exit 7; }
tail -3 $O/ab_c5.log
timeout -k 10 120 python tools/ab_variants.py --variants 40,50 --rounds 4 --spp 64 --width 512 --height 512 --scene scenes/cornell_box.scene.json > $O/ab_c2.log 2>&1 || { tail -5 $O/ab_c2.log; exit 8; }
tail -3 $O/ab_c2.log
echo "== done"
