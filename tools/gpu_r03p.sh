#!/bin/bash
# Pops folded into the walk (variants 42/43): parity, then in-process A/B against 40/41 on C3, C5
# geometry and cornell.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "variant" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python tools/ab_variants.py --variants 40,42 --rounds 4 --spp 1024 > $O/ab_c3_$i.log 2>&1 || { tail -5 $O/ab_c3_$i.log; exit 4; }
  tail -1 $O/ab_c3_$i.log
done
timeout -k 10 200 python tools/ab_variants.py --variants 41,43 --rounds 3 --spp 64 --scene $(python3 -c "import bench; print(bench.scene_path('stress_100k'))") > $O/ab_c5.log 2>&1 || { tail -5 $O/ab_c5.log; exit 4; }
tail -1 $O/ab_c5.log
timeout -k 10 200 python tools/ab_variants.py --variants 40,42 --rounds 6 --spp 64 --width 512 --height 512 --scene scenes/cornell_box.scene.json > $O/ab_c2.log 2>&1 || { tail -5 $O/ab_c2.log; exit 4; }
tail -1 $O/ab_c2.log
echo "== done"
