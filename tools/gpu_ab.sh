#!/bin/bash
# Variant A/B + GPU parity tests.  Each GPU step time-limited; fatal exits stop the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== ab generated"; timeout -k 10 300 python tools/ab_variants.py ${AB_ARGS:-} > gpurun_out/ab.log 2>&1
rc=$?; tail -3 gpurun_out/ab.log; stop_if_fatal $rc ab
echo "== ab cornell"; timeout -k 10 300 python tools/ab_variants.py --scene scenes/cornell_box.scene.json --width 512 --height 512 --spp 64 ${AB_ARGS:-} > gpurun_out/ab_cornell.log 2>&1
rc=$?; tail -3 gpurun_out/ab_cornell.log; stop_if_fatal $rc ab_cornell
if [ -n "${SIMD_VARIANTS:-}" ]; then echo "== simd efficiency"; timeout -k 10 300 python tools/simd_eff.py --variants ${SIMD_VARIANTS:-3,6} > gpurun_out/simd.log 2>&1
rc=$?; cat gpurun_out/simd.log | tail -40; stop_if_fatal $rc simd; fi
if [ -n "${STRESS_VARIANTS:-}" ]; then
echo "== stress scene"; python tools/make_stress_scene.py /tmp/stress_100k.json > /dev/null && \
  timeout -k 10 600 python tools/ab_variants.py --scene /tmp/stress_100k.json --spp 32 --rounds 3 --variants $STRESS_VARIANTS > gpurun_out/ab_stress.log 2>&1
rc=$?; tail -1 gpurun_out/ab_stress.log; stop_if_fatal $rc stress
fi
if [ "${RUN_TESTS:-1}" = "1" ]; then
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q -rf --maxfail=6 ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
fi
echo "== done"
