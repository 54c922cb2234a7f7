#!/bin/bash
# Stress-scene A/B of the cache-read variants ($SV, default 34,41) and the full GPU parity suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
python tools/make_stress_scene.py /tmp/stress_100k.json > /dev/null && \
  timeout -k 10 300 python tools/ab_variants.py --scene /tmp/stress_100k.json --spp 32 --rounds 3 --variants ${SV:-34,41} > gpurun_out/abs.log 2>&1 || exit 3
tail -1 gpurun_out/abs.log
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
