#!/bin/bash
# Same-box A/B of the working tree's prebuilt libraries against the prebuilt snapshot in _ab_old/
# (no rebuild on the box), alternating sides; then the GPU parity suite.  Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
R=$PWD
for i in 1 2 3; do
  for side in new old; do
    dir=.; [ $side = old ] && dir=_ab_old
    (cd "$dir" && timeout -k 10 200 python tools/ab_variants.py --variants ${VARIANTS:-0} --rounds 5 --spp ${SPP:-64} \
        > "$R/gpurun_out/snap_${side}_$i.log" 2>&1) || { echo "FATAL $side $i"; exit 5; }
  done
done
grep -o '"Msamples_s": [0-9.]*' gpurun_out/snap_*.log
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
fi
