#!/bin/bash
# C5 (100k quadrics): the cache-read walk (variants 41/46) with the retuned deferral (14212) against
# the shipped 13212; same-box A/B at 512 spp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
python -c "import bench; print(bench.scene_path('stress_100k'))" || exit 4
TAG=r03q/ab SIDES=". _snap/c5d4" PAIRS=3 SPP=512 AB_ARGS="--scene /tmp/pt_stress_100k.json" bash tools/gpu_ab_snap.sh || exit 5
echo "== done"
