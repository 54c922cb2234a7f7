#!/bin/bash
# Deferred-shading and traversal-exit parameters of the default walk (kV40Walk), same-box A/B against
# four snapshots with one parameter moved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03o/ab SIDES=". _snap/w14216 _snap/w12216 _snap/w13220 _snap/w13212" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh || exit 5
echo "== done"
