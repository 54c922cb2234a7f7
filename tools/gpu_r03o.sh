#!/bin/bash
# Deferred-shading and traversal-exit parameters of the default walk (kV40Walk), same-box A/B against
# four snapshots with one parameter moved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03p/ab SIDES=". _snap/w14216 _snap/w15216 _snap/w14212 _snap/w24216 _snap/w4216" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh || exit 5
echo "== done"
