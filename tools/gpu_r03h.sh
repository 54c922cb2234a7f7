#!/bin/bash
# Scheduler-flag A/B: the working tree against three snapshots built with extra LLVM options.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03h/ab SIDES=". _snap/maxilp _snap/trackers _snap/bias0" PAIRS=3 SPP=512 bash tools/gpu_ab_snap.sh || exit 5
echo "== done"
