#!/bin/bash
# A/B of the deferred-shading variants on the bench scenes (each step time-limited; stops on a fatal exit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 python tools/ab_variants.py "$@" > gpurun_out/$name.log 2>&1
  local rc=$?; tail -1 gpurun_out/$name.log; [ $rc -eq 0 ] || { echo "FATAL $name $rc"; exit $rc; }; }
run d_gen --variants ${GEN_V:-40,63,56} --rounds 5
run d_cornell --scene scenes/cornell_box.scene.json --width 512 --height 512 --spp 64 --variants ${CB_V:-48,73,47,72} --rounds 5
run d_n8 --spp 1024 --n 8 --rank 0 --variants ${N8_V:-47,72} --rounds 3
python tools/make_stress_scene.py /tmp/stress_100k.json > /dev/null || exit 3
run d_stress --scene /tmp/stress_100k.json --spp 32 --rounds 3 --variants ${ST_V:-46,71,75,41,70,74}
echo "== done"
