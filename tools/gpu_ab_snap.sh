#!/bin/bash
# Same-box A/B of the working tree against the prebuilt snapshot in _snap/ (alternating sides,
# separate processes), then optional probes.  Each step time-limited; stops on a fatal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O="$R/gpurun_out/${TAG:-ab}"; mkdir -p "$O"; export TMPDIR=/tmp
for i in $(seq 1 ${PAIRS:-3}); do
  for side in ${SIDES:-. _snap}; do
    dir=$side
    (cd "$dir" && timeout -k 10 200 python tools/ab_variants.py --variants 0 --rounds ${ROUNDS:-3} --spp ${SPP:-512} ${AB_ARGS:-} \
        > "$O/snap_${side//[\/.]/x}_$i.log" 2>&1) || { echo "FATAL $side $i"; tail -5 "$O/snap_${side//[\/.]/x}_$i.log"; exit 5; }
  done
done
grep -o '"Msamples_s": [0-9.]*' "$O"/snap_*.log
if [ -n "${PROBES:-}" ]; then
  j=0
  while IFS= read -r args; do
    [ -z "$args" ] && continue; j=$((j+1)); echo "== probe $j: $args"
    timeout -k 10 300 python tools/tail_probe.py $args > "$O/probe_$j.log" 2>&1 || { echo "FATAL probe $j"; tail -5 "$O/probe_$j.log"; exit 6; }
    tail -1 "$O/probe_$j.log"
  done <<< "$PROBES"
fi
echo "== done"
