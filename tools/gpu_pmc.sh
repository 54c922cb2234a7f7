#!/bin/bash
# rocprofv3 counter passes on the trace kernel (one --pmc group per run, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
stop_if_fatal() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
if [ "${LIST:-0}" = "1" ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; stop_if_fatal $? list
fi
CMD="python3 $R/tools/ab_variants.py --variants ${VARIANT:-1} --rounds 1 --spp ${SPP:-64}"
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pmc $i: $grp"
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --stats -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv -- $CMD) > "$R/gpurun_out/pmc/p$i.log" 2>&1
  rc=$?; tail -2 "$R/gpurun_out/pmc/p$i.log"; stop_if_fatal $rc "pmc $i"
done < "${PMC_FILE:-tools/pmc_groups.txt}"
echo "== done"
