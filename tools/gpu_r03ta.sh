#!/bin/bash
# Vector-memory pipeline load of the C3 timed launch: which TA/TD/TCP counters gfx950 offers, then
# one pass with the address and data units' busy counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/r03ta"; mkdir -p "$O"; export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 60 rocprofv3 -L) > "$O/list.txt" 2>&1 || true
grep -o "\bT[ACD][A-Z_]*BUSY[A-Za-z_]*\|\bTCP_[A-Z_]*\b" "$O/list.txt" | sort -u | head -60
cmd="$R/bench.py --steps 1 --warmup 0 --cpu-baseline 0 --secondary 0"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace -d "$O/p1" -o run --output-format csv -- python3 $cmd) > "$O/p1.log" 2>&1
rc=$?; tail -2 "$O/p1.log"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py "$O/p1" "trace_kernel<false" | head -20
echo "== done"
