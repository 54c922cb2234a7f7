#!/bin/bash
# Instruction-cache behaviour of the C3 timed launch (the default kernel is ~5,300 instructions).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/r03ic"; mkdir -p "$O"; export TMPDIR=/tmp
cmd="$R/bench.py --steps 1 --warmup 0 --cpu-baseline 0 --secondary 0"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE --kernel-trace -d "$O/p1" -o run --output-format csv -- python3 $cmd) > "$O/p1.log" 2>&1
rc=$?; tail -2 "$O/p1.log"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py "$O/p1" "trace_kernel<false" | head -20
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --kernel-trace -d "$O/p2" -o run --output-format csv -- python3 $cmd) > "$O/p2.log" 2>&1
rc=$?; tail -2 "$O/p2.log"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py "$O/p2" "trace_kernel<false" | head -20
echo "== done"
