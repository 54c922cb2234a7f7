#!/bin/bash
# PMC A/B of trace-kernel variants on one launch of a workload (tools/one_launch.py), one rocprofv3
# --pmc pass per counter group and variant.  Usage on the GPU box, from the repository root:
#   OUT=<dir under gpurun_out> VARIANTS="40 60" tools/pmc_variants.sh
# Summaries: python tools/pmc_summary.py gpurun_out/<dir>/v<variant> trace_kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/${OUT:-pmcab}"; mkdir -p "$O"; export TMPDIR=/tmp
for v in ${VARIANTS:-40 60}; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT"; do
    i=$((i+1))
    echo "== v$v pass $i: $grp"
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d "$O/v$v/p$i" -o run --output-format csv -- \
        python3 "$R/tools/one_launch.py" --variant $v --reps 2 ${ARGS:-}) > "$O/v${v}_p$i.log" 2>&1
    rc=$?; tail -1 "$O/v${v}_p$i.log"
    if [ $rc -ne 0 ]; then echo "FATAL: v$v pass $i exited $rc"; exit $rc; fi
  done
done
echo "== done"
