#!/bin/bash
# Round 3: parity suite; group vs single in one process (with / without torch first); WRITE_SIZE and
# instruction counts of one C3 launch; bench (lane utilisation incl. leaf family counters);
# occupancy probe (tile times at fewer waves per SIMD).  Each GPU step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"; O="$R/gpurun_out/r03d"; mkdir -p "$O"; export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL: $2 exited $1"; exit "$1"; fi; }
echo "== pytest"; timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; tail -2 "$O/pytest.log"; fatal $rc pytest
for t in 0 1; do
  echo "== group vs single torch=$t"; timeout -k 10 200 python tools/group_vs_single.py --torch $t > "$O/gvs_$t.json" 2> "$O/gvs_$t.err"
  rc=$?; cat "$O/gvs_$t.json"; fatal $rc "gvs $t"
done
for grp in WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
  t=${grp%% *}
  echo "== pmc $t"
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-trace -d "$O/pmc_$t" -o run --output-format csv -- python3 $R/tools/one_launch.py --spp 1024) > "$O/pmc_$t.log" 2>&1
  rc=$?; tail -1 "$O/pmc_$t.log"; fatal $rc "pmc $t"
done
echo "== bench"; timeout -k 10 300 python bench.py --secondary 0 --cpu-baseline 0 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['lane_utilisation'])"; fatal $rc bench
echo "== occupancy probe"; timeout -k 10 300 python tools/occupancy_probe.py > "$O/occ.log" 2>&1
rc=$?; tail -1 "$O/occ.log"; fatal $rc occ
echo "== occupancy probe C4 share n=8"; timeout -k 10 300 python tools/occupancy_probe.py --width 3840 --height 2160 --n 8 --spp 512 --occ 5,2,1 > "$O/occ_c4.log" 2>&1
rc=$?; tail -1 "$O/occ_c4.log"; fatal $rc occc4
echo "== done"
