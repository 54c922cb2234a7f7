#!/bin/bash
# Head groups (pt_set_head_groups): parity tests, then the first K tiles of the cost order in G groups
# beside a plain launch of the rest, against the shipped schedule: C4 N = 8 share, C3 N = 2 share, C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03h2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssg.py tests/test_gpu_parity.py -k "head_groups or schedule_knobs" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift
  timeout -k 10 300 python tools/sched_probe.py --spans "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 4; }
  python - "$O/$name.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["image"], "n", d["n"], "spp", d["spp"], "min", d["ms_min"], "all", d["ms_all"])
print("   tiles max/top1%/mean", d["tile_ms_max_top1pct_mean"])
PY
}
run c4n8 --n 8 --width 3840 --height 2160 --spp 4096 --scheds a,h16g2,h64g2,h160g2,h64g4 --rounds 2
run c3n2 --n 2 --scheds a,h16g2,h64g2,h256g2,h64g4 --rounds 3
run c3 --scheds a,h16g2,h64g2 --rounds 3
echo "== done"
