#!/bin/bash
# Tail groups (pt_set_head_groups mode 3): parity, then C3 1080p and its N = 2 share.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03t2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssg.py -k "head_groups" -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -7 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift
  timeout -k 10 300 python tools/sched_probe.py "$@" > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 4; }
  python - "$O/$name.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["image"], "n", d["n"], "spp", d["spp"], "min", d["ms_min"], "all", d["ms_all"])
PY
}
run c3 --scheds a,t1024g2,t2048g2,t4096g2,t2048g4 --rounds 4
run c3n2 --n 2 --scheds a,t1024g2,t2048g2 --rounds 3
echo "== done"
