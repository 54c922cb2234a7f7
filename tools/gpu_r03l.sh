#!/bin/bash
# Issue-priority policies on the refined cost order: off, first 4096 positions, first 12/25/50 %,
# graded by quarter; C3 at N = 1, 2, 4 (sample groups automatic), the C4 N = 8 share, C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "schedule_knobs" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo FATAL pytest; tail -5 $O/pytest.log; exit 5; }
S="a,p4096,f12,f25,f50,q"
run() { name=$1; shift; timeout -k 10 400 python tools/sched_probe.py "$@" > $O/$name.json 2> $O/$name.err || { echo FATAL $name; tail -3 $O/$name.err; exit 5; }; python - $O/$name.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["image"], "n", d["n"], "spp", d["spp"], "groups", d["groups"], {k: (v, sorted(d["ms_all"][k])[len(d["ms_all"][k])//2]) for k, v in d["ms_min"].items()})
PY
}
run c3_n1 --scheds $S --rounds 4
run c3_n2 --n 2 --scheds $S --rounds 4
run c3_n4 --n 4 --groups 0 --scheds $S --rounds 4
run c3_n8 --n 8 --groups 0 --scheds $S --rounds 4
run c4_n8 --width 3840 --height 2160 --spp 4096 --n 8 --scheds a,p4096,f25,f50,q --rounds 2
run c2 --scene scenes/cornell_box.scene.json --width 512 --height 512 --spp 64 --scheds $S --rounds 4
echo "== done"
