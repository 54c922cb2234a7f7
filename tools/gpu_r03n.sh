#!/bin/bash
# Graded-priority bounds on the strong-scaling shares (C4 N = 8, C3 N = 2) and C3 N = 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03n; mkdir -p $O
S="q,g10_30_60,g5_15_40,g20_40_60,g33_66_100,g15_35_55"
run() { name=$1; shift; timeout -k 10 400 python tools/sched_probe.py "$@" > $O/$name.json 2> $O/$name.err || { echo FATAL $name; tail -3 $O/$name.err; exit 5; }; python - $O/$name.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["image"], "n", d["n"], "spp", d["spp"], {k: (v, sorted(d["ms_all"][k])[len(d["ms_all"][k])//2]) for k, v in d["ms_min"].items()})
PY
}
run c4_n8 --width 3840 --height 2160 --spp 4096 --n 8 --scheds $S --rounds 2
run c3_n2 --n 2 --scheds $S --rounds 3
run c3_n1 --scheds $S --rounds 3
echo "== done"
