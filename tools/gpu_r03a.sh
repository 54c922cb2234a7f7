#!/bin/bash
# Round 3: GPU suite, path-level pin record, bench plain vs in-process group at N = 1.
set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python tools/pin_png.py --corr > $O/pin.json || exit 1
cat $O/pin.json
for i in 1 2; do
  timeout -k 10 200 python bench.py --secondary 0 --cpu-baseline 0 --steps 5 > $O/bench_single_$i.json || exit 1
  timeout -k 10 200 python bench.py --secondary 0 --cpu-baseline 0 --steps 5 --group 1 > $O/bench_group_$i.json || exit 1
done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d.get('group_timing'))"; done
