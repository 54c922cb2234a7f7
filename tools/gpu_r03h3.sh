#!/bin/bash
# Head groups under a kernel trace: C4 N = 8 share, first 64 tiles in 2 groups; the plain launch beside it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03h3; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/head_probe.py --n 8 --width 3840 --height 2160 --spp 4096 --head 64 --groups 2 --launches 2 > $O/c4n8.log 2> $O/c4n8.err || { tail -5 $O/c4n8.err; exit 3; }
tail -1 $O/c4n8.log
timeout -k 10 200 python3 tools/head_probe.py --n 2 --head 32 --groups 2 --launches 3 > $O/c3n2.log 2>&1 || { tail -5 $O/c3n2.log; exit 4; }
tail -1 $O/c3n2.log
find $O/kt -name "*.csv" -size +1M -exec gzip {} \;
echo "== done"
