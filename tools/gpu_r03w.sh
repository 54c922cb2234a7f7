#!/bin/bash
# 1080p N = 8 shares under sample groups: per-launch times, group stats and kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/ssg_ranks.py --n 8 --launches 5 > $O/ranks.log 2> $O/ranks.err || { tail -5 $O/ranks.err; exit 3; }
tail -1 $O/ranks.log | cut -c1-2000
find $O/kt -name "*.csv" -size +1M -exec gzip {} \;
echo "== done"
