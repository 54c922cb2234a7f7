#!/bin/bash
# PC sampling of the default C3 kernel: the line-table build of HEAD in _snap/pcs (tools/snap_rev.sh
# pcs HEAD -gline-tables-only; its gfx950 ISA is identical to the plain build's), host-trap first,
# then stochastic; the sample CSVs are gzipped for tools/pc_hotspots.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
echo "== host_trap"
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 20 -d $O/ht -o run --output-format csv -- \
  python3 _snap/pcs/tools/one_launch.py --spp 256 --reps 2 > $O/ht.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 $O/ht.log; find $O/ht -type f -exec ls -la {} \;
[ $rc -eq 0 ] || exit 3
find $O/ht -name "*.csv" -size +1M -exec gzip {} \;
echo "== stochastic"
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 1048576 -d $O/st -o run --output-format csv -- \
  python3 _snap/pcs/tools/one_launch.py --spp 256 --reps 2 > $O/st.log 2>&1
rc=$?
echo "rc=$rc"; tail -5 $O/st.log; find $O/st -type f -exec ls -la {} \;
find $O/st -name "*.csv" -size +1M -exec gzip {} \;
echo "== done"
