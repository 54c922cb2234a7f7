#!/bin/bash
# Same-box A/B of the working tree against an older snapshot in $OLD (default _ab_old/, a copy of
# pathtracercuda_amd/ include/ Makefile tools/ scenes/ oracle/ from an earlier commit; git-ignored).
# Box-to-box variance is a few percent, so only same-run comparisons are meaningful.
#   OLD=_ab_old VARIANTS=28 bash tools/ab_compare.sh
set -u
OLD="${OLD:-_ab_old}"
V="${VARIANTS:-0}"
make -s -j16 >/dev/null 2>&1 || exit 3
(cd "$OLD" && make -s -j16 pathtracercuda_amd/lib/libpt_hip.so pathtracercuda_amd/lib/libpt_host.so >/dev/null 2>&1) || exit 4
for i in 1 2; do
  for side in new old; do
    dir=.; [ $side = old ] && dir="$OLD"
    (cd "$dir" && timeout -k 10 200 python tools/ab_variants.py --variants $V --rounds 5 > "$OLDPWD/gpurun_out/cmp_${side}_$i.log" 2>&1) || exit 5
    (cd "$dir" && timeout -k 10 200 python tools/ab_variants.py --variants $V --rounds 5 --scene scenes/cornell_box.scene.json \
        --width 512 --height 512 > "$OLDPWD/gpurun_out/cmpc_${side}_$i.log" 2>&1) || exit 6
  done
done
grep -o '"Msamples_s": [0-9.]*' gpurun_out/cmp_*.log gpurun_out/cmpc_*.log
