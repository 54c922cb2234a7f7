#!/bin/bash
# Build libpt_hip.so of an earlier commit into _snap/<name>/ (a minimal tree tools/ab_variants.py
# runs from) for same-box A/Bs against the working tree (tools/gpu_ab_snap.sh).  Host library and
# Python package come from the working tree (the C ABI is unchanged between the two).
#   [SED='<sed expression on pt_kernels.hip>'] tools/snap_rev.sh <name> <git-rev> ["<extra hipcc flags>"]
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=$2; flags=${3:-}
d=_snap/$name; src=$(mktemp -d)
rm -rf "$d"; mkdir -p "$d/pathtracercuda_amd/lib" "$d/tools"
git archive "$rev" pathtracercuda_amd/csrc include | tar -x -C "$src"
# optional source edit for parameter A/Bs, e.g. SED='s/kV40Walk = 13216/kV40Walk = 14216/'
if [ -n "${SED:-}" ]; then sed -i "$SED" "$src/pathtracercuda_amd/csrc/pt_kernels.hip"; fi
# the Python package of the same revision (it binds exactly that revision's C ABI)
git archive "$rev" pathtracercuda_amd/__init__.py pathtracercuda_amd/_native.py pathtracercuda_amd/distributed.py | tar -x -C "$d"
cp pathtracercuda_amd/lib/libpt_host.so "$d/pathtracercuda_amd/lib/"
cp tools/ab_variants.py tools/one_launch.py "$d/tools/"
cp -r scenes "$d/"
base=$(make -s print-HIPFLAGS | sed 's/-Iinclude//')
/opt/rocm/bin/hipcc $base -I"$src/include" $flags -shared \
  -o "$d/pathtracercuda_amd/lib/libpt_hip.so" "$src/pathtracercuda_amd/csrc/pt_kernels.hip" -lrccl
rm -rf "$src"
echo "built $d from $rev ($flags)"
