#!/bin/bash
# Build a copy of libpt_hip.so with extra compiler flags into _snap/<name>/ (a minimal tree that
# tools/ab_variants.py can run from), for same-box A/B of compiler options: tools/gpu_ab_dirs.sh.
#   tools/build_snap.sh <name> "<extra hipcc flags>"
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=${2:-}
d=_snap/$name
rm -rf "$d"; mkdir -p "$d/pathtracercuda_amd/lib" "$d/tools"
cp pathtracercuda_amd/*.py "$d/pathtracercuda_amd/"
cp pathtracercuda_amd/lib/libpt_host.so "$d/pathtracercuda_amd/lib/"
cp tools/ab_variants.py "$d/tools/"
cp -r scenes "$d/"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -fvisibility=hidden \
  -mcode-object-version=5 -Iinclude -Wall -Wno-unused-result $flags -shared \
  -o "$d/pathtracercuda_amd/lib/libpt_hip.so" pathtracercuda_amd/csrc/pt_kernels.hip -lrccl
echo "built $d ($flags)"
