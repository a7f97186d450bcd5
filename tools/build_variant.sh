#!/bin/bash
# Build a side library from an alternative kernel source (A/B experiments; load it with
# KGPU_LIB_PATH): tools/build_variant.sh <kernels.hip> <out.so>.  The host object is the in-tree one.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; OUT=$2
API=$(ls -t $R/build/obj/kgpu_api.cpp.*.o | head -1)
TMPO=$(mktemp /tmp/kvar.XXXXXX.o)
cp "$SRC" $R/kubernetes-1_amd/csrc/.variant_$$.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
  -Wall -Wno-unused-result -I$R/include -c $R/kubernetes-1_amd/csrc/.variant_$$.hip -o $TMPO
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT.tmp" $TMPO $API -ldl
mv "$OUT.tmp" "$OUT"
rm -f $TMPO $R/kubernetes-1_amd/csrc/.variant_$$.hip
