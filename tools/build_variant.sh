#!/bin/bash
# Build a side library from an alternative kernel source (A/B experiments; load it with
# KGPU_LIB_PATH): tools/build_variant.sh <kernels.hip> <out.so>.  The host objects (kgpu_api.cpp,
# kgpu_compile.cpp) are the in-tree ones.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; OUT=$2
# the host object compiled from the CURRENT tree (an object of another revision would disagree with
# the variant about the launch-argument layouts)
API=$(mktemp /tmp/kapi.XXXXXX.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-result \
  -I$R/include -c $R/kubernetes-1_amd/csrc/kgpu_api.cpp -o $API
CMP=$(mktemp /tmp/kcmp.XXXXXX.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-result \
  -I$R/include -c $R/kubernetes-1_amd/csrc/kgpu_compile.cpp -o $CMP
TMPO=$(mktemp /tmp/kvar.XXXXXX.o)
cp "$SRC" $R/kubernetes-1_amd/csrc/.variant_$$.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -mllvm -amdgpu-kernarg-preload-count=16 \
  -Wall -Wno-unused-result -I$R/include -c $R/kubernetes-1_amd/csrc/.variant_$$.hip -o $TMPO
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT.tmp" $TMPO $API $CMP -ldl
mv "$OUT.tmp" "$OUT"
rm -f $TMPO $API $CMP $R/kubernetes-1_amd/csrc/.variant_$$.hip
