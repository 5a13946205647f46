#!/bin/bash
# Build libkh_gpu.so variants for on-GPU A/B timing: tools/build_variants.sh "LB LBH H" ...
# (every translation unit is compiled with the variant's flags; EXTRA adds more -D flags)
set -e
cd "$(dirname "$0")/../keyhunt_amd"
VARS=("$@")
for v in "${VARS[@]}"; do
  read -r lb lbh h <<< "$v"
  d=../variants/lb${lb}_h${lbh}_w${h}
  mkdir -p $d
  F="-O3 -std=c++17 -fPIC -I../include -Icsrc -DKH_WALK_LB=$lb -DKH_WALK_LB_HASH=$lbh -DKH_WALK_H=$h $EXTRA"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c csrc/kh_kernels.hip -o $d/k.o &
  /opt/rocm/bin/hipcc --offload-host-only $F -c csrc/kh_capi.cpp -o $d/c.o &
done
wait
for v in "${VARS[@]}"; do
  read -r lb lbh h <<< "$v"
  d=../variants/lb${lb}_h${lbh}_w${h}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libkh_gpu.so $d/k.o $d/c.o -Wl,-rpath,/opt/rocm/lib
  rm -f $d/k.o $d/c.o
done
