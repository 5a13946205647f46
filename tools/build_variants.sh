#!/bin/bash
# Build libkh_gpu.so variants for on-GPU A/B timing:
#   tools/build_variants.sh "LB LBH H [NAME [-DFLAG ...]]" ...
# Every translation unit is compiled with the variant's flags; the library lands in
# variants/NAME (default lb<LB>_h<LBH>_w<H>).  Run with KH_LIB=variants/NAME/libkh_gpu.so.
set -e
cd "$(dirname "$0")/../keyhunt_amd"
VARS=("$@")
name_of() { read -r lb lbh h name rest <<< "$1"; echo "${name:-lb${lb}_h${lbh}_w${h}}"; }
for v in "${VARS[@]}"; do
  read -r lb lbh h name rest <<< "$v"
  d=../variants/$(name_of "$v")
  mkdir -p $d
  F="-O3 -std=c++17 -fPIC -I../include -Icsrc -DKH_WALK_LB=$lb -DKH_WALK_LB_HASH=$lbh -DKH_WALK_H=$h $rest"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c csrc/kh_kernels.hip -o $d/k.o &
  /opt/rocm/bin/hipcc --offload-host-only $F -c csrc/kh_capi.cpp -o $d/c.o &
done
wait
for v in "${VARS[@]}"; do
  d=../variants/$(name_of "$v")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libkh_gpu.so $d/k.o $d/c.o -Wl,-rpath,/opt/rocm/lib
  rm -f $d/k.o $d/c.o
done
