#!/bin/bash
# debug: test120 BSGS window with both layer-1 layouts
set -o pipefail
R=$PWD
mkdir -p gpurun_out/t120 && cd gpurun_out/t120 && cp $R/tests/golden/data/test120.txt .
for L in blocked reference; do
  timeout -k 10 200 $R/keyhunt_amd/bin/keyhunt-amd -m bsgs -f test120.txt -b 120 -q -s 0 -L $L > out_$L.log 2>&1
  echo "L=$L rc=$?" >> rc.txt
  [ -f KEYFOUNDKEYFOUND.txt ] && mv KEYFOUNDKEYFOUND.txt kf_$L.txt
done
cat rc.txt
