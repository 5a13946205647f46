# Host-side AddressSanitizer/UBSan run of the CLI (bin/keyhunt-amd-asan, host code only; the GPU
# code is not instrumented) over small known-answer windows; prints any sanitizer report.
set -o pipefail
O=$(pwd)/gpurun_out/${1:-asan}; mkdir -p $O
B=$(pwd)/keyhunt_amd/bin/keyhunt-amd-asan
T=$(mktemp -d); cp tests/golden/data/* $T; cd $T
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
run() { timeout -k 10 120 $B "$@" -q -s 0 > out.txt 2>&1; rc=$?; n=$(grep -c "AddressSanitizer\|runtime error" out.txt); echo "rc=$rc sanitizer_reports=$n :: $*"; [ $n -eq 0 ] || { cat out.txt; return 1; }; }
run -m address -f 1to32.txt -r 1:FFFFF -n 0x100000 && \
run -m rmd160 -f 1to32.rmd -l compress -r 1:FFFFF -n 0x100000 -e && \
run -m xpoint -f 1to63_65.txt -r 1:FFFFF -n 0x100000 -S && \
run -m vanity -v 1Kha -v 1PUB -r 1:FFFFF -n 0x100000 && \
run -m bsgs -f 63.pub -n 0x1000000 -k 4 -r 7cce5efdac000000:7cce5efdad000000 -S && \
run -m bsgs -f 63.pub -n 0x1000000 -k 4 -r 7cce5efdac000000:7cce5efdad000000 -S -B both && \
run -m bsgs -f 63.pub -n 0x1000000 -k 4 -B ggsb --bsgs-block-count 4 -r 7cce5efdac000000:7cce5efdad000000
rc=$?; cp out.txt $O/last_out.txt; exit $rc
