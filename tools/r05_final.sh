# round-5 final tree: full GPU suite, smoke, default bench line
set -o pipefail
P=${1:-r05ap}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${P}_tests.log
[ $rc -gt 1 ] && exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || exit 1
exit $rc
