# full GPU suite, smoke, then the default bench line (stages on stderr)
set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/full_t.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/full_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --stages > gpurun_out/full_bench.json 2> gpurun_out/full_bench.err
