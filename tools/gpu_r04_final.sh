set -o pipefail
cd /root/repo
O=gpurun_out/r04_final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
echo "suite rc $?" | tee -a $O/gpu_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/profile_round.sh $O > $O/profile_round.log 2>&1 || exit $?
exit 0
