#!/bin/bash
# New / changed GPU tests first, the round profile (block, linear, net; summarised on
# the box, raw databases dropped), then the suite.
set -o pipefail
O=${1:-gpurun_out/r06_b}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_film_backward.py tests/test_gpu_large_golden.py tests/test_gpu_rccl.py \
  "tests/test_gpu_parity.py::test_global_conv_skip_engines" > $O/new_tests.log 2>&1 || exit $?
bash tools/profile_round.sh $O/prof > $O/profile.log 2>&1 || exit $?
python tools/rocpd_summary.py $O/prof $O/summary > $O/summary.txt 2>&1 || exit $?
cp $O/prof/*.json $O/prof/*.txt $O/summary/ 2>/dev/null
rm -rf $O/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/gpu_suite.log 2>&1; rc=$?; echo "suite rc $rc" >> $O/gpu_suite.log; exit $rc
