#!/bin/bash
# The encoder tests with the added edge cases (a single partial tile per field, Cout < 256).
set -o pipefail
O=${1:-gpurun_out/r06_ad}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_mlp_gen.py > $O/tests.log 2>&1; rc=$?
grep -h "differ\|rel\|passed\|failed\|Error" $O/tests.log | tail -20; exit $rc
