#!/bin/bash
# The round-6 switches in the variants test and both sides of the buffer-addressing test.
set -o pipefail
O=${1:-gpurun_out/r06_aj}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 800 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_buf_addressing.py tests/test_gpu_variants.py > $O/tests.log 2>&1; rc=$?
grep -h "differ\|PASSED\|FAILED\|passed\|failed\|Error" $O/tests.log | tail -60; exit $rc
