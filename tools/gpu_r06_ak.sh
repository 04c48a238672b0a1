#!/bin/bash
# Switches no test exercised before: the variants test (block goldens) and the encoder /
# decoder kernel variants (bitwise against the default).
set -o pipefail
O=${1:-gpurun_out/r06_ak}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_mlp_gen.py tests/test_gpu_variants.py > $O/tests.log 2>&1; rc=$?
grep -h "differ\|PASSED\|FAILED\|passed\|failed\|Error" $O/tests.log | tail -80; exit $rc
