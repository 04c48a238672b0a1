#!/bin/bash
# HEAD refresh with the round-6 defaults: smoke, the round profile (block, linear, net;
# summarised on the box, raw databases dropped), then the full -m gpu suite.
set -o pipefail
O=${1:-gpurun_out/r06_end6}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
bash tools/profile_round.sh $O/prof > $O/profile.log 2>&1 || exit $?
python tools/rocpd_summary.py $O/prof $O/summary > $O/summary.txt 2>&1 || exit $?
cp $O/prof/*.json $O/prof/*.txt $O/summary/ 2>/dev/null
rm -rf $O/prof
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/gpu_suite.log 2>&1; rc=$?; echo "suite rc $rc" >> $O/gpu_suite.log; exit $rc
