#!/bin/bash
# Persistent encoder with one pixel group per wave and 8 waves (two per SIMD,
# MSFNO_MG_PG=1) against two groups and 4 waves (default): tests under both, PMC of the
# PG=1 kernel, interleaved A/B of the net line.
set -o pipefail
O=${1:-gpurun_out/r06_q}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p $O
for pg in 1 2; do
  MSFNO_MG_PG=$pg timeout -k 10 300 python -u -m pytest -v -s --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_mlp_gen.py > $O/mlp_gen_tests_pg$pg.log 2>&1 || exit $?
done
MSFNO_MG_PG=1 timeout -s KILL 120 rocprofv3 --kernel-include-regex mlp_gen_hp --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
  SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
  SQ_INSTS_VALU --kernel-trace -d $O/pmc_raw -o p -f csv -- python3 bench.py --workload net --steps 2 \
  --warmup 1 --cpu-baseline 0 > $O/pmc.json 2>&1 || exit $?
mkdir -p $O/pm/a && find $O/pmc_raw -name "*.csv" -exec mv {} $O/pm/a/ \; && \
python tools/pmc_summary.py $O/pm mlp_gen_hp > $O/pmc_mlp_gen_hp_pg1.txt 2>&1; rm -rf $O/pmc_raw $O/pm
net() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload net --steps 30 --cpu-baseline 0 \
    > $O/n_$tag.json 2> $O/n_$tag.err || exit $?
  python - $O/n_$tag.json $tag <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
print("net", sys.argv[2], b["value"], r.get("ms_per_step"), r.get("all_stages_ms", {}).get("mlp_gen"))
PY
}
for i in 1 2 3; do
  net pg2_$i MSFNO_MG_PG=2
  net pg1_$i MSFNO_MG_PG=1
done > $O/summary.txt
grep -h "differ\|passed\|failed" $O/mlp_gen_tests_pg*.log | tail -8
cat $O/pmc_mlp_gen_hp_pg1.txt $O/summary.txt
