# Re-check the defaults against their A/B switches on this round's build (config 2,
# interleaved with the default; 2 runs each)
set -o pipefail
cd /root/repo
O=gpurun_out/r04_sweep
mkdir -p $O
B="python bench.py --linear-check 0 --cpu-baseline 0 --steps 30"
run() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 $B > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json;print('$tag', json.loads(open('$O/$tag.json').readline())['value'])" | tee -a $O/summary.txt
}
for i in 1 2; do
  run base_$i MSFNO_NONE=1 || exit $?
  run x3fns2_$i MSFNO_X3F_NS=2 || exit $?
  run x3cns2_$i MSFNO_X3C_NS=2 || exit $?
  run r2c8x3_$i MSFNO_R2C_CFG=8x3 || exit $?
  run c2rwv4_$i MSFNO_C2R_WV=4 MSFNO_C2R_AREG=0 || exit $?
  run prio_normal_$i MSFNO_SIDE_PRIO=normal || exit $?
  run skipx3_$i MSFNO_SKIP_H=0 || exit $?
  run side0_$i MSFNO_SIDE_STREAM=0 || exit $?
done
# the linear filter: skip forked after the contraction (A/B)
for i in 1 2; do
  for v in "MSFNO_NONE=1" "MSFNO_LIN_SKIP_AT=inv"; do
    tag=lin_${v%%=*}_$i
    env $v timeout -k 10 240 python bench.py --filter linear --linear-check 0 --cpu-baseline 0 > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "import json;print('$tag', json.loads(open('$O/$tag.json').readline())['value'])" | tee -a $O/summary.txt
  done
done
# the network step: the side-stream fork captured into the graph (A/B)
for i in 1 2; do
  for v in "MSFNO_NONE=1" "MSFNO_GRAPH_FORK=1"; do
    tag=net_${v%%=*}_$i
    env $v timeout -k 10 240 python bench.py --workload net --cpu-baseline 0 > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "import json;print('$tag', json.loads(open('$O/$tag.json').readline())['value'])" | tee -a $O/summary.txt
  done
done
exit 0
