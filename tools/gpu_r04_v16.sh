# One run: (1) the unpadded encoder / decoder stream, built as
# msfno_amd/libmsfno_nopad.so, and the encoder's addend kept in flight under the last
# unit with exact waits, libmsfno_addw.so (MSFNO_LIB A/B) — parity, then interleaved
# network benches;
# (2) this round's new A/B switches (graph-captured skip fork, late linear skip fork) —
# variant parity and interleaved benches.  Build the two variant libraries first, on the
# CPU: bash tools/build_ab_variants.sh
set -o pipefail
cd /root/repo
O=gpurun_out/r04_v16
mkdir -p $O
NOPAD=$PWD/modulated-spherical-fourier-neural-operator_amd/msfno_amd/libmsfno_nopad.so
ADDW=$PWD/modulated-spherical-fourier-neural-operator_amd/msfno_amd/libmsfno_addw.so
T="python -u -m pytest -q --timeout-method thread -m gpu"
MSFNO_LIB=$NOPAD timeout -k 10 400 $T -x --timeout 200 tests/test_gpu_mlp_gen.py tests/test_gpu_configs.py -k "mlp or deferred or config3" > $O/tests_nopad.log 2>&1
echo "nopad tests rc $?" | tee -a $O/summary.txt
MSFNO_LIB=$ADDW timeout -k 10 300 $T -x --timeout 200 tests/test_gpu_mlp_gen.py > $O/tests_addw.log 2>&1
echo "addw tests rc $?" | tee -a $O/summary.txt
timeout -k 10 400 $T -x --timeout 200 tests/test_gpu_variants.py -k "BM64 or LIN_SKIP" > $O/tests_variants.log 2>&1 || exit $?
ab() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 240 python bench.py --cpu-baseline 0 --linear-check 0 $EXTRA > $O/$tag.json 2> $O/$tag.err || return $?
  python3 -c "import json;print('$tag', json.loads(open('$O/$tag.json').readline())['value'])" | tee -a $O/summary.txt
}
for i in 1 2; do
  EXTRA="--workload net" ab net_base_$i MSFNO_NONE=1 || exit $?
  EXTRA="--workload net" ab net_nopad_$i MSFNO_LIB=$NOPAD || exit $?
  EXTRA="--workload net" ab net_addw_$i MSFNO_LIB=$ADDW || exit $?
  EXTRA="--workload net" ab net_gfork_$i MSFNO_GRAPH_FORK=1 || exit $?
  EXTRA="--filter linear" ab lin_base_$i MSFNO_NONE=1 || exit $?
  EXTRA="--filter linear" ab lin_late_$i MSFNO_LIN_SKIP_AT=inv || exit $?
done
exit 0
