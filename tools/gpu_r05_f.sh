set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_f
mkdir -p $O
for v in 0 1; do
  MSFNO_SKIP_P=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt$v -o kt -- python3 tools/skip_time.py > $O/skip_kt$v.txt 2>&1 || exit $?
done
MSFNO_SKIP_P=1 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $O/fetch -o fetch -- python3 tools/skip_time.py > $O/skip_f.txt 2>&1 || exit $?
MSFNO_SKIP_P=1 timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $O/write -o write -- python3 tools/skip_time.py > $O/skip_w.txt 2>&1 || exit $?
MSFNO_SKIP_P=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -f csv -d $O/sq -o sq -- python3 tools/skip_time.py > $O/skip_sq.txt 2>&1 || exit $?
exit 0
