set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_i
mkdir -p $O
K="--kernel-include-regex skip_h"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- python3 tools/skip_time.py > $O/skip_kt.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 $K --pmc FETCH_SIZE --kernel-trace -f csv -d $O/fetch -o fetch -- python3 tools/skip_time.py > $O/skip_f.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 $K --pmc WRITE_SIZE --kernel-trace -f csv -d $O/write -o write -- python3 tools/skip_time.py > $O/skip_w.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -f csv -d $O/p1 -o p1 -- python3 tools/skip_time.py > $O/p1.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 $K --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-trace -f csv -d $O/p2 -o p2 -- python3 tools/skip_time.py > $O/p2.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 $K --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr --kernel-trace -f csv -d $O/p3 -o p3 -- python3 tools/skip_time.py > $O/p3.txt 2>&1 || exit $?
exit 0
