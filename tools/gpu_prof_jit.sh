#!/bin/bash
# rocprofv3 passes over tools/prof_target.py (MODE=jit|interp|jit-precise)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-jit}
mkdir -p $OUT
export MODE=${MODE:-jit}
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 tools/prof_target.py 10 > $OUT/log.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/pmc1 -o pmc1 -- python3 tools/prof_target.py 3 >> $OUT/log.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o pmc2 -- python3 tools/prof_target.py 3 >> $OUT/log.txt 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_SALU --output-format csv -d $OUT/pmc3 -o pmc3 -- python3 tools/prof_target.py 3 >> $OUT/log.txt 2>&1 || exit $?
find $OUT -name "*.csv" | head -20
