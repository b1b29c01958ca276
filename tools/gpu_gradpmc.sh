#!/bin/bash
# Gradient kernel (config #5 shard, tools/prof_grad.py): per-pass times, a
# kernel trace and two PMC passes, summarised by tools/pmc_summary.py.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/gradprof; mkdir -p $OUT
SRHIP_DEBUG_PASSES=1 timeout -k 10 200 python3 tools/prof_grad.py 2 2>&1 | tail -4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 tools/prof_grad.py 3 > $OUT/out.json 2> $OUT/log.txt || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc1 -o pmc1 -- python3 tools/prof_grad.py 1 >> $OUT/log.txt 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SMEM --output-format csv -d $OUT/pmc2 -o pmc2 -- python3 tools/prof_grad.py 1 >> $OUT/log.txt 2>&1 || exit $?
KERNEL=sr_jit_grad WORKLOAD="config#5 shard dL/dc" python3 tools/pmc_summary.py $OUT
