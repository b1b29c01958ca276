#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC
# counter passes (each its own run, within the per-block slot limits).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r01}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu"}
echo "== kernel trace" | tee -a $OUT/log.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py $ARGS >> $OUT/log.txt 2>&1 || exit $?
echo "== pmc1" | tee -a $OUT/log.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $OUT/pmc1 -o pmc1 -- python3 bench.py $ARGS >> $OUT/log.txt 2>&1 || exit $?
echo "== pmc2" | tee -a $OUT/log.txt
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o pmc2 -- python3 bench.py $ARGS >> $OUT/log.txt 2>&1 || exit $?
echo "== pmc3" | tee -a $OUT/log.txt
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/pmc3 -o pmc3 -- python3 bench.py $ARGS >> $OUT/log.txt 2>&1 || exit $?
echo "== done" | tee -a $OUT/log.txt
find $OUT -name "*.csv" | head -20
