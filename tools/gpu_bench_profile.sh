#!/bin/bash
# Profiles of the bench command itself (config #2): kernel trace + stats of a
# warm 20-step run, then one run per PMC pass; summary for profiles/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/benchprof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 bench.py --steps 20 --warmup 10 --no-cpu --no-row-shard > $OUT/bench_kt.json 2> $OUT/log.txt || exit $?
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_BRANCH"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES"
P3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32"
P4="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE"
P5="FETCH_SIZE"
P6="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o pmc$i -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-row-shard > $OUT/bench_pmc$i.json 2>> $OUT/log.txt || exit $?
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
