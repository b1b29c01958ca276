#!/bin/bash
# PMC passes over one microbench config: tools/pmc_micro.sh "<config>" [tag]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CFG=${1:-"+-*"}; TAG=${2:-m}
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
pass() { name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- python3 tools/microbench.py 1000000 "$CFG" >> $OUT/log.txt 2>&1 || { echo "pass $name failed"; exit 1; }
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS
pass p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_IFETCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC
pass p3 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_MISSES GRBM_GUI_ACTIVE
pass p4 SQ_WAVES SQ_LEVEL_WAVES SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32
echo done
