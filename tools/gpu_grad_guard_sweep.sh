#!/bin/bash
# Gradient-code guard thresholds (SRHIP_GJIT_*_LOG2): tight Float32-oracle
# gradient parity (tools/debug_grad32.py, both opsets) and the config #5 shard
# gradient time (tools/prof_grad.py) per setting, each in its own process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/ggs.jsonl
for cfg in "7 4 10" "7 4 6" "8 3 6" "9 3 5" "7 3 7"; do
  set -- $cfg
  export SRHIP_GJIT_CAN_LOG2=$1 SRHIP_GJIT_EXP_GUARD_LOG2=$2 SRHIP_GJIT_TRIG_GUARD_LOG2=$3
  echo "{\"setting\": \"kc$1_te$2_tt$3\"}" >> gpurun_out/ggs.jsonl
  timeout -k 10 200 python3 tools/debug_grad32.py cfg5 2>&1 | cut -c 1-400 >> gpurun_out/ggs.jsonl || exit 1
  timeout -k 10 200 python3 tools/debug_grad32.py wide w 2>&1 | cut -c 1-400 >> gpurun_out/ggs.jsonl || exit 1
  timeout -k 10 200 python3 tools/prof_grad.py 3 2>&1 | tail -1 | cut -c 1-300 >> gpurun_out/ggs.jsonl || exit 1
done
cat gpurun_out/ggs.jsonl
