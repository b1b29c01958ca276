#!/bin/bash
# Sweep of the round-4 loss-parity guard thresholds (tools/guard_sweep.py),
# each setting in its own process (the thresholds are read once per process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/guard_sweep.jsonl
for cfg in "7 4 10" "8 5 10" "9 6 12" "8 4 10" "7 6 10" "10 6 14" "9 5 11"; do
  set -- $cfg
  SRHIP_JIT_CAN_LOG2=$1 SRHIP_JIT_EXP_GUARD_LOG2=$2 SRHIP_JIT_TRIG_GUARD_LOG2=$3 \
    timeout -k 10 200 python3 -u tools/guard_sweep.py "kc$1_te$2_tt$3" >> gpurun_out/guard_sweep.jsonl 2>> gpurun_out/guard_sweep.err || exit 1
  tail -1 gpurun_out/guard_sweep.jsonl
done
SRHIP_JIT_LOSS_GUARDS=0 timeout -k 10 200 python3 -u tools/guard_sweep.py "r3" >> gpurun_out/guard_sweep.jsonl 2>> gpurun_out/guard_sweep.err || exit 1
tail -1 gpurun_out/guard_sweep.jsonl
