#!/bin/bash
# Config #5 shard gradient time (tools/prof_grad.py) under the guard variants,
# one process each, same box: round-3 guards, round-4 defaults, the gradient's
# tight trig threshold, and the PRECISE forward.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/grad_ab.txt
for v in "SRHIP_JIT_LOSS_GUARDS=0" "SRHIP_X=0" "SRHIP_GJIT_TRIG_GUARD_LOG2=6" "SRHIP_GJIT_FAST=0" "SRHIP_JIT_LOSS_GUARDS=0" "SRHIP_GJIT_TRIG_GUARD_LOG2=6"; do
  echo -n "$v " >> gpurun_out/grad_ab.txt
  env $v timeout -k 10 200 python3 tools/prof_grad.py 3 2>&1 | tail -1 | grep -o '"kernel_ms": [0-9.]*' >> gpurun_out/grad_ab.txt || exit 1
done
cat gpurun_out/grad_ab.txt
