#!/bin/bash
# round 3: threaded staged output copy (config #3 per-row outputs)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pytest_3h.log 2>&1 || { tail -30 gpurun_out/pytest_3h.log; exit 1; }
tail -2 gpurun_out/pytest_3h.log
timeout -k 10 400 python -u tools/out_copy.py 1 8 16 24 32 > gpurun_out/out_copy.txt 2>&1 || exit 1
cat gpurun_out/out_copy.txt
