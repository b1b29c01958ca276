#!/bin/bash
# GPU parity suite, then microbench with the threaded interpreter on and off
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/microbench.py > gpurun_out/micro_ti.log 2>&1 || exit $?
echo "== TI"; cat gpurun_out/micro_ti.log
SRHIP_TI=0 timeout -k 10 200 python -u tools/microbench.py > gpurun_out/micro_noti.log 2>&1 || exit $?
echo "== no TI"; cat gpurun_out/micro_noti.log
