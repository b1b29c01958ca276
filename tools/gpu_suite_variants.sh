#!/bin/bash
# The GPU suite under the fallback schedules (compiled static loops:
# SRHIP_JIT_DYNLOOP=0 SRHIP_INTERP_DYN=0) and with every program as tree code
# (SRHIP_JIT=1), each in one process; logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
SRHIP_JIT_DYNLOOP=0 SRHIP_INTERP_DYN=0 timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_static.log 2>&1
rc=$?; echo "static loops rc=$rc"; tail -2 gpurun_out/pytest_static.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SRHIP_JIT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_jitall.log 2>&1
rc=$?; echo "SRHIP_JIT=1 rc=$rc"; tail -2 gpurun_out/pytest_jitall.log; grep -E "^FAILED" gpurun_out/pytest_jitall.log | head
exit 0
