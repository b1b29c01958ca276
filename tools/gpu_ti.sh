#!/bin/bash
# threaded interpreter: GPU parity suite, then microbench of the default lib and
# of the variants named on the command line (lib/libsrhip_<v>.so)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/microbench.py > gpurun_out/micro_base.log 2>&1 || exit $?
echo "== base"; cat gpurun_out/micro_base.log
for v in "$@"; do
  SRHIP_LIB=$PWD/symbolicregression.jl_amd/lib/libsrhip_$v.so timeout -k 10 200 python -u tools/microbench.py > gpurun_out/micro_$v.log 2>&1 || exit $?
  echo "== $v"; cat gpurun_out/micro_$v.log
done
