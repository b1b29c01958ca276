#!/bin/bash
# Experimental interpreter variants: GPU parity tests + per-operator microbench
# for each lib/libsrhip_<name>.so given on the command line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/variants
for v in "$@"; do
  lib="$PWD/symbolicregression.jl_amd/lib/libsrhip${v:+_$v}.so"
  [ "$v" = base ] && lib="$PWD/symbolicregression.jl_amd/lib/libsrhip.so"
  echo "=== $v"
  SRHIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/variants/pytest_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/variants/pytest_$v.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  SRHIP_LIB=$lib timeout -k 10 200 python -u tools/microbench.py > gpurun_out/variants/micro_$v.log 2>&1 || exit $?
  cat gpurun_out/variants/micro_$v.log
done
