#!/bin/bash
# bisect helper: the same tree-code tests against several builds (SRHIP_LIB);
# an argument NAME=VALUE sets an environment variable for the builds after it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for V in "$@"; do
  case "$V" in *=*) export "$V"; continue ;; esac
  lib=symbolicregression.jl_amd/lib/libsrhip_$V.so
  [ "$V" = cur ] && lib=symbolicregression.jl_amd/lib/libsrhip.so
  SRHIP_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_jit_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "precise_tree_code_equals or constant_divisor" > gpurun_out/bisect_$V.log 2>&1
  rc=$?; echo "$V rc=$rc ($(env | grep ^SRHIP_ | tr '\n' ' '))"; tail -2 gpurun_out/bisect_$V.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
