#!/bin/bash
# GPU probe: each step in its own process under a short timeout; stop at the first hang/crash.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
libs=${LIBS:-"libsrhip.so"}
steps=${STEPS:-"leaf|const|cos|rand 3|rand 50|loss 50"}
for lib in $libs; do
  export SRHIP_LIB=$GRAFT_REPO_ROOT/symbolicregression.jl_amd/lib/$lib
  IFS='|'; for s in $steps; do unset IFS
    echo "== $lib $s" | tee -a gpurun_out/diag.log
    timeout -k 5 ${TMO:-40} python -u tools/diag.py $s >> gpurun_out/diag.log 2>&1
    rc=$?
    echo "rc=$rc" | tee -a gpurun_out/diag.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
