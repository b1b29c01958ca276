#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SRHIP_RG_XCD=1 timeout -k 10 300 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rgxcd.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_rgxcd.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run() { echo "== $*"; env "$@" timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/rx.log 2>&1 || exit $?;
        tail -1 gpurun_out/rx.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4))"; }
run SRHIP_RG_XCD=0
run SRHIP_RG_XCD=1
run SRHIP_RG_XCD=0
run SRHIP_RG_XCD=1
for c in 0 1; do SRHIP_RG_XCD=$c timeout -k 10 120 python3 tools/prof_grad.py 2 > gpurun_out/gx.log 2>&1 || exit $?; echo "grad rg_xcd=$c $(tail -1 gpurun_out/gx.log | cut -c1-160)"; done
