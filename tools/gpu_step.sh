#!/bin/bash
# tree-code + parity GPU tests, then the bench and its kernel trace (per-step overheads)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_gpu_parity.py tests/test_jit_grad_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_step.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_step.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 10 > gpurun_out/step.log 2>&1 || exit $?
tail -1 gpurun_out/step.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stepkt -o kt -- python3 bench.py --steps 20 --warmup 10 --no-cpu > gpurun_out/step_kt.json 2> gpurun_out/step_kt.err || exit $?
cut -c1-150 gpurun_out/stepkt/kt_kernel_stats.csv
