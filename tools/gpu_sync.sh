#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py tests/test_gpu_parity.py tests/test_threaded.py tests/test_gradients.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_sync.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sync.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for nt in 4096 512; do
  timeout -k 10 200 python3 bench.py --no-cpu --ntrees $nt --steps 40 --warmup 10 > gpurun_out/sync.log 2>&1 || exit $?
  tail -1 gpurun_out/sync.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ntrees', d['config']['ntrees'], 'kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3), 'value', d['value'])"
done
