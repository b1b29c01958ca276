#!/bin/bash
# packed tree code (v_pk_*_f32) A/B on config #2 + tree-code GPU tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_jit_gpu.py tests/test_jit_grad_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_packed.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_packed.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in "SRHIP_JIT_PACKED=0 SRHIP_JIT_PKMOV=0" "SRHIP_JIT_PACKED=1 SRHIP_JIT_PKMOV=0" "SRHIP_JIT_PACKED=1 SRHIP_JIT_PKMOV=1" "SRHIP_JIT_PACKED=0 SRHIP_JIT_PKMOV=0"; do
  env $cfg timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 10 > gpurun_out/pk.log 2>&1 || exit $?
  tail -1 gpurun_out/pk.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'kernel_ms', round(d['roofline']['kernel_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
done
