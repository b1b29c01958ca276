#!/bin/bash
# Tree-compiler + distributed GPU tests, then the bench with tree code (default) and without.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${TMO:-420} python -u -m pytest ${TESTS:-tests/test_jit_gpu.py tests/test_distributed_gpu.py} -x -v \
  --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_jit.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_jit.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_jit.json 2> gpurun_out/bench_jit.err || exit $?
cat gpurun_out/bench_jit.json
SRHIP_JIT=0 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_nojit.json 2>&1 || exit $?
cat gpurun_out/bench_nojit.json
timeout -k 10 200 python3 tools/jit_diag.py > gpurun_out/jit_diag.txt 2>&1 || exit $?
cat gpurun_out/jit_diag.txt
