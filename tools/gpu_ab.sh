#!/bin/bash
# Tree-code tests, then the bench under the default and under $AB (an env assignment, e.g. SRHIP_JIT_INLINE=0).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 ${TMO:-420} python -u -m pytest ${TESTS:-tests/test_jit_gpu.py} -x -v \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_a$k.json 2> gpurun_out/bench_a$k.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_a$k.json'));print('A', d['ms_per_step'], d['roofline']['kernel_ms'], d['tree_code'])"
  env $AB timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_b$k.json 2> gpurun_out/bench_b$k.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/bench_b$k.json'));print('B', d['ms_per_step'], d['roofline']['kernel_ms'], d['tree_code'])"
done
