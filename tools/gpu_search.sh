#!/bin/bash
# Default-Options EquationSearch on the engine (srhip.evolution): the GPU
# tests of the search paths, then the recorded runs of BASELINE configs #1
# (20 islands x 40 iterations) and #4 (64 islands, 10 x 100k) under
# gpurun_out/ (copied to profiles/r05_search_config*.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_evolution.py tests/test_search.py tests/test_configs_gpu.py -m gpu -v \
  --timeout 600 --timeout-method thread -k "search or evolution or config4 or config1" -s > gpurun_out/pytest_search.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|evals" gpurun_out/pytest_search.log | tail -8; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/run_search.py config1 --iterations 40 --out gpurun_out/search_config1.json > gpurun_out/search_c1.log 2>&1 || exit $?
tail -3 gpurun_out/search_c1.log | cut -c1-400
timeout -k 10 600 python -u tools/run_search.py config4 --iterations ${C4_ITERS:-3} --out gpurun_out/search_config4.json > gpurun_out/search_c4.log 2>&1 || exit $?
tail -5 gpurun_out/search_c4.log | cut -c1-600
