#!/bin/bash
# One runner for the GPU box (gpurun): each step under its own time limit,
# the first crash / hang / abort ends the script (no retries).
#   tools/gpu_run.sh suite    GPU test suite            -> gpurun_out/pytest_gpu.log
#   tools/gpu_run.sh smoke    __graft_entry__.smoke()   -> gpurun_out/smoke.log
#   tools/gpu_run.sh bench    bench.py (BENCH_ARGS)     -> gpurun_out/bench.json
#   tools/gpu_run.sh profile  bench under rocprofv3: kernel trace + PMC passes (tools/gpu_bench_profile.sh)
#   tools/gpu_run.sh configs  tools/bench_configs.py   -> gpurun_out/configs.jsonl
#   tools/gpu_run.sh final    suite, smoke, bench, profile
# Several modes may be given: tools/gpu_run.sh suite bench
# The round-3 measurements in profiles/ came from these tools, each step under
# its own `timeout -k 10 ...` on the box: ab_env.py (env-knob A/Bs: tail split,
# tree groups, waves), step_overhead.py, out_copy.py + hostcopy.cpp (per-row
# outputs), prof_grad.py / pmc_grad.sh / debug_grads.py (gradient tree code),
# pmc_shard.sh (512 vs 4096 trees), bench_constopt.py / prof_constopt.py,
# census.py (no GPU: the VALU-issue budget).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run_suite() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  local rc=$?
  echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  # 1 = test failures (the GPU is fine): go on; anything else (crash, time limit) stops
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run_smoke() {
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/smoke.log
}
run_bench() {
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
  tail -c 600 gpurun_out/bench.json
}
run_configs() {
  timeout -k 10 400 python -u tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || exit $?
  cat gpurun_out/configs.jsonl
}
run_profile() {
  bash tools/gpu_bench_profile.sh > gpurun_out/benchprof.log 2>&1 || exit $?
  tail -30 gpurun_out/benchprof.log
}
for mode in "$@"; do
  case "$mode" in
    suite) run_suite ;;
    smoke) run_smoke ;;
    bench) run_bench ;;
    profile) run_profile ;;
    configs) run_configs ;;
    final) run_suite; run_smoke; run_bench; run_profile ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
done
