#!/bin/bash
# The one runner for the GPU box (gpurun): each step under its own time limit,
# the first crash / hang / abort ends the script (no retries). Several modes
# may be given: tools/gpu_run.sh suite bench
#   suite     GPU test suite (one process)               -> gpurun_out/pytest_gpu.log
#   smoke     __graft_entry__.smoke()                    -> gpurun_out/smoke.log
#   bench     bench.py $BENCH_ARGS                       -> gpurun_out/bench.json
#   profile   bench.py under rocprofv3: kernel trace + the PMC passes -> gpurun_out/benchprof/summary.json
#             (copy to profiles/current_pmc_summary.json: bench.py attaches it when kernel + lib hash match)
#   pmc       PMC passes of any command: PMC_KERNEL=<name substring> PMC_CMD="python3 tools/x.py ..."
#   configs   tools/bench_configs.py                     -> gpurun_out/configs.jsonl
#   search    default-Options EquationSearch: the search GPU tests, configs #1 and #4
#             (tools/run_search.py)                      -> gpurun_out/search_config{1,4}.json
#   n2        bench.py's N > 1 paths rehearsed with two ranks on GPU 0 over gloo (not a measurement)
#   variants  the suite under the static tree loops and with every program as tree code
#   final     suite, smoke, bench, profile
#   tests     some GPU tests: TESTS="tests/test_a.py tests/test_b.py -k x"   -> gpurun_out/pytest_some.log
#   tool      one measurement tool: TOOL="tools/ab_build.py --grad A B"       -> gpurun_out/tool.log
#   envab     bench kernel time under environment settings, interleaved over ROUNDS (default 2):
#             ENV_VARIANTS="default SRHIP_TREE_NT=6 SRHIP_JIT_GCOLS=16,SRHIP_JIT_STICKY_TREE=1 SRHIP_LIB=ab/x.so"
#             (replaces the single-use *_probe.sh / *_ab.sh scripts of rounds 3-6)
# Measurement tools run on the box through this script (each under timeout):
# ab_env.py / loop_ab.py (interleaved A/Bs), step_overhead.py, out_copy.py,
# prof_grad.py, prof_target.py, shard_probe.py, bench_constopt.py,
# prof_constopt.py; census.py needs no GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTEST="python -u -m pytest -v --timeout 300 --timeout-method thread"

run_suite() {
  timeout -k 10 900 $PYTEST tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
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
# pmc_passes <outdir> <kernel substring> <command...>: the counter passes of
# MI355X_MICROARCH.md, each its own run (rocprofv3 does not split passes)
pmc_passes() {
  local out=$1 kern=$2; shift 2
  mkdir -p "$out"
  local P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_BRANCH"
  local P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES"
  local P3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32"
  local P4="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE"
  local i=0 P
  for P in "$P1" "$P2" "$P3" "$P4" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d "$out/pmc$i" -o pmc$i -- "$@" \
      > "$out/run_pmc$i.out" 2>> "$out/log.txt" || { echo "pmc pass $i failed"; exit 1; }
  done
  KERNEL="$kern" WORKLOAD="${WORKLOAD:-config#2}" python3 tools/pmc_summary.py "$out" > "$out/summary.json" && cat "$out/summary.json"
}
run_profile() {
  local OUT=gpurun_out/benchprof
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 bench.py --steps 20 --warmup 10 --no-cpu --no-row-shard > $OUT/bench_kt.json 2> $OUT/log.txt || exit $?
  pmc_passes $OUT sr_jit_eval python3 bench.py --steps 3 --warmup 1 --no-cpu --no-row-shard
}
run_pmc() {
  [ -n "$PMC_CMD" ] || { echo "PMC_CMD not set"; exit 2; }
  mkdir -p gpurun_out/pmc
  # the same command under the kernel trace first: the summary's avg_ms_kernel_trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o kt -- $PMC_CMD \
    > gpurun_out/pmc/kt.out 2>> gpurun_out/pmc/log.txt || { echo "kernel trace failed"; exit 1; }
  WORKLOAD="${PMC_WORKLOAD:-unlabelled}" pmc_passes gpurun_out/pmc "${PMC_KERNEL:-sr_jit}" $PMC_CMD
}
run_search() {
  timeout -k 10 700 $PYTEST tests/test_evolution.py tests/test_search.py tests/test_configs_gpu.py -m gpu -s \
    -k "search or evolution or config4 or config1" > gpurun_out/pytest_search.log 2>&1
  local rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_search.log | tail -8
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 400 python -u tools/run_search.py config1 --iterations 40 --out gpurun_out/search_config1.json \
    > gpurun_out/search_c1.log 2>&1 || exit $?
  tail -3 gpurun_out/search_c1.log | cut -c1-400
  timeout -k 10 400 python -u tools/run_search.py config1 --iterations 40 --batching --out gpurun_out/search_config1_batching.json \
    > gpurun_out/search_c1b.log 2>&1 || exit $?
  tail -3 gpurun_out/search_c1b.log | cut -c1-400
  timeout -k 10 600 python -u tools/run_search.py config4 --iterations ${C4_ITERS:-3} --out gpurun_out/search_config4.json \
    > gpurun_out/search_c4.log 2>&1 || exit $?
  tail -5 gpurun_out/search_c4.log | cut -c1-600
}
run_n2() {
  SRHIP_BENCH_SHARED_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 5 --warmup 2 --rs-steps 2 \
    > gpurun_out/bench_n2_rows.json 2> gpurun_out/bench_n2_rows.err || { tail -20 gpurun_out/bench_n2_rows.err; exit 1; }
  SRHIP_BENCH_SHARED_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --shard trees --steps 5 --warmup 2 --no-row-shard \
    > gpurun_out/bench_n2_trees.json 2> gpurun_out/bench_n2_trees.err || { tail -20 gpurun_out/bench_n2_trees.err; exit 1; }
  tail -c 300 gpurun_out/bench_n2_rows.json gpurun_out/bench_n2_trees.json
}
run_variants() {
  [ -n "$JITALL_ONLY" ] && { run_jitall; return; }
  SRHIP_JIT_DYNLOOP=0 SRHIP_INTERP_DYN=0 timeout -k 10 600 $PYTEST tests -m gpu > gpurun_out/pytest_static.log 2>&1
  local rc=$?; echo "static loops rc=$rc"; tail -2 gpurun_out/pytest_static.log
  [ $rc -le 1 ] || exit $rc
  # (the search tests run thousands of small programs: as tree code each one costs a code-object load)
  run_jitall
}
run_tests() {
  timeout -k 10 600 $PYTEST $TESTS -m gpu > gpurun_out/pytest_some.log 2>&1
  local rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_some.log | tail -12
  [ $rc -le 1 ] || exit $rc
}
run_tool() {
  [ -n "$TOOL" ] || { echo "TOOL not set"; exit 2; }
  timeout -k 10 ${TOOL_TIMEOUT:-600} python -u $TOOL > gpurun_out/tool.log 2> gpurun_out/tool.err || { tail -20 gpurun_out/tool.err; exit 1; }
  cat gpurun_out/tool.log | cut -c1-700
}
run_envab() {
  mkdir -p gpurun_out/envab
  local r v E tag
  for r in $(seq ${ROUNDS:-2}); do
    for v in ${ENV_VARIANTS:-default}; do
      E=$(echo "$v" | tr ',' ' '); [ "$v" = default ] && E=""
      tag=$(echo "$v" | tr -c 'A-Za-z0-9_=\n' '_')
      env $E timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard \
        > gpurun_out/envab/${tag}_$r.json 2>> gpurun_out/envab/err.log || { echo "$v failed"; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/envab/${tag}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e12, 3), round(d['roofline']['kernel_ms'], 4))"
    done
  done
}
run_jitall() {
  SRHIP_JIT=1 timeout -k 10 600 $PYTEST tests -m gpu -k "not evolution and not search" > gpurun_out/pytest_jitall.log 2>&1
  rc=$?; echo "SRHIP_JIT=1 rc=$rc"; tail -2 gpurun_out/pytest_jitall.log
  [ $rc -le 1 ] || exit $rc
}
for mode in "$@"; do
  case "$mode" in
    suite) run_suite ;;
    smoke) run_smoke ;;
    bench) run_bench ;;
    profile) run_profile ;;
    pmc) run_pmc ;;
    configs) run_configs ;;
    search) run_search ;;
    n2) run_n2 ;;
    variants) run_variants ;;
    final) run_suite; run_smoke; run_bench; run_profile ;;
    tests) run_tests ;;
    tool) run_tool ;;
    envab) run_envab ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
done
