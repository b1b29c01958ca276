#!/bin/bash
# round 3: gradient parity with the Float32-oracle noise, set_constants timing, gradient kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_jit_grad_gpu.py -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_3e.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_3e.log; [ $rc -le 1 ] || exit $rc
SRHIP_DEBUG_SETC=1 timeout -k 10 300 python -u tools/bench_constopt.py > gpurun_out/constopt_setc.txt 2> gpurun_out/constopt_setc.err || exit 1
head -3 gpurun_out/constopt_setc.txt
python3 - <<'PY'
import re
pt, up, rc, n = [], [], [], 0
for ln in open("gpurun_out/constopt_setc.err"):
    m = re.search(r"patch ([\d.]+) us, upload of (\d+) bytes ([\d.]+) us", ln)
    if m: pt.append(float(m.group(1))); up.append((int(m.group(2)), float(m.group(3))))
    m = re.search(r"(\d+) of (\d+) trees recompiled", ln)
    if m: rc.append((int(m.group(1)), int(m.group(2))))
import statistics as st
print("calls", len(pt), "patch us median", st.median(pt), "mean", st.mean(pt))
print("upload median us", st.median(u for _, u in up), "bytes median", st.median(b for b, _ in up))
print("recompiled median", st.median(r for r, _ in rc), "of median", st.median(t for _, t in rc))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof -o gp -- python3 tools/prof_grad.py 5 > gpurun_out/prof_grad.json 2> gpurun_out/prof_grad.err || exit 1
cat gpurun_out/prof_grad.json
find gpurun_out/gprof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-200
timeout -k 10 300 python -u tools/ab_env.py --ntrees 512 --steps 40 '' 'SRHIP_TREE_NT=2' 'SRHIP_MIN_PER_GROUP=32' 'SRHIP_MIN_PER_GROUP=32 SRHIP_TREE_NT=2' 'SRHIP_TREE_NT=3' > gpurun_out/ab_512.txt 2>&1 || exit 1
cat gpurun_out/ab_512.txt
