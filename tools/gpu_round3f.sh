#!/bin/bash
# round 3: constant map with folded values, varying-constants programs; constopt timing
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_constant_optimization.py tests/test_jit_grad_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_3f.log 2>&1 || { tail -30 gpurun_out/pytest_3f.log; exit 1; }
tail -2 gpurun_out/pytest_3f.log
SRHIP_DEBUG_SETC=1 timeout -k 10 300 python -u tools/bench_constopt.py > gpurun_out/constopt_setc.txt 2> gpurun_out/constopt_setc.err || exit 1
head -3 gpurun_out/constopt_setc.txt
python3 - <<'PY'
import re, statistics as st
pt, up, rc = [], [], []
for ln in open("gpurun_out/constopt_setc.err"):
    m = re.search(r"patch ([\d.]+) us, upload of (\d+) bytes ([\d.]+) us", ln)
    if m: pt.append(float(m.group(1))); up.append((int(m.group(2)), float(m.group(3))))
    m = re.search(r"(\d+) of (\d+) trees recompiled", ln)
    if m: rc.append((int(m.group(1)), int(m.group(2))))
print("calls", len(pt), "patch us median", st.median(pt), "mean", st.mean(pt), "total ms", sum(pt) / 1e3)
print("upload median us", st.median(u for _, u in up), "total ms", sum(u for _, u in up) / 1e3, "bytes median", st.median(b for b, _ in up))
print("recompiled median", st.median(r for r, _ in rc), "max", max(r for r, _ in rc), "of median", st.median(t for _, t in rc))
PY
timeout -k 10 300 python -u tools/prof_constopt.py > gpurun_out/constopt_profile.txt 2>&1 || exit 1
head -25 gpurun_out/constopt_profile.txt
SRHIP_DEBUG_PASSES=1 timeout -k 10 300 python -u tools/prof_grad.py 3 > gpurun_out/prof_grad_dbg.json 2> gpurun_out/prof_grad_dbg.err || exit 1
cat gpurun_out/prof_grad_dbg.json; grep "grad tree code" gpurun_out/prof_grad_dbg.err | tail -4
