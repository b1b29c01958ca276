#!/bin/bash
# GPU suite, then config #2 bench with the tree-order rotation off/on (SRHIP_ROT)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rot.log 2>&1 || exit $?
for r in 0 1 0 1; do SRHIP_ROT=$r timeout -k 10 120 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/ab_$r.log 2>&1 || exit $?; echo "rot=$r $(python -c "import json;d=json.loads(open('gpurun_out/ab_$r.log').read().strip().splitlines()[-1]);print(d['roofline']['kernel_ms'], d['value']/1e12)")"; done
