#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/inl.log 2>&1 || exit $?;
        tail -1 gpurun_out/inl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel_ms', round(d['roofline']['kernel_ms'],3), 'frac', round(d['roofline']['frac'],4), 'code', d['tree_code']['code_bytes'])"; }
run SRHIP_JIT_INLINE=0
run SRHIP_JIT_INLINE=1 SRHIP_JIT_INLINE_MAX=200
run SRHIP_JIT_INLINE=1 SRHIP_JIT_INLINE_MAX=320
run SRHIP_JIT_INLINE=1
run SRHIP_JIT_INLINE=0
