#!/bin/bash
# Round-4 loss-parity guards: full-size FAST parity (tools/fast_parity.py) and the
# bench kernel time with the guards / sticky PRECISE on and off.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u tools/fast_parity.py both > gpurun_out/fp.log 2>&1 || exit 1
for cfg in "1 1" "0 1" "1 0" "1 1"; do set -- $cfg
  SRHIP_JIT_LOSS_GUARDS=$1 SRHIP_JIT_STICKY=$2 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/bg_$1_$2.json 2>>gpurun_out/bg.err || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/bg_$1_$2.json')); print('guards $1 sticky $2', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['tree_code'])
"
done
grep -v "^    " gpurun_out/fp.log
