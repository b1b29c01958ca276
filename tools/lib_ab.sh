# Two libsrhip builds A/B, interleaved: the gradient workload (tools/prof_grad.py) and the bench kernel.
# LIB_B = the other build (SRHIP_LIB), e.g. ab/libsrhip_taylor.so
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/libab
for r in 1 2 3; do
  for v in cur other; do
    if [ $v = cur ]; then E=""; else E="SRHIP_LIB=$PWD/$LIB_B"; fi
    env $E timeout -k 10 300 python3 tools/prof_grad.py 5 > gpurun_out/libab/g_$v.json 2>> gpurun_out/libab/err.log || { echo "grad $v failed"; exit 1; }
    echo "grad $v $(tail -c 300 gpurun_out/libab/g_$v.json)"
    env $E timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/libab/b_$v.json 2>> gpurun_out/libab/err.log || { echo "bench $v failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/libab/b_$v.json').read().strip().splitlines()[-1]); print('bench $v', round(d['value']/1e12,3), round(d['roofline']['kernel_ms'],4))"
  done
done
