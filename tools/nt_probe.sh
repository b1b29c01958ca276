# tiles per workgroup of the loss tree code (SRHIP_TREE_NT): bench kernel time per setting
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/nt
for nt in 4 6 8 4 6 8; do
  SRHIP_TREE_NT=$nt timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/nt/nt$nt.json 2> gpurun_out/nt/nt$nt.err || { echo "nt $nt failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/nt/nt$nt.json').read().strip().splitlines()[-1]); print('nt $nt', d['value']/1e12, d['roofline']['kernel_ms'])"
done
