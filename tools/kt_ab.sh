cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out/kt && export TMPDIR=/tmp && 
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt/on -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/kt/on.json 2> gpurun_out/kt/on.err &&
SRHIP_JIT_GCOLS=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt/off -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/kt/off.json 2> gpurun_out/kt/off.err &&
SRHIP_JIT_GCOLS=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt/g16 -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-row-shard > gpurun_out/kt/g16.json 2> gpurun_out/kt/g16.err &&
find gpurun_out/kt -name "*stats*" | head
