timeout -k 10 400 python -u tools/debug_tree.py 1000 2800 > gpurun_out/debug_tree.txt 2>&1; grep "\[" gpurun_out/debug_tree.txt | cut -c1-150
bash tools/gpu_run.sh suite bench && \
timeout -k 10 300 python -u tools/bench_constopt.py > gpurun_out/constopt.json 2>&1 && \
timeout -k 10 400 python -u tools/fast_parity.py cfg2 > gpurun_out/fast_parity.log 2>&1; \
tail -1 gpurun_out/constopt.json; grep -E "fast:|precise:" gpurun_out/fast_parity.log | cut -c1-300
