timeout -k 10 600 python -u tools/debug_outliers.py > gpurun_out/debug_outliers.txt 2>&1; head -10 gpurun_out/debug_outliers.txt
bash tools/gpu_run.sh suite bench && \
timeout -k 10 300 python tools/prof_constopt.py > gpurun_out/prof_constopt.txt 2>&1 && \
timeout -k 10 400 python -u tools/fast_parity.py both > gpurun_out/fast_parity.log 2>&1; \
head -12 gpurun_out/prof_constopt.txt; grep -E "fast:|precise:" gpurun_out/fast_parity.log | cut -c1-300
