# round 3: suite, smoke, bench (with the row-shard leg), profile, then the side measurements
bash tools/gpu_run.sh final
timeout -k 10 300 python -u tools/prof_grad.py > gpurun_out/prof_grad.json 2>&1; tail -1 gpurun_out/prof_grad.json
timeout -k 10 300 python tools/prof_constopt.py > gpurun_out/prof_constopt.txt 2>&1; head -14 gpurun_out/prof_constopt.txt
timeout -k 10 400 python -u tools/fast_parity.py both > gpurun_out/fast_parity.log 2>&1; grep -E "fast:|precise:" gpurun_out/fast_parity.log | cut -c1-250
