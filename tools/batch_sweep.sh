set -e
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/sw_b256.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --graph > gpurun_out/sw_b256g.log 2>&1
timeout -k 10 240 python bench.py --steps 8 --warmup 3 --batch 384 > gpurun_out/sw_b384.log 2>&1
timeout -k 10 300 python bench.py --steps 6 --warmup 3 --batch 512 > gpurun_out/sw_b512.log 2>&1
for f in gpurun_out/sw_*.log; do echo $f; grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus[^,]*, "steps[^,]*, "warmup[^,]*, "ms_per_step": [0-9.]*' $f; grep -o '"peak_mem_gb": [0-9.]*' $f; done
