source scripts/gpu_steps.sh
step quick_bench 300 python3 bench.py --steps 10 --warmup 3 --methods none --json_out gpurun_out/quick.json
