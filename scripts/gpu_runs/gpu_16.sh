#!/bin/bash
# Side-stream SGD vs fused-epilogue SGD on the flagship step (N=1).
source scripts/gpu_steps.sh
step side_tests 300 python -m pytest tests/test_side_opt_gpu.py -q -m gpu -x
step b_fused 600 python bench.py --steps 20 --warmup 3
step b_side32 600 python bench.py --steps 20 --warmup 3 --side_opt 32
step b_side16 600 python bench.py --steps 20 --warmup 3 --side_opt 16
step b_side64 600 python bench.py --steps 20 --warmup 3 --side_opt 64
step b_fused2 600 python bench.py --steps 20 --warmup 3
