set -o pipefail
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention" -p no:cacheprovider 2>&1 | tail -5
timeout -k 10 200 python tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -q -x -p no:cacheprovider 2>&1 | tail -3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch 64 2>&1 | tail -1
