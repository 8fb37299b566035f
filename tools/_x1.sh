set -o pipefail
mkdir -p gpurun_out/x5
S=tools/gpu_steps.sh
$S 200 python -u -m pytest tests/test_gpu_jpeg.py -x -v --timeout 60 --timeout-method thread ::: \
   300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ::: \
   200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline ::: \
   200 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d gpurun_out/x5/tr -o run -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-profile
