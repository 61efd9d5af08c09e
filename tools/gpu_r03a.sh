set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03_pytest_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 > gpurun_out/r03_bench.log 2>&1
