set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gmd_gpu.py tests/test_cmc_gpu.py > gpurun_out/gmd1.log 2>&1
