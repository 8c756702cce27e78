set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gmd_gpu.py -k many > gpurun_out/gmd2.log 2>&1 &&
timeout -k 10 300 python -u tools/gmd_bench.py --steps 200 > gpurun_out/gmd_bench.json 2> gpurun_out/gmd_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gmdprof -o gmd -- python -u tools/gmd_bench.py --streams 8 --steps 100 > gpurun_out/gmd_prof.log 2>&1
