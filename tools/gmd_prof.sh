#!/bin/bash
# GMD / GMC checks and timing in one GPU call: the bit-exact GMD + GMC tests, tools/gmd_bench.py
# (8 streams), and a rocprofv3 kernel-trace summary of the same bench.  OUT_DIR under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r4gmd}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gmd_gpu.py tests/test_gmc_gpu.py tests/test_golden_gpu.py -m gpu -q \
  --timeout 200 --timeout-method thread -k "gmd or gmc or motion or global" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/gmd_bench.py --streams 8 > $O/gmd_bench.txt 2>&1 || { echo "bench failed"; tail -20 $O/gmd_bench.txt; exit 1; }
grep -v amdgpu.ids $O/gmd_bench.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o gmd -- python -u tools/gmd_bench.py --streams 8 --steps 100 > $O/gmd_prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/gmd_prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -16
