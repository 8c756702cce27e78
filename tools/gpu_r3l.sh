# round-3 check: C-ABI program build, motion-reset two-launch tracker, halo kernels; then the
# halo probe, concurrent autotune and the bench
set -o pipefail
O=gpurun_out/${OUT_DIR:-r3l}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_program_build_gpu.py tests/test_cmc_gpu.py tests/test_gmd_gpu.py tests/test_pipeline_gpu.py tests/test_tracker_gpu.py -k "not driver_loop" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_detector_gpu.py -k conv_variants > $O/pytest_det.log 2>&1 || { tail -30 $O/pytest_det.log; exit 1; }
tail -2 $O/pytest_det.log
timeout -k 10 200 python -u tools/halo_probe.py --plan plans/exp/s_640x512_i640_b8_fp32_r3h.json --ops 72,73,76,80,30,74,1,19,29,7 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v "^{" $O/probe.log
OUT_DIR=${OUT_DIR:-r3l} SKIP_BASE=1 bash tools/gpu_r3c.sh
