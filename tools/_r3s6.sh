mkdir -p gpurun_out/r3_step13
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_full_geometry_gpu.py -x -v --timeout 200 --timeout-method thread -k "xattn or full_half or full_geometry_matches_oracle" > gpurun_out/r3_step13/pytest.log 2>&1 && bash tools/_ab.sh r3_step13 ACTH_FUSED_XATTN=1 ACTH_FUSED_XATTN=0 --steps 5 --warmup 1
rc=$?; tail -4 gpurun_out/r3_step13/pytest.log; exit $rc
