# round 4: redo paths (fall-through stubs), fp8 row-sum split A/B, full suite
L=xf_flash_attention_cutlass_amd/lib/libpaged-attention.so
timeout -k 10 200 python -u -m pytest tests/test_fwd4_redo_gpu.py tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_redo.log 2>&1; e=$?; tail -3 gpurun_out/r4_redo.log; [ $e -eq 0 ] || exit $e
timeout -k 10 150 python tools/lib_ab.py variants/lib_f8prev.so $L --mode fwd_fp8 --rounds 7 > gpurun_out/ab_f8.log 2>&1 && timeout -k 10 150 python tools/lib_ab.py variants/lib_f8prev.so $L --mode fwd_fp8 --rounds 5 --noncausal >> gpurun_out/ab_f8.log 2>&1; e=$?; grep -E "fwd|check" gpurun_out/ab_f8.log; [ $e -eq 0 ] || exit $e
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r4_suite5.log 2>&1; e=$?; tail -3 gpurun_out/r4_suite5.log; exit $e
