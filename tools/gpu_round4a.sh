XFA_TEST_OPTIONS=fp8_w4=1 timeout -k 10 240 python -u -m pytest tests/test_fp8_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_fp8w4.log 2>&1; e=$?; tail -25 gpurun_out/r4_fp8w4.log
if [ $e -gt 1 ]; then echo "STOP e=$e"; exit $e; fi
if [ $e -eq 0 ]; then
  timeout -k 10 150 python tools/lib_ab.py xf_flash_attention_cutlass_amd/lib/libpaged-attention.so@fp8_w4=0 xf_flash_attention_cutlass_amd/lib/libpaged-attention.so@fp8_w4=1 --mode fwd_fp8 --rounds 5 > gpurun_out/ab_fp8w4.log 2>&1 || exit $?
  timeout -k 10 150 python tools/lib_ab.py xf_flash_attention_cutlass_amd/lib/libpaged-attention.so@fp8_w4=0 xf_flash_attention_cutlass_amd/lib/libpaged-attention.so@fp8_w4=1 --mode fwd_fp8 --rounds 5 --noncausal >> gpurun_out/ab_fp8w4.log 2>&1 || exit $?
  grep -E "fwd|check" gpurun_out/ab_fp8w4.log
fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_suite1.log 2>&1; e=$?; tail -5 gpurun_out/r4_suite1.log
if [ $e -gt 1 ]; then exit $e; fi
timeout -k 10 200 python tools/lib_ab.py variants/lib_k8incr.so variants/lib_warm.so --rounds 7 > gpurun_out/ab_warm_c.log 2>&1 && grep -E "fwd|check" gpurun_out/ab_warm_c.log && timeout -k 10 200 python tools/lib_ab.py variants/lib_k8incr.so variants/lib_warm.so --rounds 5 --noncausal > gpurun_out/ab_warm_nc.log 2>&1 && grep -E "fwd|check" gpurun_out/ab_warm_nc.log
