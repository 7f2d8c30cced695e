# round 4: fp8 4-wave validation + A/B, graph-capturable dropout tests
L=xf_flash_attention_cutlass_amd/lib/libpaged-attention.so
timeout -k 10 150 python -u tools/fp8w4_debug.py > gpurun_out/fp8dbg.log 2>&1; e=$?; cat gpurun_out/fp8dbg.log; [ $e -le 1 ] || exit $e
XFA_TEST_OPTIONS=fp8_w4=1 timeout -k 10 240 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_fp8w4.log 2>&1; e=$?; tail -15 gpurun_out/r4_fp8w4.log; [ $e -le 1 ] || exit $e
if [ $e -eq 0 ]; then
  timeout -k 10 150 python tools/lib_ab.py $L@fp8_w4=0 $L@fp8_w4=1 --mode fwd_fp8 --rounds 5 > gpurun_out/ab_fp8w4.log 2>&1 || exit $?
  timeout -k 10 150 python tools/lib_ab.py $L@fp8_w4=0 $L@fp8_w4=1 --mode fwd_fp8 --rounds 5 --noncausal >> gpurun_out/ab_fp8w4.log 2>&1 || exit $?
  grep -E "fwd|check" gpurun_out/ab_fp8w4.log
fi
timeout -k 10 150 python tools/lib_ab.py variants/lib_decold.so $L@comb_row=0 $L@comb_row=1 --mode decode --rounds 7 > gpurun_out/ab_dec.log 2>&1 && timeout -k 10 150 python tools/lib_ab.py variants/lib_decold.so $L@comb_row=0 $L@comb_row=1 --mode decode --ragged --rounds 7 >> gpurun_out/ab_dec.log 2>&1; e=$?; grep -E "decode|check" gpurun_out/ab_dec.log; [ $e -eq 0 ] || exit $e
timeout -k 10 200 python -u -m pytest tests/test_dropout_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/drop.log 2>&1; e=$?; tail -15 gpurun_out/drop.log; [ $e -le 1 ] || exit $e
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r4_suite2.log 2>&1; e=$?; tail -12 gpurun_out/r4_suite2.log; exit $e
