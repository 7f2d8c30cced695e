# round 4: fp8 idle-step epilogue (tests + A/B), decode load cache-policy A/B
L=xf_flash_attention_cutlass_amd/lib/libpaged-attention.so
timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_f8e.log 2>&1; e=$?; tail -2 gpurun_out/r4_f8e.log; [ $e -eq 0 ] || exit $e
timeout -k 10 150 python tools/lib_ab.py variants/lib_f8noepi.so $L --mode fwd_fp8 --rounds 9 > gpurun_out/ab_f8e.log 2>&1 || exit $?
grep -hE "^fwd|check" gpurun_out/ab_f8e.log
timeout -k 10 150 python tools/lib_ab.py $L variants/lib_nt2.so variants/lib_nt1.so --mode decode --rounds 9 > gpurun_out/ab_nt.log 2>&1 && timeout -k 10 150 python tools/lib_ab.py $L variants/lib_nt2.so variants/lib_nt1.so --mode decode --ragged --rounds 9 >> gpurun_out/ab_nt.log 2>&1; e=$?; grep -hE "^decode|check" gpurun_out/ab_nt.log; exit $e
