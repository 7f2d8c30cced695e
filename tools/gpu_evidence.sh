# One lease at HEAD: the GPU parity suite (+ parity report) and smoke, the default bench line
# (all sub-results), and the rocprofv3 stats + PMC passes of every mode, for profiles/<tag>_*
# (summarised on the CPU side by tools/pmc_report.py).
set -o pipefail
XFA_PARITY_REPORT=gpurun_out/parity.json timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -5 gpurun_out/gpu_suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/gpu_suite.log 2>&1 || { tail -5 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
rm -rf gpurun_out/prof
bash tools/pmc_round.sh fwd fwdbwd varlen decode decode_ragged fwd_fp8
