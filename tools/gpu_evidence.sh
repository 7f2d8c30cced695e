# One lease: the default bench line (all sub-results) and the rocprofv3 stats + PMC passes of
# every mode, for profiles/<tag>_* (summarised on the CPU side by tools/pmc_report.py).
set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
bash tools/pmc_round.sh fwd fwdbwd varlen decode decode_ragged fwd_fp8
