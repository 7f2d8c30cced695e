# One lease at HEAD: the GPU parity suite (+ parity report) and smoke, the default bench line
# (all sub-results), the forward schedule A/B (tools/lease_ab.sh without its bench), and the
# rocprofv3 stats + PMC passes of every mode, for profiles/<tag>_* (summarised on the CPU side by
# tools/pmc_report.py).   usage: bash tools/gpu_evidence.sh <tag>
set -o pipefail
tag=${1:-ev}
XFA_PARITY_REPORT=gpurun_out/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -5 gpurun_out/gpu_suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/gpu_suite.log 2>&1 || { tail -5 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
bash tools/lease_ab.sh ${tag} || exit 1
rm -rf gpurun_out/prof
bash tools/pmc_round.sh fwd fwd_nc fwd_alibi fwd_window fwdbwd varlen decode decode_ragged fwd_fp8
