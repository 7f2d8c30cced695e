# Evidence call A (one lease): the GPU suite with the parity report and smoke, then the default
# bench line and the forward schedule A/B (tools/lease_ab.sh).  Call B: tools/pmc_round.sh.
# usage: bash tools/evidence_a.sh <tag>
set -o pipefail
tag=${1:-ev}
mkdir -p gpurun_out
XFA_PARITY_REPORT=gpurun_out/parity.json timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || { tail -5 gpurun_out/gpu_suite.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/gpu_suite.log 2>&1 || { tail -5 gpurun_out/gpu_suite.log; exit 1; }
tail -3 gpurun_out/gpu_suite.log
bash tools/lease_ab.sh ${tag} || exit 1
