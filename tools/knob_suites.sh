# The GPU suite under non-default knob values (every knob is result-preserving, so the whole
# suite must pass under each): usage: bash tools/knob_suites.sh "fwd_w4=2" "fwd_w4=3" ...
set -o pipefail
for o in "$@"; do
  echo "== XFA_TEST_OPTIONS=$o"
  XFA_TEST_OPTIONS="$o" timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
done
