#!/bin/bash
# Parity of the given scoring variants on the pre-filter tests (each under its own time limit,
# so a hung variant ends the script), then an interleaved C2 step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${1:-89}
for v in ${V//,/ }; do
  timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_parity.py \
      -k "prefilter_equals and $v" > gpurun_out/vc_$v.log 2>&1
  rc=$?; echo "variant $v tests rc=$rc $(tail -1 gpurun_out/vc_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
ROUNDS=${ROUNDS:-6} timeout -k 10 200 python3 -u scripts/step_variant_ab.py $V 2>&1 | grep variant
