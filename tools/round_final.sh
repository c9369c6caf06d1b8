#!/bin/bash
# End-of-round evidence in one call: the full -m gpu suite, then tools/profile_round.sh TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gt_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/gt_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh $TAG
