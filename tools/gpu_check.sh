#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, the default bench line, then the
# rocprof passes of tools/prof.sh.  Every GPU step has its own time limit and
# the chain stops at the first failure.
#   tools/gpu_check.sh <tag> [tests|bench|prof|all]
set -eo pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r01}
WHAT=${2:-all}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/tests_$TAG.log" 2>&1
  echo "tests ok"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1
  echo "smoke ok"
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  timeout -k 10 300 python -u bench.py > "$O/bench_$TAG.log" 2>&1
  tail -1 "$O/bench_$TAG.log"
fi
if [ "$WHAT" = prof ] || [ "$WHAT" = all ]; then
  bash "$R/tools/prof.sh" "$TAG" c2
  cat "$O/prof_$TAG/summary.txt"
fi
