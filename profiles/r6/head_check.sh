#!/bin/bash
# Round-6 check of a build on one MI355X (repo root, under gpurun):
#   the GPU suite, the default bench line (configs[1] with the CPU legs),
#   the PMC passes for the build (collect_pmc.sh) and a rocprofv3 kernel trace
#   of the bench (prof_bench.sh).  SKIP="tests pmc prof" drops steps.
set -o pipefail
T=${TAG:-head}
OUT=gpurun_out/r6/check_$T
mkdir -p $OUT
skip() { [[ " $SKIP " == *" $1 "* ]]; }
if ! skip tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 500 python3 -u bench.py > $OUT/c4.json 2> $OUT/c4.err || { tail -20 $OUT/c4.err; exit 1; }
tail -c 600 $OUT/c4.json; echo
if ! skip pmc; then
  TAG=_$T bash profiles/r6/collect_pmc.sh > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
fi
if ! skip prof; then
  bash profiles/r6/prof_bench.sh $T > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  head -20 $OUT/prof.log
fi
echo check done
