#!/bin/bash
# Round-5 GPU session A: the GPU suite, the default bench (configs[1]), the
# chess bench (configs[4] shard), and the 16-wave tower variant's parity +
# alternating in-bench A/B.  Every GPU step under its own time limit.
set -o pipefail
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 \
  || { tail -30 $out/gpu_tests.log; exit 1; }
tail -3 $out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
tail -c 400 $out/bench.json; echo
timeout -k 10 300 python bench.py --game chess --no-cpu-baseline > $out/chess.json 2> $out/chess.err || { tail -5 $out/chess.err; exit 1; }
tail -c 400 $out/chess.json; echo
AZ_LIB_PATH=$PWD/profiles/ab_libs/nwm4/libaz.so timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q \
  -k "forward or network or tower" --timeout 200 --timeout-method thread > $out/nwm4_tests.log 2>&1 || { tail -20 $out/nwm4_tests.log; exit 1; }
tail -2 $out/nwm4_tests.log
bash profiles/r5/ab_bench.sh 2 "" base nwm4
