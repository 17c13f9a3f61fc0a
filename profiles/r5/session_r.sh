#!/bin/bash
# Round-5 GPU session R: the stem's board loads beside the plan load (product)
# vs after it (variants/noprebd.py): tower parity, then the isolated forward
# at 456 and 4096 boards and configs[1], alternating.
set -o pipefail
out=gpurun_out/r5r
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k "forward or network or tower" --timeout 200 \
  --timeout-method thread > $out/tests.log 2>&1 || { tail -20 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for r in 1 2; do
  for v in base noprebd; do
    if [ "$v" = base ]; then lib=$PWD/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else lib=$PWD/profiles/ab_libs/$v/libaz.so; fi
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 456 20 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
    AZ_LIB_PATH=$lib timeout -k 10 120 python3 profiles/conv_bench.py 4096 10 0 2>&1 | tail -1 | sed "s/^/$v /" | tee -a $out/iso.txt || exit 1
  done
done
bash profiles/r5/ab_bench.sh 2 "" base noprebd 2>&1 | tee $out/ab.txt
