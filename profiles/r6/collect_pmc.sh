#!/bin/bash
# Round-6 PMC collection for the benched build (repo root, under gpurun):
# rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES +
# SQ_INSTS_MFMA + GRBM_GUI_ACTIVE -- each its own run) over the network
# forward at the live lane batch of each config, folded by profiles/pmc_fold.py
# into profiles/r6/pmc_tower.json (6x7 "tower16", 9x9 "tower16_9x9") and
# pmc_chess.json ("tower16_rows"), stamped with the build id bench.py matches.
#  - configs[1]: $C4B boards (the dual launch's 96-row tiles of two boards at
#    3 lanes' ~122 live boards; the kernel is tower16_dual_kernel, hence the
#    "tower16_" pattern)
#  - configs[2]: $C5B 9x9 boards (192-row tiles of two boards)
#  - chess: 128 boards through the input-row tower (64-row tiles)
set -o pipefail
C4B=${C4B:-122}
C5B=${C5B:-3443}
R=$PWD
OUT=$R/gpurun_out/r6/pmc${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() {  # run <dir> <script args...> for each counter pass
  local d=$1; shift
  for c in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE:sq"; do
    timeout -s KILL 120 rocprofv3 --pmc ${c%%:*} -d $OUT/$d/${c##*:} -o run --output-format csv -- \
      python3 "$@" > $OUT/${d}_${c##*:}.txt 2>&1 || return 1
  done
}
run c4 $R/profiles/conv_bench.py $C4B 10 0 || exit 1
run c5 $R/profiles/conv_bench.py $C5B 10 0 9 9 || exit 1
run chess $R/profiles/chess_conv_bench.py 128 10 || exit 1
cd $R
python3 profiles/pmc_fold.py $OUT/c4 $C4B tower16_ tower16 > $OUT/pmc_c4.json || exit 1
python3 profiles/pmc_fold.py $OUT/c5 $C5B tower16_ tower16_9x9 "profiles/conv_bench.py (9x9)" > $OUT/pmc_c5.json || exit 1
python3 profiles/pmc_merge.py $OUT/pmc_c4.json $OUT/pmc_c5.json > $OUT/pmc_tower.json || exit 1
python3 profiles/pmc_fold.py $OUT/chess 128 tower16_ tower16_rows profiles/chess_conv_bench.py > $OUT/pmc_chess.json || exit 1
cat $OUT/pmc_tower.json $OUT/pmc_chess.json
