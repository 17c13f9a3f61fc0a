#!/bin/bash
# Round-5 PMC + trace collection for the benched build (repo root, under gpurun):
#  1. kernel trace + stats of a short bench.py run (its HIP-event avg_launch_ms
#     must agree with rocprof's average for tower16_kernel)
#  3. the same passes at configs[2]'s 9x9 batch (key tower16_9x9, merged into
#     pmc_tower.json) and over the chess forward (profiles/chess_conv_bench.py,
#     128 boards) -> profiles/r5/pmc_chess.json [tower16_rows]
#  2. PMC passes over az_forward at the live lane batch ($C4B boards: configs[1] on 3 lanes): FETCH_SIZE,
#     WRITE_SIZE, then MFMA busy (each its own pass) -> profiles/r5/pmc_tower.json,
#     stamped with the build id bench.py matches
set -o pipefail
C4B=${C4B:-456}
R=$PWD
OUT=$R/gpurun_out/prof_r5${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --no-cpu-baseline --no-cache-window > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc/fetch -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py $C4B 10 0 > $OUT/pmc_fetch.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc/write -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py $C4B 10 0 > $OUT/pmc_write.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $OUT/pmc/sq -o run --output-format csv -- \
  python3 $R/profiles/conv_bench.py $C4B 10 0 > $OUT/pmc_sq.txt 2>&1 || exit 1
# configs[2]: 9x9 boards (192-row tiles, two boards each) at its live lane batch
for c in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE:sq"; do
  timeout -s KILL 120 rocprofv3 --pmc ${c%%:*} -d $OUT/pmc_9x9/${c##*:} -o run --output-format csv -- \
    python3 $R/profiles/conv_bench.py 3443 10 0 9 9 > $OUT/pmc_9x9_${c##*:}.txt 2>&1 || exit 1
done
# chess: the input-row tower at the self-play lane batch (128 boards, 64-row tiles)
for c in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE:sq"; do
  timeout -s KILL 120 rocprofv3 --pmc ${c%%:*} -d $OUT/pmc_chess/${c##*:} -o run --output-format csv -- \
    python3 $R/profiles/chess_conv_bench.py 128 10 > $OUT/pmc_chess_${c##*:}.txt 2>&1 || exit 1
done
cd $R
python3 profiles/pmc_fold.py $OUT/pmc $C4B tower16_kernel tower16 > $OUT/pmc_tower.json || exit 1
python3 profiles/pmc_fold.py $OUT/pmc_9x9 3443 tower16_kernel tower16_9x9 "profiles/conv_bench.py (9x9)" > $OUT/pmc_9x9.json || exit 1
python3 profiles/pmc_merge.py $OUT/pmc_tower.json $OUT/pmc_9x9.json > $OUT/pmc_tower_all.json || exit 1
mv $OUT/pmc_tower_all.json $OUT/pmc_tower.json
python3 profiles/pmc_fold.py $OUT/pmc_chess 128 tower16_kernel tower16_rows profiles/chess_conv_bench.py > $OUT/pmc_chess.json || exit 1
cat $OUT/pmc_chess.json
python3 profiles/summarize.py $OUT r5 > $OUT/summary.md 2>&1
find $OUT -name "*kernel_trace.csv" -size +20M -delete
cat $OUT/pmc_tower.json
tail -30 $OUT/summary.md
