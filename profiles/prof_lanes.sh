set -e
R=$PWD
export TMPDIR=/tmp
for l in 1 2 3; do
  OUT=$R/gpurun_out/trace_l$l
  mkdir -p $OUT
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-cache-window --steps 3 --warmup 10 --lanes $l > $OUT/b.json 2> $OUT/err.txt)
  f=$(find $OUT -name "*kernel_trace.csv" | head -1)
  echo "lanes=$l"; python3 $R/profiles/busy.py $f 0.3
done
