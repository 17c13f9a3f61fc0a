set -o pipefail
R=$PWD; OUT=$R/gpurun_out/tree_iso; mkdir -p $OUT; export TMPDIR=/tmp
for lib in prev base; do
  if [ $lib = base ]; then L=$R/custom-alphazero_amd/custom_alphazero/_lib/libaz.so; else L=$R/profiles/ab_libs/prev/libaz.so; fi
  (cd /tmp && AZ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$lib -o run --output-format csv -- python3 $R/profiles/tree_iso.py 2 10 > $OUT/$lib.txt 2>&1) || exit 1
  grep "lanes" $OUT/$lib.txt
  find $OUT/$lib -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | grep -v rocclr | head -6
  find $OUT/$lib -name "*kernel_trace.csv" -delete
done
bash profiles/r2g_check.sh prev base prev base
