#!/bin/bash
# Build an A/B variant of libaz from the product sources plus a patch script
# (profiles/r6/variants/<name>.py: string replacements on a copy of csrc/),
# into profiles/ab_libs/<name>/libaz.so (git-ignored; travels with gpurun and
# loads through AZ_LIB_PATH).  The product sources never carry the variant.
set -e
name=$1
R=$(cd "$(dirname "$0")/../.." && pwd)
W=/tmp/azvar_$name
rm -rf $W && mkdir -p $W/csrc $W/include
cp -p $R/custom-alphazero_amd/csrc/*.hip $R/custom-alphazero_amd/csrc/*.h $R/custom-alphazero_amd/csrc/*.py $R/custom-alphazero_amd/csrc/Makefile $W/csrc/
cp $R/include/*.h $W/include/
# the Makefile includes ../../include: mirror the layout
mkdir -p $W/x && mv $W/csrc $W/x/csrc && mv $W/include $W/include_tmp && mkdir -p $W/include && mv $W/include_tmp/* $W/include/ && rmdir $W/include_tmp
(cd $W/x/csrc && python3 $R/profiles/r6/variants/$name.py)
mkdir -p $R/profiles/ab_libs/$name
make -s -j8 -C $W/x/csrc OUT=$R/profiles/ab_libs/$name/libaz.so OBJDIR=$W/obj EXTRA="-DAZ_VARIANT_$name" 2>&1 | grep -E "error" -A3 || true
ls -la $R/profiles/ab_libs/$name/libaz.so
