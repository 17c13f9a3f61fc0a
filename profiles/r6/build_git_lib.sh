#!/bin/bash
# Build libaz from a git revision's sources into profiles/ab_libs/<name>/libaz.so
# (A/B against the working tree): build_git_lib.sh <rev> <name>
set -e
rev=$1; name=$2
R=$(cd "$(dirname "$0")/../.." && pwd)
W=/tmp/azgit_$name
rm -rf $W && mkdir -p $W
git -C $R archive $rev custom-alphazero_amd/csrc include | tar x -C $W
mkdir -p $R/profiles/ab_libs/$name
make -s -j8 -C $W/custom-alphazero_amd/csrc OUT=$R/profiles/ab_libs/$name/libaz.so OBJDIR=$W/obj EXTRA="-DAZ_VARIANT_$name" 2>&1 | grep -E "error" -A3 || true
ls -la $R/profiles/ab_libs/$name/libaz.so
