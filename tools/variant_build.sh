#!/bin/bash
# Builds an experimental engine variant: tools/variant_build.sh <name> <hipcc flags...>
# into varlib/var_<name>.so (select it with RCMDYN_LIB=varlib/var_<name>.so, e.g. in
# tools/ab_bench.sh or bench.py).  The sources are copied to a scratch tree first so the
# in-tree objects are untouched.
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
W=/tmp/rcm_var_$name
rm -rf $W && mkdir -p $W/regcm_amd/csrc $W/include
cp regcm_amd/csrc/*.hip regcm_amd/csrc/*.hpp regcm_amd/csrc/Makefile $W/regcm_amd/csrc/
cp include/*.h $W/include/
mkdir -p varlib
# SCHED_NH="<flags>" replaces the Makefile's device-scheduler flags of kernels_nh.hip, SCHED_K those
# of kernels.hip (SCHED_kernels), SCHED_TC those of kernels_nh_tc.hip (k_nh_tend_c)
MV=()
[ -n "${SCHED_NH+x}" ] && MV+=("SCHED_kernels_nh=$SCHED_NH")
[ -n "${SCHED_K+x}" ] && MV+=("SCHED_kernels=$SCHED_K")
[ -n "${SCHED_TC+x}" ] && MV+=("SCHED_kernels_nh_tc=$SCHED_TC")
make -s -C $W/regcm_amd/csrc -j8 HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-function $*" "${MV[@]}"
cp $W/regcm_amd/librcmdyn.so varlib/var_$name.so
echo "built varlib/var_$name.so"
