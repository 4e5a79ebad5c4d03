#!/bin/bash
# Experiment builds of the ICP pass (never shipped): build/exp/lib_<name>.so, selected with R360_LIB.
#   base     the shipped source
#   nogather target gathers replaced by values derived from the index (compute + source stream only)
#   noacc    residual / Jacobian / JtJ math replaced by a trivial sum (projection + memory only)
# usage: tools/exp_variants.sh [name ...]      (CPU; hipcc cross-compiles)
set -e
cd "$(dirname "$0")/../rgbd360_amd/csrc"
make -s -j8
OUT=../lib/exp; mkdir -p $OUT
OBJS=$(ls ../../build/obj/*.o | grep -v k_icp_kernels.o | grep -v k_icp_stamps.o)
for v in ${@:-base nogather noacc}; do
  case $v in base) D="";; minb6) D="-DR360_ICP_MINB=6";; minb4) D="-DR360_ICP_MINB=4";; nogather) D="-DR360_EXP_NOGATHER";; noacc) D="-DR360_EXP_NOACC";; both) D="-DR360_EXP_NOGATHER -DR360_EXP_NOACC";; nokt) D="-DR360_EXP_NOKT";; nodrain) D="-DR360_EXP_NODRAIN";; noloop) D="-DR360_EXP_NOLOOP";; tpb256) D="-DR360_ICP_TPB=256";; w5) D="-DR360_ICP_MINB=5";; t1024) D="-DR360_ICP_TPB=1024";; tpb512) D="-DR360_ICP_TPB=512";; norec) D="-DR360_EXP_NOLOOP -DR360_EXP_NOREC";; noepi) D="-DR360_EXP_NOLOOP -DR360_EXP_NOEPI";; nobfly) D="-DR360_EXP_NOLOOP -DR360_EXP_NOBFLY";; bothnokt) D="-DR360_EXP_NOGATHER -DR360_EXP_NOACC -DR360_EXP_NOKT";; *) D="$EXPFLAGS";; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -fno-slp-vectorize $D -c kernels/icp_kernels.hip -o $OUT/icp_$v.o &
done
wait
for v in ${@:-base nogather noacc}; do
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fopenmp -Wl,-rpath,/opt/rocm/llvm/lib -Wl,-rpath,/opt/rocm/lib -lz $OBJS $OUT/icp_$v.o -o $OUT/lib_$v.so
done
rm -f $OUT/*.o
ls -la $OUT/*.so
