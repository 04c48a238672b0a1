#!/bin/bash
# Build the A/B library variants that tools/gpu_r04_v16.sh loads through MSFNO_LIB
# (on the CPU, before the GPU run): each patch under tools/patches/ applied to a clean
# mlp_gen_h.hip, linked as msfno_amd/libmsfno_<name>.so, then the source restored and the
# default library rebuilt.
set -e
cd "$(dirname "$0")/../modulated-spherical-fourier-neural-operator_amd/csrc"
for pair in nopad:mlp_gen_unpadded_stream addw:mlp_gen_addend_exact_waits; do
  name=${pair%%:*}; patch=../../tools/patches/${pair#*:}.patch
  git apply "$patch"
  make -j8 OUT=../msfno_amd/libmsfno_$name.so
  git checkout -- mlp_gen_h.hip
done
make -j8
