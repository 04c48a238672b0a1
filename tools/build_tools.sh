#!/bin/bash
# Builds the microbenchmarks under tools/bin against the in-tree libmsfno.so
set -e
cd "$(dirname "$0")/.."
CS=modulated-spherical-fourier-neural-operator_amd/csrc
LIB=modulated-spherical-fourier-neural-operator_amd/msfno_amd
mkdir -p tools/bin
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-value -Wno-unused-result -I $CS tools/gemm_x6_bench.hip \
  -L $LIB -lmsfno -Wl,-rpath,'$ORIGIN/../../'$LIB -o tools/bin/gemm_x6_bench
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -Wno-unused-result -I $CS tools/corun_probe.cpp \
  -L $LIB -lmsfno -Wl,-rpath,'$ORIGIN/../../'$LIB -o tools/bin/corun_probe
python3 tools/gen_pk_opsel_sweep.py tools/bin/pk_opsel_sweep.cpp
/opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 -std=c++17 tools/bin/pk_opsel_sweep.cpp -o tools/bin/pk_opsel_sweep
