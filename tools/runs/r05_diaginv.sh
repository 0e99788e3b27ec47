#!/bin/bash
# r05: the diagonal kernel's 32×32 block inverses as two 16×16 substitutions + two 16×16 matrix-core
# products (product) vs the 32-step substitution (tools/_p/libgp2d_inv0.so, the previous commit's
# factor.hpp): phase stamps, fit medians, kernel stats; alternated
set -o pipefail
mkdir -p gpurun_out/r05_diaginv
export TMPDIR=/tmp
for v in st_inv1 st_inv0; do
  GP2D_LIB=tools/_p/libgp2d_$v.so timeout -k 10 300 python3 tools/probe_diag.py 1024 > gpurun_out/r05_diaginv/$v.txt 2>&1 || exit 1
done
for v in prod inv0 prod2 inv0b; do
  lib=2d-gp_amd/gp2d/libgp2d.so; case $v in inv0*) lib=tools/_p/libgp2d_inv0.so;; esac
  GP2D_LIB=$lib timeout -k 10 300 python3 tools/probe_diag.py 4096 1024 16384 > gpurun_out/r05_diaginv/$v.txt 2>&1 || exit 1
done
for v in prod inv0; do
  lib=2d-gp_amd/gp2d/libgp2d.so; [ "$v" = inv0 ] && lib=tools/_p/libgp2d_inv0.so
  GP2D_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r05_diaginv/prof_$v -o run -- \
    python3 tools/probe_diag.py 4096 > gpurun_out/r05_diaginv/prof_$v.txt 2>&1 || exit 1
  find gpurun_out/r05_diaginv/prof_$v -name "*kernel_trace.csv" -delete
done
