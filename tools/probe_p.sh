#!/bin/bash
# Accuracy vs operand precision of the Ozaki engine (dev): builds libgp2d with
# -DGP2D_OZ_PW=<pW> -DGP2D_OZ_PB=<pB> into tools/_p/ for each "pW:pB" argument;
# tools/probe_accuracy.py is then run against each (GP2D_LIB=tools/_p/libgp2d_<pW>_<pB>.so).
set -euo pipefail
mkdir -p tools/_p
for pp in "$@"; do
  pw=${pp%:*}; pb=${pp#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value \
    -DGP2D_OZ_PW=$pw -DGP2D_OZ_PB=$pb -o tools/_p/libgp2d_${pw}_${pb}.so 2d-gp_amd/csrc/gp2d.hip &
done
wait
