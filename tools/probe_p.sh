#!/bin/bash
# Accuracy vs operand precision p of the Ozaki engine (dev): builds libgp2d with
# -DGP2D_OZ_P=<p> into tools/_p/ and runs tools/probe_accuracy.py against each.
set -euo pipefail
mkdir -p tools/_p
for p in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value \
    -DGP2D_OZ_P=$p -o tools/_p/libgp2d_p$p.so 2d-gp_amd/csrc/gp2d.hip
done
