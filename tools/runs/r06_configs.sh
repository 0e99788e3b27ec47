#!/bin/bash
# r06: the BASELINE configs B and D at HEAD (C and E: r06_parity.sh)
set -o pipefail
R=gpurun_out/r06_configs
mkdir -p $R
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --config B --f64-steps 0 --dropin-steps 0 > $R/config_B.json 2> $R/config_B.err && \
timeout -k 10 600 python -u bench.py --config D --f64-steps 0 --dropin-steps 0 > $R/config_D.json 2> $R/config_D.err
