set -o pipefail
mkdir -p gpurun_out/r02s
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "potrf" --timeout 120 --timeout-method thread > gpurun_out/r02s/potrf.log 2>&1 && \
for S in 1 0; do echo "== GP2D_SYRK_SPLIT=$S" >> gpurun_out/r02s/fit.log; GP2D_SYRK_SPLIT=$S timeout -k 10 200 python -u tools/probe_fit.py 4096 16384 >> gpurun_out/r02s/fit.log 2>&1 || exit 1; done && \
timeout -k 10 200 python -u - > gpurun_out/r02s/bitid.log 2>&1 <<'PY'
import os, subprocess, sys
code = r"""
import sys, numpy as np, torch
sys.path[:0]=['.','2d-gp_amd']
from gp2d import data as D, engine as E
x1,x2,u,v=D.synthetic_tracks(4096, seed=2016)
gp=E.fit(E.KernelSpec(kind='df',l_df=5.0), np.stack([x1,x2],1), np.concatenate([u,v]), 0.0025)
np.save(sys.argv[1], gp.W.cpu().numpy()[::7, ::5])
"""
for s in ("1", "0"):
    subprocess.run([sys.executable, "-c", code, f"/tmp/W{s}.npy"], env=dict(os.environ, GP2D_SYRK_SPLIT=s), check=True)
import numpy as np
print("bit-identical:", np.array_equal(np.load("/tmp/W1.npy"), np.load("/tmp/W0.npy")))
PY
