"""runKrig.py driver (reference runKrig.py:1-37): argv[1] is a 1-based job-array index
into the (T, dt, skip, nK) tables; builds the model with krig.kriging.

Data: the reference reads Filtered_2016_2_7.pkl; here tracks come from the .npz given
by $GP2D_TRACKS (fields time, lat, lon, u, v) or, if unset, the seeded synthetic
drifters of krig.Tracks.synthetic().
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import krig  # noqa: E402

T = np.array([1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1])
dt = np.array([1, 1, 2, 2, 2, 1, 1, 2, 2, 2, 1, 1, 2, 2, 2])
skp = np.array([1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3])
nK = np.array([1, 2, 1, 2, 3, 1, 2, 1, 2, 3, 1, 2, 1, 2, 3])


def main(argv):
    ind = int(argv[1]) - 1
    kernel_type = int(os.environ.get("GP2D_KERNEL_TYPE", "2"))
    st = 0
    et = st + T[ind] * 24 * 60 // 15
    out_dir = os.environ.get("GP2D_OUT", "skip_" + str(skp[ind]))
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, "rbfModel_T" + str(T[ind]) + "_dt" + str(dt[ind]) + "_nK" + str(nK[ind]))
    path = os.environ.get("GP2D_TRACKS")
    tracks = krig.Tracks.load(path) if path else krig.Tracks.synthetic()
    krig.kriging(st, et, sample_step=-dt[ind], skip=skp[ind], nKernels=nK[ind], output=out,
                 kernelType=kernel_type, tracks=tracks)
    return out


if __name__ == "__main__":
    main(sys.argv)
