"""runPredict.py driver (reference runPredict.py:1-49): argv[1] is a 1-based job index;
the first idt0.size jobs predict v, the rest u, with krig.scikit_prior on the
ylim=[1,15], xlim=[-5,15], dx=0.1 window at time tg[idt].

Model inputs: $GP2D_MODEL (the output prefix written by runKrig / krig.kriging) and
hyperparameters $GP2D_HP (comma-separated [var1,lt,ly,lx,(var2,lt,ly,lx,)noise]).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

import krig  # noqa: E402


def main(argv):
    ind = int(argv[1]) - 1
    idt0 = np.arange(8, 24, 4)
    dtg = 0.5
    tg = np.arange(12, 36, dtg)
    if ind >= idt0.size:
        ind = ind - idt0.size
        var = "u"
    else:
        var = "v"
    idt = idt0[ind]
    ylim = [1, 15]
    xlim = [-5, 15]
    dx = float(os.environ.get("GP2D_DX", "0.1"))
    model = os.environ["GP2D_MODEL"]
    hp = [float(v) for v in os.environ.get("GP2D_HP", "1,10,10,10,0.01").split(",")]
    return krig.scikit_prior(model, varname=var, dt=tg[idt], tlim=8, radar="", xlim=xlim, ylim=ylim, dx=dx,
                             HP=hp)


if __name__ == "__main__":
    main(sys.argv)
