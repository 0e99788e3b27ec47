"""`import krig` compatibility module: the reference's krig surface (krig.py) backed
by the MI355X engine.  See gp2d/krig.py."""
from gp2d.krig import (Krig, Tracks, boundData, getData, getGrid, kriging, laser, predict,  # noqa: F401
                       predictTest, project, radar_grid, rmse, runRestarts, scikit_prior,
                       nad83, x_ori, y_ori)
from gp2d.kern import myKernel, nonDivK, nonRotK  # noqa: F401
