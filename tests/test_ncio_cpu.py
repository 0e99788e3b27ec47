"""NetCDF-3 writer/reader (gp2d.ncio) on CPU.

The reference writes with netCDF4 (printNCFiles.py:5-44, NETCDF3_64BIT); netCDF4 is not
installed here, so conformance is checked against scipy.io.netcdf_file, an independent
classic-format implementation: files written by gp2d.ncio must read back through scipy with
the reference's dimensions, types and values, and scipy-written CDF-1/CDF-2 files must read
through gp2d.ncio.  Values are f4, so comparisons are exact after the float32 cast.
"""
import numpy as np
import pytest
from scipy.io import netcdf_file

from gp2d import ncio


def _grids(nt=3, ny=4, nx=6, seed=0):
    rng = np.random.default_rng(seed)
    T = np.arange(nt) * 0.5
    Y = np.linspace(0, 10, ny)
    X = np.linspace(-5, 5, nx)
    F = [rng.normal(size=(nt, ny, nx)) for _ in range(4)]
    return T, Y, X, F


def test_prediction_file_reads_back_through_scipy(tmp_path):
    T, Y, X, (V, U, VV, UV) = _grids()
    p = str(tmp_path / "pred.nc")
    ncio.write_prediction(p, T, Y, X, V, U, VV, UV, [1.0, 2.0, 3.0, 4.0], [5.0, 6.0, 7.0, 8.0])
    with open(p, "rb") as fh:
        head = fh.read(8)
    assert head[:4] == b"CDF\x02" and int.from_bytes(head[4:8], "big") == 3    # 64-bit offset, 3 records
    with netcdf_file(p, "r", mmap=False) as f:
        assert f.dimensions == {"time": None, "y": 4, "x": 6, "hyperparam": 4}
        for name in ("y", "x", "time", "hyperparam_u", "hyperparam_v", "v", "u", "vvar", "uvar"):
            assert f.variables[name].typecode() == "f"
        assert f.variables["v"].dimensions == ("time", "y", "x")
        for name, a in (("v", V), ("u", U), ("vvar", VV), ("uvar", UV)):
            assert np.array_equal(f.variables[name][:], a.astype(np.float32))
        assert np.array_equal(f.variables["time"][:], T.astype(np.float32))
        assert np.array_equal(f.variables["y"][:], Y.astype(np.float32))
        assert np.array_equal(f.variables["hyperparam_u"][:], np.float32([5, 6, 7, 8]))


def test_partial_records_hold_fill_values(tmp_path):
    T, Y, X, (V, U, _, _) = _grids(nt=3)
    p = str(tmp_path / "part.nc")
    ncio.createNC(p, T, Y, X, [0.0])
    with ncio.openNC(p, "a") as f:
        ncio.writeNC(f, "v", V[:2])
    d = ncio.readNC(p)
    assert d["v"].shape == (3, 4, 6)
    assert np.array_equal(d["v"][:2], V[:2].astype(np.float32))
    assert np.all(d["v"][2] == np.float32(9.9692099683868690e36))
    assert np.all(d["u"] == np.float32(9.9692099683868690e36))
    with netcdf_file(p, "r", mmap=False) as f:
        assert np.array_equal(f.variables["v"][:2], V[:2].astype(np.float32))


def test_append_mode_keeps_other_variables(tmp_path):
    T, Y, X, (V, U, VV, UV) = _grids()
    p = str(tmp_path / "app.nc")
    ncio.write_prediction(p, T, Y, X, V, U, VV, UV, [1.0], [2.0])
    with ncio.openNC(p, "a") as f:
        ncio.writeNC(f, "u", 2 * U)
    d = ncio.readNC(p)
    assert np.array_equal(d["u"], (2 * U).astype(np.float32))
    assert np.array_equal(d["v"], V.astype(np.float32))


@pytest.mark.parametrize("version", [1, 2])
def test_reads_scipy_written_files(tmp_path, version):
    p = str(tmp_path / f"s{version}.nc")
    rng = np.random.default_rng(version)
    a = rng.normal(size=(5, 3)).astype(np.float32)
    b = rng.integers(-100, 100, size=7).astype(np.int32)
    r = rng.normal(size=(2, 5)).astype(np.float64)
    with netcdf_file(p, "w", version=version) as f:
        f.history = "made by scipy"
        f.createDimension("t", None)
        f.createDimension("i", 5)
        f.createDimension("j", 3)
        f.createDimension("k", 7)
        va = f.createVariable("a", "f", ("i", "j"))
        va[:] = a
        va.units = "m/s"
        f.createVariable("b", "i", ("k",))[:] = b
        f.createVariable("r", "d", ("t", "i"))[:] = r
    with ncio.NCFile(p, "r") as g:
        assert g.version == version and g.numrecs == 2
        assert g.attributes["history"] == "made by scipy"
        assert g.variables["a"].attributes["units"] == "m/s"
        assert np.array_equal(g.variables["a"].data, a)
        assert np.array_equal(g.variables["b"].data, b)
        assert np.array_equal(g.variables["r"].data, r)


def test_own_attributes_and_types_roundtrip(tmp_path):
    p = str(tmp_path / "t.nc")
    with ncio.NCFile(p, "w") as f:
        f.attributes["title"] = "gp2d"
        f.createDimension("n", 3)
        f.createDimension("rec", None)
        v = f.createVariable("d", "f8", ("n",))
        v[:] = [1.5, 2.5, 3.5]
        v.attributes["scale"] = np.array([2.0])
        f.createVariable("s", "i2", ("rec", "n"))[0:2] = [[1, 2, 3], [4, 5, 6]]
    with netcdf_file(p, "r", mmap=False) as f:
        assert f.title == b"gp2d"
        assert np.array_equal(f.variables["d"][:], [1.5, 2.5, 3.5])
        assert f.variables["d"].scale == 2.0
        assert np.array_equal(f.variables["s"][:], [[1, 2, 3], [4, 5, 6]])


def _write_radar(path, lon, lat, xc, yc, t_days):
    """A synthetic HF-radar file with the variables krig.scikit_prior reads (krig.py:99-108)."""
    with ncio.NCFile(path, "w") as f:
        f.createDimension("two", 2)
        f.createDimension("x", xc.size)
        f.createDimension("y", yc.size)
        f.createDimension("time", None)
        f.createVariable("imageOriginPosition", "f8", ("two",))[:] = np.array([lon, lat])
        f.createVariable("xCoords", "f8", ("x",))[:] = xc
        f.createVariable("yCoords", "f8", ("y",))[:] = yc
        f.createVariable("time", "f8", ("time",))[:] = np.array([t_days])
        f.createVariable("ux", "f4", ("time", "y", "x"))[:] = np.zeros((1, yc.size, xc.size), np.float32)
        f.createVariable("uy", "f4", ("time", "y", "x"))[:] = np.zeros((1, yc.size, xc.size), np.float32)


def test_radar_grid_branch(tmp_path):
    """scikit_prior's radar grid (krig.py:98-118) from a radar NetCDF written here: origin
    projected (the documented NAD83 stand-in) and shifted to the drifter frame in km, xCoords /
    yCoords in m, time in days since 2016-01-01 → hours since 2016-02-07 02:15, meshgrid
    (yg, tg, xg) flattening."""
    import krig as K
    from datetime import datetime, timedelta
    p = str(tmp_path / "radar.nc")
    xc = np.arange(0.0, 9000.0, 1500.0)
    yc = np.arange(-2000.0, 4000.0, 1000.0)
    _write_radar(p, -88.5, 28.9, xc, yc, 37.25)
    X, tg, yg, xg = K.radar_grid(p)
    x0, y0 = K.nad83(-88.5, 28.9)
    assert np.allclose(xg, (x0 - K.x_ori) / 1000.0 + xc / 1000.0, rtol=0, atol=1e-12)
    assert np.allclose(yg, (y0 - K.y_ori) / 1000.0 + yc / 1000.0, rtol=0, atol=1e-12)
    hours = (datetime(2016, 1, 1) + timedelta(37.25) - datetime(2016, 2, 7, 2, 15)).total_seconds() / 3600
    assert tg.shape == (1,) and tg[0] == hours
    assert X.shape == (yg.size * xg.size, 3) and np.all(X[:, 0] == hours)
    assert np.array_equal(X[:xg.size, 2], xg) and np.all(X[:xg.size, 1] == yg[0])
