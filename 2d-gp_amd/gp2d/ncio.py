"""NetCDF-3 output of the kriging products.

Mirrors printNCFiles.createNC / writeNC (printNCFiles.py:5-44) and the write sequence of
krig.predict (krig.py:559-570): a NETCDF3_64BIT (CDF-2) file with

  dimensions  time (unlimited), y, x, hyperparam
  variables   y(y), x(x), time(time), hyperparam_u(hyperparam), hyperparam_v(hyperparam),
              v, u, vvar, uvar (time, y, x) — all 'f4'

netCDF4 (the reference's dependency) is not installed in this image, so this module is a
small self-contained implementation of the classic format (CDF-1 read, CDF-2 read/write):
big-endian header of dimension / attribute / variable lists, non-record variables, then
the records (one vsize slab per record variable per record).  Unwritten record entries
hold the NetCDF default fill values, as netCDF4 would leave them.  The file is rewritten
whole on close — the products are a few MB (grid × time × 4 fields of f4).
"""
from __future__ import annotations

import struct

import numpy as np

_DIM, _VAR, _ATT = 10, 11, 12
# nc_type codes, big-endian numpy dtypes and default fill values (netcdf.h NC_FILL_*)
_TYPES = {
    1: (">i1", -127), 2: ("S1", b"\x00"), 3: (">i2", -32767), 4: (">i4", -2147483647),
    5: (">f4", 9.9692099683868690e36), 6: (">f8", 9.9692099683868690e36),
}
_CODES = {"i1": 1, "b": 1, "c": 2, "S1": 2, "i2": 3, "h": 3, "i4": 4, "i": 4, "f4": 5, "f": 5, "f8": 6, "d": 6}
GRID_VARS = ("v", "u", "vvar", "uvar")


def _pad4(n: int) -> int:
    return (n + 3) & ~3


class _Reader:
    def __init__(self, buf: bytes):
        self.b, self.o = buf, 0

    def take(self, n: int) -> bytes:
        s = self.b[self.o:self.o + n]
        if len(s) != n:
            raise ValueError("truncated NetCDF file")
        self.o += n
        return s

    def i4(self) -> int:
        return struct.unpack(">i", self.take(4))[0]

    def u4(self) -> int:
        return struct.unpack(">I", self.take(4))[0]

    def i8(self) -> int:
        return struct.unpack(">q", self.take(8))[0]

    def name(self) -> str:
        n = self.i4()
        s = self.take(_pad4(n))[:n]
        return s.decode("utf-8")


class Variable:
    """A variable of an NCFile; numpy-style slicing, growing along the record dimension."""

    def __init__(self, f: "NCFile", name: str, code: int, dims: tuple, attrs=None, data=None):
        self._f, self.name, self.code, self.dimensions = f, name, code, tuple(dims)
        self.attributes = dict(attrs or {})
        dt, fill = _TYPES[code]
        shape = tuple(f._dimlen(d) for d in self.dimensions)
        self.data = data if data is not None else np.full(shape, fill, dtype=dt)

    @property
    def isrec(self) -> bool:
        return bool(self.dimensions) and self._f.dimensions[self.dimensions[0]] is None

    @property
    def shape(self):
        return self.data.shape

    def _stop(self, key):
        k = key[0] if isinstance(key, tuple) else key
        if isinstance(k, slice):
            if k.stop is None:
                return None
            return k.stop
        if isinstance(k, (int, np.integer)):
            return int(k) + 1
        return None

    def __setitem__(self, key, value):
        if self.isrec:
            stop = self._stop(key)
            if stop is None:   # [:] on a record variable: the value's leading extent
                stop = np.shape(value)[0] if np.ndim(value) else self._f.numrecs
            self._f._grow(stop)
        self.data[key] = value

    def __getitem__(self, key):
        return self.data[key]

    def __len__(self):
        return self.data.shape[0] if self.data.ndim else 1


class NCFile:
    """Minimal netCDF classic-format file: mode 'r', 'w' (CDF-2) or 'a' (read, modify, rewrite)."""

    def __init__(self, path: str, mode: str = "r", version: int = 2):
        if mode not in ("r", "w", "a"):
            raise ValueError("mode must be 'r', 'w' or 'a'")
        self.path, self.mode, self.version = path, mode, int(version)
        self.dimensions: dict = {}          # name -> length (None = unlimited)
        self.variables: dict = {}
        self.attributes: dict = {}
        self.numrecs = 0
        self._closed = False
        if mode in ("r", "a"):
            with open(path, "rb") as fh:
                self._parse(fh.read())

    # -------------------------------------------------------------- structure
    def _dimlen(self, name):
        n = self.dimensions[name]
        return self.numrecs if n is None else n

    def createDimension(self, name: str, size):
        if size is None and any(v is None for v in self.dimensions.values()):
            raise ValueError("only one unlimited dimension is allowed")
        self.dimensions[name] = None if size is None else int(size)

    def createVariable(self, name: str, datatype: str, dimensions) -> Variable:
        if isinstance(dimensions, str):
            dimensions = (dimensions,)
        dims = tuple(dimensions)
        for i, d in enumerate(dims):
            if d not in self.dimensions:
                raise KeyError(f"unknown dimension {d!r}")
            if self.dimensions[d] is None and i != 0:
                raise ValueError("the unlimited dimension must come first")
        v = Variable(self, name, _CODES[datatype], dims)
        self.variables[name] = v
        return v

    def _grow(self, nrec: int):
        if nrec <= self.numrecs:
            return
        for v in self.variables.values():
            if v.isrec:
                dt, fill = _TYPES[v.code]
                ext = np.full((nrec - v.data.shape[0],) + v.data.shape[1:], fill, dtype=dt)
                v.data = np.concatenate([v.data, ext], 0)
        self.numrecs = nrec

    # -------------------------------------------------------------- reading
    def _atts(self, r: _Reader) -> dict:
        tag, n = r.i4(), r.i4()
        if tag == 0:
            return {}
        if tag != _ATT:
            raise ValueError("bad attribute list")
        out = {}
        for _ in range(n):
            name = r.name()
            code, cnt = r.i4(), r.i4()
            dt, _ = _TYPES[code]
            size = np.dtype(dt).itemsize * cnt
            raw = r.take(_pad4(size))[:size]
            out[name] = raw.decode("utf-8") if code == 2 else np.frombuffer(raw, dtype=dt).copy()
        return out

    def _parse(self, buf: bytes):
        r = _Reader(buf)
        magic = r.take(4)
        if magic[:3] != b"CDF" or magic[3] not in (1, 2):
            raise ValueError("not a netCDF classic (CDF-1/CDF-2) file")
        self.version = magic[3]
        off = r.i4 if self.version == 1 else r.i8
        nrec = r.u4()
        tag, n = r.i4(), r.i4()
        dnames = []
        if tag == _DIM:
            for _ in range(n):
                name = r.name()
                ln = r.i4()
                self.dimensions[name] = None if ln == 0 else ln
                dnames.append(name)
        self.attributes = self._atts(r)
        tag, n = r.i4(), r.i4()
        specs = []
        if tag == _VAR:
            for _ in range(n):
                name = r.name()
                nd = r.i4()
                dims = tuple(dnames[r.i4()] for _ in range(nd))
                atts = self._atts(r)
                code, vsize, begin = r.i4(), r.i4(), off()
                specs.append((name, dims, atts, code, vsize, begin))
        self.numrecs = 0 if nrec == 0xFFFFFFFF else nrec
        recvars = [s for s in specs if s[1] and self.dimensions[s[1][0]] is None]
        recsize = sum(s[4] for s in recvars)
        if len(recvars) == 1:   # a lone record variable is stored without padding
            s = recvars[0]
            recsize = int(np.prod([self.dimensions[d] for d in s[1][1:]], dtype=np.int64)) * \
                np.dtype(_TYPES[s[3]][0]).itemsize
        for name, dims, atts, code, vsize, begin in specs:
            dt = np.dtype(_TYPES[code][0])
            isrec = bool(dims) and self.dimensions[dims[0]] is None
            inner = tuple(self.dimensions[d] for d in (dims[1:] if isrec else dims))
            count = int(np.prod(inner, dtype=np.int64))
            if isrec:
                rows = [np.frombuffer(buf, dtype=dt, count=count, offset=begin + i * recsize)
                        for i in range(self.numrecs)]
                data = (np.stack(rows) if rows else np.zeros((0,) + inner, dt)).reshape((self.numrecs,) + inner)
            else:
                data = np.frombuffer(buf, dtype=dt, count=count, offset=begin).reshape(inner)
            self.variables[name] = Variable(self, name, code, dims, atts, data.copy())

    # -------------------------------------------------------------- writing
    @staticmethod
    def _name(s: str) -> bytes:
        b = s.encode("utf-8")
        return struct.pack(">i", len(b)) + b + b"\x00" * (_pad4(len(b)) - len(b))

    def _att_bytes(self, atts: dict) -> bytes:
        if not atts:
            return struct.pack(">ii", 0, 0)
        out = [struct.pack(">ii", _ATT, len(atts))]
        for k, v in atts.items():
            if isinstance(v, str):
                code, raw, cnt = 2, v.encode("utf-8"), len(v.encode("utf-8"))
            else:
                a = np.atleast_1d(np.asarray(v))
                code = 6 if a.dtype.kind == "f" else 4
                raw = a.astype(_TYPES[code][0]).tobytes()
                cnt = a.size
            out.append(self._name(k) + struct.pack(">ii", code, cnt) + raw + b"\x00" * (_pad4(len(raw)) - len(raw)))
        return b"".join(out)

    def _serialize(self) -> bytes:
        dnames = list(self.dimensions)
        vars_ = list(self.variables.values())
        recvars = [v for v in vars_ if v.isrec]

        def inner_bytes(v):
            dims = v.dimensions[1:] if v.isrec else v.dimensions
            n = int(np.prod([self.dimensions[d] for d in dims], dtype=np.int64))
            return n * np.dtype(_TYPES[v.code][0]).itemsize

        vsizes = {v.name: _pad4(inner_bytes(v)) for v in vars_}
        if len(recvars) == 1:
            vsizes[recvars[0].name] = inner_bytes(recvars[0])
        offw = 4 if self.version == 1 else 8

        def header(begins):
            h = [b"CDF" + bytes([self.version]), struct.pack(">I", self.numrecs)]
            if dnames:
                h.append(struct.pack(">ii", _DIM, len(dnames)))
                for d in dnames:
                    h.append(self._name(d) + struct.pack(">i", self.dimensions[d] or 0))
            else:
                h.append(struct.pack(">ii", 0, 0))
            h.append(self._att_bytes(self.attributes))
            if vars_:
                h.append(struct.pack(">ii", _VAR, len(vars_)))
                for v in vars_:
                    h.append(self._name(v.name) + struct.pack(">i", len(v.dimensions)))
                    h.append(b"".join(struct.pack(">i", dnames.index(d)) for d in v.dimensions))
                    h.append(self._att_bytes(v.attributes))
                    h.append(struct.pack(">ii", v.code, min(vsizes[v.name], 2 ** 31 - 1)))
                    h.append(struct.pack(">i" if offw == 4 else ">q", begins.get(v.name, 0)))
            else:
                h.append(struct.pack(">ii", 0, 0))
            return b"".join(h)

        pos = len(header({}))
        begins = {}
        for v in vars_:
            if not v.isrec:
                begins[v.name] = pos
                pos += vsizes[v.name]
        for v in recvars:
            begins[v.name] = pos
            pos += vsizes[v.name]
        out = [header(begins)]
        for v in vars_:
            if not v.isrec:
                raw = np.ascontiguousarray(v.data, dtype=_TYPES[v.code][0]).tobytes()
                out.append(raw + b"\x00" * (vsizes[v.name] - len(raw)))
        for r in range(self.numrecs):
            for v in recvars:
                raw = np.ascontiguousarray(v.data[r], dtype=_TYPES[v.code][0]).tobytes()
                out.append(raw + b"\x00" * (vsizes[v.name] - len(raw)))
        return b"".join(out)

    def close(self):
        if self._closed:
            return
        self._closed = True
        if self.mode in ("w", "a"):
            with open(self.path, "wb") as fh:
                fh.write(self._serialize())

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ------------------------------------------------------------------ reference API
def createNC(outFile, T, Y, X, hyp):
    """printNCFiles.createNC (printNCFiles.py:5-34): dimensions, coordinate variables and the
    (time, y, x) fields; hyp sizes the hyperparam dimension (values come with writeNC)."""
    T, Y, X = (np.atleast_1d(np.squeeze(np.asarray(a, dtype=np.float64))) for a in (T, Y, X))
    with NCFile(outFile, "w", version=2) as f:          # NETCDF3_64BIT
        f.createDimension("time", None)
        f.createDimension("y", Y.size)
        f.createDimension("x", X.size)
        f.createDimension("hyperparam", int(np.size(hyp)))
        f.createVariable("y", "f4", ("y",))[:] = Y
        f.createVariable("x", "f4", ("x",))[:] = X
        times = f.createVariable("time", "f4", ("time",))
        f.createVariable("hyperparam_u", "f4", ("hyperparam",))
        f.createVariable("hyperparam_v", "f4", ("hyperparam",))
        for name in GRID_VARS:
            f.createVariable(name, "f4", ("time", "y", "x"))
        times[:] = T


def openNC(outFile, mode="a") -> NCFile:
    """netCDF4.Dataset(outFile, 'a') in krig.py:566."""
    return NCFile(outFile, mode)


def writeNC(f: NCFile, varname, data):
    """printNCFiles.writeNC (printNCFiles.py:37-44): data[0:NT] into a 1-D or (time, y, x) variable."""
    data = np.asarray(data)
    NT = np.size(data, 0)
    var = f.variables[varname]
    if len(var.dimensions) == 1:
        var[0:NT] = data
    elif len(var.dimensions) == 3:
        var[0:NT, :, :] = data
    return f


def write_prediction(outFile, T, Y, X, V, U, VVar, UVar, hyp_v, hyp_u):
    """krig.predict's output sequence (krig.py:559-570) in one call."""
    createNC(outFile, T, Y, X, hyp_v)
    with openNC(outFile, "a") as f:
        for name, arr in (("v", V), ("u", U), ("vvar", VVar), ("uvar", UVar)):
            writeNC(f, name, arr)
        writeNC(f, "hyperparam_v", np.atleast_1d(hyp_v))
        writeNC(f, "hyperparam_u", np.atleast_1d(hyp_u))


def readNC(path) -> dict:
    """All variables of a classic-format file as numpy arrays."""
    with NCFile(path, "r") as f:
        return {k: np.asarray(v.data) for k, v in f.variables.items()}
