"""gp2d — MI355X-native GP-kriging engine (drop-in for rafaelcgon/2D-GP's hot path).

Layers:
  _native   ctypes binding of libgp2d.so (hand-written HIP for gfx950)
  engine    device-resident fit / predict over the C ABI
  kern      the GPy-Kern-style plugin classes (myKernel, nonDivK, nonRotK)
  krig      the reference's krig module surface (Krig, kriging, predict, ...)
  data      index / grid / synthetic-input work (bit-exact with the reference)
  distributed  grid sharding over GPUs, factor broadcast over RCCL
"""
from ._native import NativeLibraryError, GP2DError  # noqa: F401

__version__ = "0.1.0"
