"""Predict-chunk size sweep of the Ozaki path at N = 4096 (dev tool)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "2d-gp_amd"), os.path.join(ROOT, "tools")]
import probe_perf as P
for chunk in (int(c) for c in (sys.argv[1:] or ["8192", "16384", "32768"])):
    P.run(4096, 256, chunk=chunk, variance="ozaki")
