"""Host AddressSanitizer + UndefinedBehaviorSanitizer run of the C ABI's argument validation
(SURVEY.md §5 'host ASan/UBSan build of the C-ABI shim'): tests/asan/abi_validation.cpp calls
every entry point of include/gp2d.h with malformed arguments (each must return < 0 with a
message, before any device work) and the host-only functions with valid ones.  Runs on a
CPU-only host; the sanitizers instrument the host side only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "asan")


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc and make")
def test_abi_validation_under_asan_ubsan(tmp_path):
    out = str(tmp_path / "build")
    subprocess.run(["make", "-s", f"OUT={out}"], cwd=HERE, check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(out, "abi_validation")], env=env, capture_output=True, text=True, timeout=120)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log
    assert "runtime error" not in log and "AddressSanitizer" not in log, log
    assert " 0 failed" in log
