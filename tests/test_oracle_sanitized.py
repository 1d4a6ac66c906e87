"""Host sanitizers on the CPU restatement (VERDICT r1 aux): the oracle is rebuilt
with ASan + UBSan (make -C oracle san; any report aborts) and tests/test_oracle.py -- every oracle
entry point against the reference's golden vectors -- runs again on that build in a child process
(ASan must be preloaded into the Python interpreter that dlopens the library)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _libasan():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return None
    path = p.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_oracle_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("gcc's libasan.so is not available")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "san"], check=True)
    san = os.path.join(REPO, "oracle", "_san", "liboracle_san.so")
    env = dict(os.environ, LD_PRELOAD=asan, PMP_ORACLE_LIB=san, OMP_NUM_THREADS="4",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    # the sanitized build is the one loaded
    probe = ("from oracle import oracle as O; O.lib(); "
             "import sys; sys.exit(0 if 'liboracle_san.so' in open('/proc/self/maps').read() else 3)")
    p = subprocess.run([sys.executable, "-c", probe], cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    p = subprocess.run([sys.executable, "-m", "pytest", "tests/test_oracle.py", "-x", "-q", "-m", "not gpu",
                        "-p", "no:cacheprovider"], cwd=REPO, env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
