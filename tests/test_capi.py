"""The C-ABI library loads (no GPU needed) and exports every symbol include/pmp.h declares."""
import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(REPO, "include", "pmp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pmp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from python_motion_planning_amd import _lib

    L = _lib.load_library()
    names = declared_symbols()
    assert "pmp_astar2d_batch" in names
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, f"{n} declared in pmp.h but not bound in _lib.SIGNATURES"
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (pmp_[a-z0-9_]+)", out))
    assert set(names) <= exported


def test_version_string_without_gpu():
    from python_motion_planning_amd import _lib

    assert b"gfx950" in _lib.load_library().pmp_version()


def test_kernels_are_gfx950_code_objects():
    from python_motion_planning_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"__CLANG_OFFLOAD_BUNDLE__" in data  # .hip_fatbin offload bundle
    assert b"amdgcn-amd-amdhsa--gfx950" in data
