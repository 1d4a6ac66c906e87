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


def declared_prototypes():
    """name -> list of parameter type strings, from include/pmp.h."""
    src = open(os.path.join(REPO, "include", "pmp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(pmp_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", src, flags=re.S):
        params = [p.strip() for p in m.group(2).replace("\n", " ").split(",")]
        protos[m.group(1)] = [] if params == ["void"] or params == [""] else params
    return protos


def test_bindings_match_prototypes():
    """Every ctypes binding has exactly the declared arity, and pointer / 64-bit integer parameters
    are bound as c_void_p / c_int64 (an under-length argtypes list silently truncates the extra
    pointer arguments to C int)."""
    import ctypes

    from python_motion_planning_amd import _lib

    protos = declared_prototypes()
    assert protos
    for name, params in protos.items():
        res, args = _lib.SIGNATURES[name]
        assert len(args) == len(params), f"{name}: {len(args)} bound vs {len(params)} declared"
        for a, p in zip(args, params):
            if "*" in p:
                assert a in (ctypes.c_void_p, ctypes.c_char_p), f"{name}: {p!r} bound as {a}"
            elif p.startswith("int64_t"):
                assert a is ctypes.c_int64, f"{name}: {p!r} bound as {a}"
            elif p.startswith("int") or p.startswith("int32_t"):
                assert a is ctypes.c_int, f"{name}: {p!r} bound as {a}"


def test_single_query_capacity_without_gpu():
    """pmp_astar2d_sq_cap is host arithmetic (no device call): (160 KiB - 256 B) / 12 B per entry,
    a multiple of 16, on grids too large for the engine's LDS grid block; less beside a small grid."""
    from python_motion_planning_amd import _lib

    L = _lib.load_library()
    assert L.pmp_astar2d_sq_cap(1400, 1400) == 13632 == ((160 * 1024 - 256) // 12) & ~15
    assert 0 < L.pmp_astar2d_sq_cap(51, 31) < 13632
