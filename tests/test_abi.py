"""CPU checks of the C-ABI library: it loads, exports every symbol include/bf/bf.h declares,
and the ctypes struct layouts match the header's static_asserts. No GPU calls."""
import ctypes as C
import os
import subprocess

import bundlefusion_amd as bfa
from bundlefusion_amd import abi


def test_library_exists_and_loads():
    assert os.path.exists(abi.LIB_PATH)
    L = bfa.lib()
    assert L.bf_abi_version() == abi.ABI_VERSION == 4


def test_every_declared_symbol_is_exported():
    names = abi.header_functions()
    assert len(names) >= 30
    L = C.CDLL(abi.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_exported_symbols_have_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", abi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for n in abi.header_functions():
        assert n in exported, n


def test_struct_layouts():
    assert C.sizeof(abi.BFHashParams) == 224
    assert C.sizeof(abi.BFDepthCameraParams) == 32
    assert C.sizeof(abi.BFRayCastParams) == 192
    assert abi.HASH_ENTRY_DTYPE.itemsize == 32
    assert abi.VOXEL_DTYPE.itemsize == 12
    assert abi.ENTRYJ_DTYPE.itemsize == 32


def test_struct_sizes_match_the_library():
    """Every ctypes mirror has the size the C++ compiler gives the struct (bf_abi_struct_size)."""
    import bundlefusion_amd as bfa
    L = bfa.lib()
    checked = 0
    for name in dir(abi):
        cls = getattr(abi, name)
        if not (name.startswith("BF") and isinstance(cls, type) and issubclass(cls, C.Structure)):
            continue
        n = C.c_size_t()
        rc = L.bf_abi_struct_size(name.encode(), C.byref(n))
        if rc != 0:
            continue  # a Python-only helper struct
        assert C.sizeof(cls) == n.value, (name, C.sizeof(cls), n.value)
        checked += 1
    assert checked >= 26  # every BF* struct of the header that the bindings mirror


def test_error_path_without_device():
    """A null handle returns an error status and a message instead of crashing."""
    rc = bfa.lib().bf_scene_reset(None)
    assert rc < 0
    assert b"null" in bfa.lib().bf_last_error()


def test_synthetic_stream_host():
    scene = bfa.synth_scene(0)
    cam = bfa.depth_camera(80, 60, fx=577.87 / 8, fy=577.87 / 8)
    d1, c1 = bfa.synth_render_host(scene, bfa.synth_pose(3), cam, 1, 3)
    d2, c2 = bfa.synth_render_host(scene, bfa.synth_pose(3), cam, 1, 3)
    assert (d1 == d2).all() and (c1 == c2).all()
    valid = d1[d1 > 0]
    assert valid.size > 0.9 * d1.size
    assert valid.min() >= 0.1 and valid.max() <= 4.0
    # 1 mm quantisation (.sens ushort/1000 convention)
    assert abs(valid * 1000 - (valid * 1000).round()).max() < 1e-2


def test_solver_error_bits():
    """BFSolveResult.error: the recovered-timeout bit is the only non-fatal one (include/bf/types.h)."""
    assert abi.SOLVE_PCG_RECOVERED == 16 and abi.SOLVE_ERR_PCG_TIMEOUT == 8 and abi.SOLVE_ERR_PAIR_BOUND == 4
    assert abi.SOLVE_ERR_FATAL & abi.SOLVE_PCG_RECOVERED == 0
    assert abi.SOLVE_ERR_FATAL & abi.SOLVE_ERR_PCG_TIMEOUT and abi.SOLVE_ERR_FATAL & abi.SOLVE_ERR_PAIR_BOUND
    text = open(abi.HEADER_PATH.replace("bf.h", "types.h")).read()
    for name, v in (("BF_SOLVE_ERR_PAIR_BOUND", 4), ("BF_SOLVE_ERR_PCG_TIMEOUT", 8), ("BF_SOLVE_PCG_RECOVERED", 16)):
        assert f"#define {name} {v}u" in text, name


def test_configuration_is_in_the_abi_not_the_environment():
    """ABI v4: every production switch is a BFSceneOptions / BFReconOptions / BFSolverOptions field or
    bf_set_host_threads; the library reads no environment variable outside the diagnostics build
    (-DBF_RENDER_DIAG: the ray caster's per-wave / per-tile clock logs)."""
    import glob
    import re
    csrc = os.path.join(os.path.dirname(abi.LIB_PATH), "csrc")
    for path in glob.glob(os.path.join(csrc, "*.*")):
        text = open(path).read()
        for m in re.finditer(r"getenv", text):
            before = text[:m.start()]
            # the call must sit inside an #ifdef BF_RENDER_DIAG ... #endif block
            opened = before.rfind("#ifdef BF_RENDER_DIAG")
            assert opened >= 0 and before.rfind("#endif") < opened, (path, text[max(0, m.start() - 80):m.end() + 40])
    names = [n for n, _ in abi.BFSceneOptions._fields_]
    assert names[4:] == ["applyXcdRun", "applyRounds", "testFlags", "splatRowCap"]
    assert [n for n, _ in abi.BFReconOptions._fields_][-1] == "bundlingPriority"


def test_option_checks_without_device():
    """Invalid v4 options fail with BF_ERR_ARG before any device work."""
    L = bfa.lib()
    assert L.bf_set_host_threads(0) != 0 and L.bf_set_host_threads(257) != 0
    p = bfa.hash_params(voxel_size=0.01, num_buckets=1 << 10, num_blocks=1 << 10)
    for field, value, msg in (("testFlags", 2, b"testFlags"), ("applyXcdRun", 48, b"applyXcdRun"),
                              ("applyRounds", 65, b"applyRounds")):
        so = abi.BFSceneOptions()
        setattr(so, field, value)
        h = C.c_void_p()
        assert L.bf_scene_create(C.byref(p), C.byref(so), C.byref(h)) != 0
        assert msg in L.bf_last_error()
