"""The drop-in boundary: libarmour_hip.so exports exactly the C ABI include/armour_hip.h declares
(no compute calls here — the build container has no GPU), the Python binding knows every entry,
the product never reaches into the oracle, and without a device the product fails loudly."""
import os
import re
import subprocess

import numpy as np
import pytest

import armour_amd as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "armour_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(armour_\w+)\s*\(", src)))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l}


@pytest.fixture(scope="module")
def lib_path():
    if not os.path.exists(A.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "armour-dev_amd", "csrc"), "../armour_amd/libarmour_hip.so"],
                       check=True, capture_output=True)
    return A.LIB_PATH


def test_header_symbols_exported(lib_path):
    funcs = header_functions()
    assert len(funcs) >= 15
    missing = set(funcs) - exported(lib_path)
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(A.ABI_SYMBOLS) == header_functions()


def test_library_loads_and_binds(lib_path):
    L = A.lib()
    for name in A.ABI_SYMBOLS:
        assert hasattr(L, name)


def test_no_cpu_fallback_in_product():
    """The product path never imports or links the oracle / emulation."""
    pkg = os.path.join(ROOT, "armour-dev_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".h", ".hip", ".cpp", "Makefile")):
                text = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in text and "from oracle" not in text and "liboracle" not in text, f
                assert "reach_emu" not in text, f


def test_executable_built():
    exe = os.path.join(ROOT, "armour-dev_amd", "armour_amd", "armour_main")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "armour-dev_amd", "csrc")], check=True, capture_output=True)
    assert os.access(exe, os.X_OK)
    # the executable resolves the C ABI from libarmour_hip.so with dlopen (a served client never
    # maps the HIP runtime): it names the entry points it binds and links no HIP library
    strings = subprocess.run(["strings", exe], capture_output=True, text=True).stdout
    for sym in ("armour_create", "armour_plan", "armour_num_constraints", "libarmour_hip.so"):
        assert sym in strings, sym
    needed = subprocess.run(["readelf", "-d", exe], capture_output=True, text=True).stdout
    assert "amdhip" not in needed and "libarmour_hip" not in needed


def test_executable_without_device_fails_like_reference(tmp_path):
    """no server, no GPU (this container): -1 in armour.out and a non-zero status"""
    exe = os.path.join(ROOT, "armour-dev_amd", "armour_amd", "armour_main")
    (tmp_path / "armour.in").write_text("0 " * 28 + "0\n")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert (tmp_path / "armour.out").read_text().split() == ["-1"]


def test_create_without_device_fails_loudly():
    """No GPU (this container): armour_create fails with a message instead of computing on the CPU."""
    try:
        import torch

        if torch.cuda.device_count() > 0:
            pytest.skip("a device is present")
    except ImportError:
        pass
    with pytest.raises(A.ArmourError):
        A.Planner(T=10, max_obstacles=2, max_worlds=1)
    with pytest.raises(A.ArmourError):
        A.copy_bandwidth(0, 1 << 20, 1)


def test_bad_config_rejected_before_device():
    """Argument checks come first (KPR/Parameters.h: NUM_TIME_STEPS must be even)."""
    with pytest.raises(A.ArmourError, match="even"):
        A.Planner(T=11, max_obstacles=2, max_worlds=1)


def test_world_batch_marshalling():
    # Planner._worlds fills the armour_world array (include/armour_hip.h) through a NumPy view:
    # every field must equal the inputs, obstacle pointers must address each world's own block,
    # and a world without obstacles gets a null pointer
    import ctypes
    import types
    worlds = [A.make_world(s, 20) for s in range(5)] + [A.make_world(9, 0), A.make_world(11, 3)]
    holder = types.SimpleNamespace()   # owns the obstacle block, as a Planner does (self._keep)
    arr = A.Planner._worlds(holder, worlds)
    assert ctypes.sizeof(arr) == len(worlds) * ctypes.sizeof(A.World)
    for i, w in enumerate(worlds):
        a = arr[i]
        for k, f in enumerate(("q0", "qd0", "qdd0", "q_des")):
            assert np.array_equal(np.array(getattr(a, f)[:]), np.asarray(w[k], dtype=float)), (i, f)
        o = np.asarray(w[4], dtype=float).reshape(-1, 12)
        assert a.num_obstacles == o.shape[0]
        if o.shape[0]:
            got = np.ctypeslib.as_array(a.obstacles, shape=(o.shape[0] * 12,)).reshape(-1, 12)
            assert np.array_equal(got, o), i
        else:
            assert not a.obstacles
