"""DPP / permlane wave primitives (armour-dev_amd/csrc/wave.h) against ds_bpermute shuffles."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpu_unit")


def test_wave_primitives():
    L = ctypes.CDLL(os.path.join(HERE, "libwave_test.so"))
    blocks = 16
    rng = np.random.default_rng(7)
    v = rng.integers(0, 2**63, size=blocks * 64, dtype=np.uint64)
    bad = np.zeros(blocks * 64, dtype=np.int32)
    rc = L.wave_selftest(blocks, v.ctypes.data_as(ctypes.c_void_p), bad.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    names = {1: "xor_u64", 2: "xor_u32", 4: "next_f64", 8: "prev_u64", 16: "wave_sum uniform", 32: "wave_incl_scan",
             64: "wave_max"}
    fails = [n for bit, n in names.items() if np.any(bad & bit)]
    assert not fails, fails
