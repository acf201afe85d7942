"""CPU tests of the C ABI library: it loads, exports every symbol the header
declares, and refuses to compute without a GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, have_gpu
from multiview_amd import _lib, rig

HEADER = os.path.join(ROOT, "include", "mvba", "mvba.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(mvba_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ("mvba_create", "mvba_destroy", "mvba_set_params", "mvba_evaluate",
              "mvba_evaluate_device", "mvba_last_error", "mvba_sync_status"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding covers all of them
    assert set(declared_functions()) == set(_lib.SIGNATURES)


def test_abi_version():
    lib = _lib.load()
    assert lib.mvba_abi_version() == 6


@pytest.mark.skipif(have_gpu(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback_without_gpu():
    from multiview_amd.evaluator import Evaluator

    R = rig.make_rig(num_sensors=2, num_ref=5, num_points=20, obs_per_point=3, seed=5)
    P = rig.build_problem(R)
    with pytest.raises(_lib.MvbaError) as e:
        Evaluator(P)
    assert e.value.status == _lib.MVBA_E_NO_DEVICE
    n = C.c_int32(-1)
    assert _lib.load().mvba_device_count(C.byref(n)) == _lib.MVBA_E_NO_DEVICE
    assert n.value == 0
