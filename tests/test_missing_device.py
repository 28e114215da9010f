"""C-ABI entry points called with a device ordinal that does not exist must return FCG_ERR_DEVICE
and leave no sticky HIP status behind: torch's next HIP call on the real device must succeed
(round 2 saw `HIP error: invalid device ordinal` in an unrelated test after such a probe).
Every entry point returning FCG_ERR_DEVICE reads hipGetLastError first (csrc/fcg_status.hpp)."""
import ctypes
import importlib

import numpy as np
import pytest
import torch

fcg = importlib.import_module("4c_amd").fcg

pytestmark = pytest.mark.gpu

MISSING = 1 << 20


def _torch_still_works():
    x = torch.arange(1024, dtype=torch.float64, device="cuda:0")
    assert float((x * 2).sum().item()) == 2.0 * 1023 * 1024 / 2
    torch.cuda.synchronize()


def test_measure_hbm_rejects_a_missing_device():
    with pytest.raises(fcg.FcgError):
        fcg.measure_hbm(MISSING)
    _torch_still_works()


def test_measure_peaks_rejects_a_missing_device():
    with pytest.raises(fcg.FcgError):
        fcg.measure_peaks(MISSING)
    _torch_still_works()


def test_create_rejects_a_missing_device():
    mesh = fcg.BoxMesh(fcg.HEX8, (2, 2, 2))
    with pytest.raises(fcg.FcgError) as e:
        fcg.Evaluator(mesh, kinematics=fcg.LINEAR, device=MISSING)
    assert e.value.code == fcg.FCG_ERR_DEVICE
    _torch_still_works()


def test_comm_create_rejects_a_missing_device():
    L = fcg.lib()
    uid = (ctypes.c_char * 128)()
    assert L.fcg_comm_unique_id(uid) == 0
    h = ctypes.c_void_p()
    rc = L.fcg_comm_create(uid, 1, 0, MISSING, ctypes.byref(h))
    assert rc == fcg.FCG_ERR_DEVICE and not h.value
    _torch_still_works()


def test_device_alloc_rejects_a_missing_device():
    p = ctypes.c_void_p()
    assert fcg.lib().fcg_device_alloc(MISSING, 1024, ctypes.byref(p)) == fcg.FCG_ERR_DEVICE
    _torch_still_works()


def test_oversized_device_alloc_leaves_torch_usable():
    # an allocation the device cannot hold: FCG_ERR_DEVICE, then torch allocates normally
    p = ctypes.c_void_p()
    rc = fcg.lib().fcg_device_alloc(0, 1 << 50, ctypes.byref(p))
    assert rc == fcg.FCG_ERR_DEVICE
    _torch_still_works()
