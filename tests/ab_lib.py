"""The A/B library (make -C prysm_amd/csrc ab -> build/ab/libprysm_hip.so) for CPU tests of
host-only internals the product library does not export (pz_debug_*: the SHM group's
collectives, the host hasher on one message, the block parser on its own).  Loaded with
ctypes beside the product library, never through prysm_amd._lib."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(ROOT, "build", "ab", "libprysm_hip.so")


def ab_dll():
    if not os.path.exists(AB_LIB):
        pytest.skip("A/B library not built (__graft_entry__.build() builds it)")
    return ctypes.CDLL(AB_LIB)
