"""The C-ABI library loads and exports every function include/prysm_hip.h declares (no GPU
needed: nothing is called except the version query)."""
import ctypes
import os
import re

import pytest

from prysm_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "prysm_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pz_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    dll = ctypes.CDLL(_lib.library_path)
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(dll, n)]
    assert not missing, missing


def test_product_exports_no_debug_entry_points():
    """The product library carries no pz_debug_* entry points: the measurement
    hooks and host-only test entry points live in the A/B library (-DPZ_AB_BUILD)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.library_path], capture_output=True, text=True,
                         check=True).stdout
    names = [ln.split()[-1] for ln in out.splitlines() if ln.strip()]
    assert any(n.startswith("pz_") for n in names)
    assert [n for n in names if n.startswith("pz_debug")] == []


def test_binding_covers_header():
    assert set(declared_functions()) <= set(_lib.SIGNATURES)


def test_version():
    assert _lib.lib.dll.pz_version() == 1


@pytest.mark.parametrize("name,cls", [("pz_epoch_batch", _lib.EpochBatch), ("pz_validator_cols", _lib.ValidatorCols),
                                       ("pz_att_check_batch", _lib.AttCheckBatch),
                                       ("pz_attestation_cols", _lib.AttestationCols),
                                       ("pz_epoch_host", _lib.EpochHost)])
def test_struct_layout(name, cls):
    # the structs are passed by pointer from ctypes: field order/packing must match the header
    src = open(os.path.join(ROOT, "include", "prysm_hip.h")).read()
    body = src[src.index("typedef struct %s" % name):src.index("} %s;" % name)]
    body = re.sub(r"/\*.*?\*/", "", body.split("{", 1)[1], flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:
            first, *rest = decl.split(",")
            fields += [first.split()[-1].lstrip("*")] + [r.strip().lstrip("*") for r in rest]
    assert fields == [f for f, _ in cls._fields_]


def test_host_serial_hasher_matches_hashlib():
    """The host BLAKE2b used for long serial messages (prysm_amd/csrc/serial_hash.cpp; no GPU
    involved) against hashlib (RFC 7693) at every block boundary and a few long lengths."""
    import hashlib

    import numpy as np

    from ab_lib import ab_dll
    fn = ab_dll().pz_debug_host_blake2b512
    fn.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    fn.restype = None
    rng = np.random.default_rng(1)
    out = ctypes.create_string_buffer(64)
    for n in list(range(0, 300)) + [1023, 1024, 1025, 65535, 65536, 200001]:
        m = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        fn(m, n, out)
        assert out.raw == hashlib.blake2b(m).digest(), n
    assert _lib.lib.dll.pz_set_serial_threshold(12345) == 65536
    assert _lib.lib.dll.pz_set_serial_threshold(65536) == 12345
