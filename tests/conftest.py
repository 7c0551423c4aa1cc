import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


AB_LIB = os.path.join(ROOT, "build", "ab", "libprysm_hip.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "ab: measured-and-dropped forms and measurement hooks; runs only against the "
                                       "A/B library (make -C prysm_amd/csrc ab) under -m ab")
    # `-m ab` (or an expression naming ab without "not ab"): the session loads the A/B library
    # (library_path set in this process only: no environment variable, so child processes the
    # multiprocess tests start load the product library)
    expr = config.option.markexpr or ""
    if "ab" in expr.split() and "not ab" not in expr:
        from prysm_amd import _lib
        _lib.library_path = AB_LIB


def pytest_collection_modifyitems(config, items):
    from prysm_amd import _lib
    ab_loaded = _lib.library_path == AB_LIB
    skip = pytest.mark.skip(reason="A/B form: run with -m ab against build/ab/libprysm_hip.so")
    for it in items:
        if "ab" in it.keywords and not ab_loaded:
            it.add_marker(skip)

# Load PyTorch (and its HIP runtime) before the product library: see prysm_amd/_lib.py.
import torch  # noqa: E402,F401
