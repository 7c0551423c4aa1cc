"""The library also works in a process without PyTorch (the cgo situation): it then binds to
/opt/rocm's HIP runtime.  Runs a child interpreter that never imports torch."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import builtins, hashlib, sys
real_import = builtins.__import__
def guard(name, *a, **k):
    if name == "torch" or name.startswith("torch."):
        raise ImportError("torch blocked in this process")
    return real_import(name, *a, **k)
builtins.__import__ = guard
sys.path.insert(0, %r)
from prysm_amd import _lib
assert not _lib.HAVE_TORCH
msgs = [b"", b"abc", bytes(range(200)) * 3]
for m, d in zip(msgs, _lib.blake2b512_batch(msgs, 64)):
    assert d == hashlib.blake2b(m, digest_size=64).digest()
print("ok-no-torch")
""" % ROOT


def test_library_without_torch():
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok-no-torch" in r.stdout
