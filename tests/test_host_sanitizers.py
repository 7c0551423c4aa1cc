"""Host code under sanitizers (SURVEY.md §5 race detection): the serial BLAKE2b hasher and its
thread pool (prysm_amd/csrc/serial_hash.cpp) built with ASan+UBSan and with TSan by
``make -C prysm_amd/csrc san``, run on the CPU.  No GPU code is involved."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def san_build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "prysm_amd", "csrc"), "san"], check=True)
    return os.path.join(ROOT, "build")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_serial_hasher_clean_under_sanitizer(san_build, kind):
    r = subprocess.run([os.path.join(san_build, "san_" + kind)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout
    assert "ERROR" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr
