"""prysm_amd — MI355X-native (gfx950) state-transition hot path of the early Prysm beacon chain.

The product is ``libprysm_hip.so`` (HIP kernels + C ABI, ``include/prysm_hip.h``).  This
package is the host-side mirror of the reference's Go package APIs for that path
(``types``, ``casper``, ``utils``, ``blockchain``) and calls the library through ctypes.
It never falls back to the CPU: without the library or a gfx950 device every compute call
raises ``PzError``.
"""
from prysm_amd._lib import PzError, lib, library_path  # noqa: F401
