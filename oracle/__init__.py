"""ORACLE — TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.

CPU restatement of the reference's (JahanaraCo/prysm, early beacon chain, pure Go)
state-transition hot path.  It exists only to *check* the HIP path:

* ``tests/`` compare the HIP path against it on the same seeded inputs,
* ``__graft_entry__.smoke()`` checks one tiny invocation against it,
* ``bench.py``'s ``cpu_baseline`` leg times the C restatement in ``oracle/c``.

Nothing under ``prysm_amd/`` may import, call, link or execute anything in this
directory; the product path fails loudly when the HIP library is missing.

Independence / pinning
----------------------
* BLAKE2b-512: ``hashlib.blake2b`` (CPython's bundled reference C implementation of
  RFC 7693), pinned by the RFC 7693 Appendix A known-answer test (``"abc"``).
  The reference calls ``golang.org/x/crypto/blake2b`` @ a49355c7e3f8fe157a85be2f77e6e269a0f89602
  (``/root/reference/WORKSPACE:504-508``), which is not vendored.
* proto3 wire bytes: Google's ``protobuf`` runtime (upb) over a schema restated from
  ``proto/beacon/p2p/v1/messages.proto:21-130`` (field numbers/types cross-checked against
  the struct tags in ``messages.pb.go:224-985``).  golang/protobuf and gogo/protobuf (the
  reference's encoders, pinned transitively by rules_go 0.12.1) are not vendored.
* Casper / utils / blockchain logic: restated from the Go source, each function citing
  file:line, and pinned by every known-answer test the reference's own ``*_test.go`` hold
  (see ``tests/test_oracle_kats.py``).
* The reference itself cannot be compiled or run here (pure Go; no Go toolchain in the
  container or on the GPU box).  Hash digests of serialized objects are therefore pinned by
  two independent implementations agreeing (this oracle vs the product's own encoder + HIP
  BLAKE2b), plus RFC 7693; no reference test pins a literal digest.
"""
