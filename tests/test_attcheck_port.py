"""The C port of processAttestation's checks (oracle/c/attcheck_ref.c, bench.py's attcheck
cpu_baseline) against the scalar oracle (oracle/ref.py).  CPU only: oracle vs oracle."""
import numpy as np

from oracle import cport, ref
from test_attcheck_gpu import oracle_code, random_batch, table


def test_c_port_matches_scalar_oracle():
    active, cstate = ref.new_genesis_states(1024)
    cstate.last_state_recalc, cstate.last_justified_slot = 64, 60
    rng = np.random.default_rng(77)
    atts, bslots = random_batch(rng, cstate, 2000, 64, 128)
    want = [oracle_code(cstate, active, bs, a) for a, bs in zip(atts, bslots)]
    bf = [bytes(a.attester_bitfield) for a in atts]
    boffs = np.zeros(len(atts) + 1, dtype=np.uint64)
    boffs[1:] = np.cumsum([len(x) for x in bf])
    arrs = table(cstate)
    entries = [e for arr in arrs for e in arr]
    arr_offs = np.zeros(len(arrs) + 1, dtype=np.uint64)
    arr_offs[1:] = np.cumsum([len(a) for a in arrs])
    coffs = np.zeros(len(entries) + 1, dtype=np.uint64)
    coffs[1:] = np.cumsum([len(e[1]) for e in entries])
    port = cport.AttCheck([a.slot for a in atts], [a.justified_slot for a in atts], [a.shard_id for a in atts],
                          [len(a.oblique_parent_hashes) for a in atts],
                          np.frombuffer(b"".join(bf) + b"\0", dtype=np.uint8), boffs, bslots)
    try:
        got = port.run(60, 64, 128, arr_offs, np.array([e[0] for e in entries], dtype=np.uint64),
                       np.arange(len(entries), dtype=np.uint32), coffs)
    finally:
        port.close()
    assert list(got) == want
