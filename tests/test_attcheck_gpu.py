"""processAttestation's checks on the GPU (pz_check_attestations, prysm_amd/csrc/attcheck.hip)
against the oracle's scalar restatement (oracle/ref.py process_attestation, which follows
blockchain/core.go:240-297 and :348-394) on seeded random attestations that hit every
check, at 1,024 and 65,536 validators."""
import numpy as np
import pytest

from oracle import ref
from oracle import schema as opb
from prysm_amd import _lib
from prysm_amd.blockchain import check_attestations

pytestmark = pytest.mark.gpu

PROCESSED, SLOT_HIGH, SLOT_LOW, JUSTIFIED, NO_COMMITTEE, BITFIELD_LEN, TRAILING = 0, 2, 3, 4, 5, 6, 7


def oracle_code(cstate, astate, block_slot, att):
    try:
        ref.process_attestation(cstate, astate, block_slot, att)
        return PROCESSED
    except ref.GoPanic as e:
        return _lib.PZ_ERANGE if "slice bounds" in str(e) else _lib.PZ_EINDEX
    except ref.GoError as e:
        m = str(e)
        for key, code in (("higher", SLOT_HIGH), ("lower", SLOT_LOW), ("justified", JUSTIFIED),
                          ("unable to find", NO_COMMITTEE), ("bitfield length", BITFIELD_LEN),
                          ("trailing", TRAILING)):
            if key in m:
                return code
        raise


def table(cstate):
    return [[(sc.shard_id, list(sc.committee)) for sc in arr.array_shard_and_committee]
            for arr in cstate.shard_and_committees_for_slots]


def random_batch(rng, cstate, n, lsr, n_recent):
    arrs = table(cstate)
    atts, bslots = [], []
    for _ in range(n):
        bs = int(rng.integers(lsr, lsr + 200))
        s = max(0, bs - int(rng.integers(-3, 72)))
        idx = s - lsr
        if 0 <= idx < len(arrs) and rng.random() < 0.9:
            shard, comm = arrs[idx][int(rng.integers(0, len(arrs[idx])))]
        else:
            shard, comm = int(rng.integers(0, 1024)), list(range(int(rng.integers(1, 300))))
        k = len(comm)
        blen = (k + 7) // 8 + (int(rng.choice([-1, 1])) if rng.random() < 0.05 else 0)
        bf = bytearray(rng.integers(0, 256, size=max(blen, 0), dtype=np.uint8).tobytes())
        if k % 8 and blen == (k + 7) // 8 and rng.random() < 0.9:
            bf[-1] &= (0xFF << (8 - k % 8)) & 0xFF  # clear the trailing bits (most of the time)
        js = cstate.last_justified_slot if rng.random() < 0.95 else int(rng.integers(0, 1000))
        nob = int(rng.choice([0, 0, 0, 1, 2, 70]))
        atts.append(opb.AttestationRecord(slot=s, shard_id=shard, justified_slot=js, attester_bitfield=bytes(bf),
                                          oblique_parent_hashes=[bytes(rng.integers(0, 256, 32, dtype=np.uint8))
                                                                 for _ in range(nob)]))
        bslots.append(bs)
    return atts, bslots


@pytest.mark.parametrize("nval,lsr,ljs,n_recent", [(1024, 0, 0, 128), (1024, 64, 60, 128), (65536, 128, 64, 100)])
def test_checks_match_oracle(nval, lsr, ljs, n_recent):
    active, cstate = ref.new_genesis_states(nval)
    cstate.last_state_recalc = lsr
    cstate.last_justified_slot = ljs
    del active.recent_block_hashes[n_recent:]
    rng = np.random.default_rng(nval + lsr)
    atts, bslots = random_batch(rng, cstate, 3000, lsr, n_recent)
    status, comm, pstart = check_attestations(atts, bslots, ljs, lsr, len(active.recent_block_hashes), table(cstate))
    want = [oracle_code(cstate, active, bs, a) for a, bs in zip(atts, bslots)]
    assert list(status) == want
    seen = set(want)
    assert {PROCESSED, SLOT_HIGH, SLOT_LOW, JUSTIFIED, BITFIELD_LEN, _lib.PZ_ERANGE} <= seen, seen
    entries = [e for arr in table(cstate) for e in arr]
    for a, st, c, ps, bs in zip(atts, status, comm, pstart, bslots):
        if st in (PROCESSED, BITFIELD_LEN, TRAILING):
            assert entries[c][1] == ref.get_attester_indices(cstate, a)
            assert ps == bs - a.slot


def test_go_int_conversion_of_huge_slots():
    """core.go:244-253 compare int(Slot) with int(SlotNumber): a slot >= 2^63 is negative in
    Go, so it fails the lower-bound check, not the upper one."""
    _, cstate = ref.new_genesis_states(1024)
    att = opb.AttestationRecord(slot=(1 << 63) + 5, shard_id=0, attester_bitfield=b"\0\0")
    status, _, _ = check_attestations([att], [100], 0, 0, 128, table(cstate))
    assert status[0] == SLOT_LOW


def test_empty_batch():
    status, comm, pstart = check_attestations([], [], 0, 0, 128, [])
    assert len(status) == 0


@pytest.mark.parametrize("lastb", [False, True])
@pytest.mark.parametrize("natt,shift", [(4097, 0), (4096, 1), (1, 0)])
def test_device_forms_match_c_port(natt, shift, lastb):
    """pz_dev_check_attestations on bench.attcheck_columns' inputs: 16-B-aligned columns take
    the two-per-lane kernel (odd tail included), columns shifted by one element the one-per-lane
    kernel; both equal the C port (oracle/c/attcheck_ref.c), with the trailing-bits byte read
    from the bitfields or from the caller's last-byte column."""
    import ctypes

    import torch

    import bench
    from oracle import cport

    cols, tab = bench.attcheck_columns(natt, seed=5)
    dev = torch.device("cuda", 0)

    def put(v):
        a = v.view(np.int64) if v.dtype == np.uint64 else v.view(np.int32) if v.dtype == np.uint32 else v
        buf = torch.zeros(a.size + shift + 2, dtype=torch.from_numpy(a[:1]).dtype, device=dev)
        buf[shift:shift + a.size] = torch.from_numpy(a).to(dev)
        return buf, buf[shift:]

    keep, t = [], {}
    extra = {}
    if lastb:
        extra["last_byte"] = cols["bits"][(cols["boffs"][1:].astype(np.int64) - 1) % cols["bits"].size]
    for k, v in list(cols.items()) + list(tab.items()) + list(extra.items()):
        buf, view = put(v)
        keep.append(buf)
        t[k] = view
    status = torch.empty(natt + 1, dtype=torch.int32, device=dev)[shift:]
    comm = torch.empty(natt + 1, dtype=torch.int32, device=dev)[shift:]
    pstart = torch.empty(natt + 2, dtype=torch.int64, device=dev)[shift:]
    b = _lib.AttCheckBatch(natt, t["slot"].data_ptr(), t["justified_slot"].data_ptr(), t["shard_id"].data_ptr(),
                           t["n_oblique"].data_ptr(), t["bits"].data_ptr(), t["boffs"].data_ptr(),
                           t["block_slot"].data_ptr(), 0, 0, 128, 256, t["arr_offs"].data_ptr(),
                           t["arr_shard"].data_ptr(), t["arr_comm"].data_ptr(), t["coffs"].data_ptr(),
                           status.data_ptr(), comm.data_ptr(), pstart.data_ptr(),
                           t["last_byte"].data_ptr() if lastb else None)
    _lib.lib.call("pz_dev_check_attestations", ctypes.byref(b), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    port = cport.AttCheck(cols["slot"], cols["justified_slot"], cols["shard_id"], cols["n_oblique"], cols["bits"],
                          cols["boffs"], cols["block_slot"])
    try:
        want = port.run(0, 0, 128, tab["arr_offs"], tab["arr_shard"], tab["arr_comm"], tab["coffs"])
    finally:
        port.close()
    np.testing.assert_array_equal(status[:natt].cpu().numpy(), want)
    ok = want == PROCESSED
    np.testing.assert_array_equal(pstart[:natt].cpu().numpy()[ok], (cols["block_slot"] - cols["slot"])[ok].view(np.int64))
