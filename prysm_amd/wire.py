"""proto3 wire encoder for the hashed messages (host side; what ``proto.Marshal`` produces).

Restates the golang/protobuf v1.1 table marshaller's proto3 rules as used at
types/block.go:69, types/attestation.go:51 and (via gogo, same generated code)
types/state.go:141,240:
  * fields in ascending field-number order;
  * zero scalars and empty ``bytes`` scalars are omitted;
  * every element of a ``repeated bytes`` is emitted, empty ones as ``tag 00``;
  * a non-nil message field is emitted even when empty (``Timestamp{0,0}`` -> ``3a 00``);
  * ``repeated uint32/uint64`` are packed and omitted when empty;
  * negative int32/int64 are 10-byte varints (sign-extended to 64 bits).
Validators and committees are encoded with numpy (one vectorised pass per field) so a
1M-validator CrystallizedState serialises in well under a second.
"""
import numpy as np

from prysm_amd import pb

_U64 = np.uint64
M64 = (1 << 64) - 1


def varint(x):
    x &= M64
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _tag(num, wt):
    return varint((num << 3) | wt)


def _u(num, v):
    return _tag(num, 0) + varint(v) if v else b""


def _b(num, v):
    return _tag(num, 2) + varint(len(v)) + bytes(v) if v else b""


def _msg(num, body):
    return _tag(num, 2) + varint(len(body)) + body


def _packed(num, values):
    if len(values) == 0:
        return b""
    if len(values) <= 64 and not isinstance(values, np.ndarray):  # short lists: scalar path
        body = b"".join(varint(int(v)) for v in values)
    else:
        body = packed_varints(np.asarray(values, dtype=_U64))
    return _tag(num, 2) + varint(len(body)) + body


# ---- vectorised varints ---------------------------------------------------------------------
def varint_len(x):
    """Per-element varint byte length of a uint64 array (0 -> 1)."""
    x = np.asarray(x, dtype=_U64)
    n = np.ones(x.shape, dtype=np.int64)
    for k in range(1, 10):
        n += (x >= _U64(1 << (7 * k))).astype(np.int64)
    return n


def _scatter_varints(out, pos, x, nbytes):
    """Write varint(x[i]) at out[pos[i]:pos[i]+nbytes[i]] (vectorised over bytes)."""
    x = x.astype(_U64).copy()
    for k in range(int(nbytes.max()) if nbytes.size else 0):
        live = nbytes > k
        more = nbytes > k + 1
        b = (x & _U64(0x7F)).astype(np.uint8) | np.where(more, 0x80, 0).astype(np.uint8)
        out[(pos + k)[live]] = b[live]
        x >>= _U64(7)


def packed_varints(values):
    values = np.asarray(values, dtype=_U64)
    nb = varint_len(values)
    pos = np.concatenate([[0], np.cumsum(nb)[:-1]]).astype(np.int64)
    out = np.zeros(int(nb.sum()), dtype=np.uint8)
    _scatter_varints(out, pos, values, nb)
    return out.tobytes()


# ---- messages ------------------------------------------------------------------------------
def timestamp(t):
    return _u(1, t.seconds & M64) + _u(2, t.nanos & M64)


def attestation_record(a):
    """messages.proto:110-119."""
    out = [_u(1, a.slot), _u(2, a.shard_id), _u(3, a.justified_slot), _b(4, a.justified_block_hash),
           _b(5, a.shard_block_hash), _b(6, a.attester_bitfield)]
    out += [_msg(7, bytes(h)) for h in a.oblique_parent_hashes]  # repeated bytes: every element
    out.append(_packed(8, a.aggregate_sig))
    return b"".join(out)


def beacon_block(b):
    """messages.proto:37-46."""
    out = [_b(1, b.parent_hash), _u(2, b.slot_number), _b(3, b.randao_reveal), _b(4, b.pow_chain_ref),
           _b(5, b.active_state_hash), _b(6, b.crystallized_state_hash)]
    if b.timestamp is not None:
        out.append(_msg(7, timestamp(b.timestamp)))
    out += [_msg(8, attestation_record(a)) for a in b.attestations]
    return b"".join(out)


def active_state(s):
    """messages.proto:94-97."""
    out = [_msg(1, attestation_record(a)) for a in s.pending_attestations]
    out += [_msg(2, bytes(h)) for h in s.recent_block_hashes]
    return b"".join(out)


def crosslink_record(r):
    return _u(1, r.dynasty) + _b(2, r.blockhash) + _u(3, r.slot)


def shard_and_committee(sc):
    return _u(1, sc.shard_id) + _packed(2, sc.committee)


def shard_and_committee_array(arr):
    return b"".join(_msg(1, shard_and_committee(sc)) for sc in arr.array_shard_and_committee)


def validators(v, field_num=11):
    """Every ValidatorRecord of a ``pb.Validators`` block, each framed as repeated message
    ``field_num`` (CrystallizedState.validators = 11), vectorised over records."""
    n = len(v)
    if n == 0:
        return b""
    if v.withdrawal_address is not None or v.randao_commitment is not None:
        return b"".join(_msg(field_num, _validator_scalar(v, i)) for i in range(n))
    fields = [(1, v.public_key), (2, v.withdrawal_shard), (5, v.balance), (6, v.start_dynasty),
              (7, v.end_dynasty)]
    lens = []
    body = np.zeros(n, dtype=np.int64)
    for num, x in fields:
        nb = np.where(x != 0, varint_len(x), 0)
        lens.append(nb)
        body += np.where(x != 0, 1 + nb, 0)  # single-byte tags (fields 1..15)
    frame = 1 + varint_len(body.astype(_U64))  # tag 0x5a + length varint
    total = frame + body
    start = np.concatenate([[0], np.cumsum(total)[:-1]]).astype(np.int64)
    out = np.zeros(int(total.sum()), dtype=np.uint8)
    out[start] = (field_num << 3) | 2
    _scatter_varints(out, start + 1, body.astype(_U64), frame - 1)
    pos = start + frame
    for (num, x), nb in zip(fields, lens):
        present = x != 0
        out[pos[present]] = (num << 3) | 0
        _scatter_varints(out, (pos + 1)[present], x[present], nb[present])
        pos = pos + np.where(present, 1 + nb, 0)
    return out.tobytes()


def _validator_scalar(v, i):
    wa = v.withdrawal_address[i] if v.withdrawal_address is not None else b""
    rc = v.randao_commitment[i] if v.randao_commitment is not None else b""
    return (_u(1, int(v.public_key[i])) + _u(2, int(v.withdrawal_shard[i])) + _b(3, wa) + _b(4, rc) +
            _u(5, int(v.balance[i])) + _u(6, int(v.start_dynasty[i])) + _u(7, int(v.end_dynasty[i])))


def crystallized_state(s):
    """messages.proto:59-72."""
    out = [_u(1, s.last_state_recalc), _u(2, s.justified_streak), _u(3, s.last_justified_slot),
           _u(4, s.last_finalized_slot), _u(5, s.current_dynasty), _u(6, s.crosslinking_start_shard),
           _u(7, s.total_deposits), _b(8, s.dynasty_seed), _u(9, s.dynasty_seed_last_reset)]
    out += [_msg(10, crosslink_record(r)) for r in s.crosslink_records]
    out.append(validators(s.validators))
    out += [_msg(12, shard_and_committee_array(a)) for a in s.shard_and_committees_for_slots]
    return b"".join(out)


# ---- device encoder (prysm_amd/csrc/wire.hip) ------------------------------------------------
def _csr(blobs, n):
    if blobs is None:
        return None, None
    offs = np.zeros(n + 1, dtype=_U64)
    offs[1:] = np.cumsum([len(b) for b in blobs], dtype=_U64)
    data = np.frombuffer(b"".join(bytes(b) for b in blobs) + b"\0", dtype=np.uint8)
    return data, offs


def validators_device(v, field_num=11, with_offsets=False):
    """The same bytes as :func:`validators`, encoded on the GPU by ``pz_wire_validators``
    (size / scan / write kernels over the SoA columns).  ``field_num=0`` gives
    bare records; ``with_offsets`` also returns each record's start (n+1 offsets)."""
    from prysm_amd import _lib

    n = len(v)
    wa, wa_offs = _csr(v.withdrawal_address, n)
    rc, rc_offs = _csr(v.randao_commitment, n)
    cols = _lib.ValidatorCols(
        _lib.ptr(v.public_key), _lib.ptr(v.withdrawal_shard), _lib.ptr(wa), _lib.ptr(wa_offs),
        _lib.ptr(rc), _lib.ptr(rc_offs), _lib.ptr(v.balance), _lib.ptr(v.start_dynasty),
        _lib.ptr(v.end_dynasty))
    nbytes = (int(wa_offs[-1]) if wa_offs is not None else 0) + (int(rc_offs[-1]) if rc_offs is not None else 0)
    cap = int(_lib.lib.dll.pz_wire_validators_bound(n, nbytes))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    offs = np.empty(n + 1, dtype=_U64) if with_offsets else None
    length = _lib.ctypes.c_uint64(0)
    _lib.lib.call("pz_wire_validators", _lib.ctypes.byref(cols), n, field_num, _lib.ptr(out), cap,
                  _lib.ptr(offs), _lib.ctypes.byref(length))
    raw = out[:length.value].tobytes()
    return (raw, offs) if with_offsets else raw


ATT_COLS = ("slot", "shard_id", "justified_slot", "justified_block_hash", "justified_block_hash_offs",
            "shard_block_hash", "shard_block_hash_offs", "attester_bitfield", "attester_bitfield_offs",
            "oblique_parent_hashes", "oblique_offs", "oblique_first", "aggregate_sig", "aggregate_sig_first")


def attestation_columns(atts):
    """pb.AttestationRecord list -> the SoA / CSR columns of ``pz_attestation_cols``."""
    n = len(atts)
    cols = {k: np.ascontiguousarray([getattr(a, k) for a in atts], dtype=_U64)
            for k in ("slot", "shard_id", "justified_slot")}
    for k in ("justified_block_hash", "shard_block_hash", "attester_bitfield"):
        cols[k], cols[k + "_offs"] = _csr([bytes(getattr(a, k)) for a in atts], n)
    elems = [bytes(h) for a in atts for h in a.oblique_parent_hashes]
    cols["oblique_parent_hashes"], cols["oblique_offs"] = _csr(elems, len(elems))
    cols["oblique_first"] = np.zeros(n + 1, dtype=_U64)
    cols["oblique_first"][1:] = np.cumsum([len(a.oblique_parent_hashes) for a in atts])
    cols["aggregate_sig"] = np.ascontiguousarray([v & M64 for a in atts for v in a.aggregate_sig] or [0], dtype=_U64)
    cols["aggregate_sig_first"] = np.zeros(n + 1, dtype=_U64)
    cols["aggregate_sig_first"][1:] = np.cumsum([len(a.aggregate_sig) for a in atts])
    return cols


def attestations_device(cols, n, field_num=0):
    """AttestationRecords encoded on the GPU by ``pz_wire_attestations`` from columns (see
    :func:`attestation_columns`).  Returns (bytes, offsets[n+1]); with ``field_num=0`` the
    records are bare, as Attestation.Hash() hashes them."""
    from prysm_amd import _lib

    c = _lib.AttestationCols(*[_lib.ptr(np.ascontiguousarray(cols[k])) if cols.get(k) is not None else None
                               for k in ATT_COLS])
    nbytes = sum(int(cols[k][-1]) for k in ("justified_block_hash_offs", "shard_block_hash_offs",
                                            "attester_bitfield_offs", "oblique_offs")) if n else 0
    ne = int(cols["oblique_first"][-1]) if n else 0
    ns = int(cols["aggregate_sig_first"][-1]) if n else 0
    cap = int(_lib.lib.dll.pz_wire_attestations_bound(n, nbytes, ne, ns))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    offs = np.empty(n + 1, dtype=_U64)
    length = _lib.ctypes.c_uint64(0)
    _lib.lib.call("pz_wire_attestations", _lib.ctypes.byref(c), n, field_num, _lib.ptr(out), cap, _lib.ptr(offs),
                  _lib.ctypes.byref(length))
    return out[:length.value].tobytes(), offs
