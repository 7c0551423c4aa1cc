"""ctypes binding of ``libprysm_hip.so`` (include/prysm_hip.h).

Loading fails loudly: if the in-tree library is missing, importing a compute entry point
raises ``PzError`` — there is no CPU fallback anywhere in ``prysm_amd``.
"""
import ctypes
import os

import numpy as np

# One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 and loads it into the
# global symbol scope at import; when torch is present we import it BEFORE loading our
# library so that libprysm_hip.so binds to that same runtime (device pointers, streams and
# events are then interchangeable with torch's).  Without torch (e.g. a cgo host) the
# library binds to /opt/rocm's runtime.  Initialising two different HIP runtimes in one
# process fails ("No HIP GPUs are available"), so this order is load-bearing.
try:  # pragma: no cover - import side effect only
    import torch  # noqa: F401
    HAVE_TORCH = True
except ImportError:  # pragma: no cover
    HAVE_TORCH = False

HERE = os.path.dirname(os.path.abspath(__file__))
library_path = os.path.join(HERE, "libprysm_hip.so")

PZ_OK = 0
PZ_ENIL = -1
PZ_EINDEX = -2
PZ_ETOOMANY = -3
PZ_EDEVICE = -4
PZ_ENOTFOUND = -5
PZ_EINVAL = -6
PZ_ERANGE = -7

_NAMES = {PZ_ENIL: "ENIL", PZ_EINDEX: "EINDEX", PZ_ETOOMANY: "ETOOMANY", PZ_EDEVICE: "EDEVICE",
          PZ_ENOTFOUND: "ENOTFOUND", PZ_EINVAL: "EINVAL", PZ_ERANGE: "ERANGE"}


class PzError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (_NAMES.get(code, "?"), code, msg))
        self.code = code


c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_intp = ctypes.POINTER(ctypes.c_int)
u64 = ctypes.c_uint64
u32 = ctypes.c_uint32
vp = ctypes.c_void_p

# name -> argtypes (all return int status unless listed in _RESTYPES)
SIGNATURES = {
    "pz_init": [ctypes.c_int],
    "pz_device_count": [c_intp],
    "pz_last_error": [],
    "pz_version": [],
    "pz_blake2b512_batch": [vp, vp, u64, vp, u32],
    "pz_set_serial_threshold": [u64],
    "pz_set_host_threads": [u32],
    "pz_chain_set_options": [vp, vp],
    "pz_set_small_batch_threshold": [u64],
    "pz_dev_blake2b512_batch": [vp, vp, u64, vp, u32, vp],
    "pz_dev_blake2b512_fixed": [vp, u64, u64, u64, vp, u32, vp],
    "pz_validator_indices": [vp, vp, u64, u64, ctypes.c_int, vp, c_u64p],
    "pz_attesters_total_deposit": [vp, u64, c_u64p],
    "pz_calculate_rewards": [vp, vp, vp, u64, u64, u64, vp, vp, u64, c_intp],
    "pz_crosslink_tally": [vp, vp, u64, vp, vp, vp, u64, vp, u64, vp, vp],
    "pz_process_crosslinks": [vp, vp, u64, vp, vp, vp, vp, u64, vp, u64, vp, u64, u64, vp, vp, vp],
    "pz_shuffle_indices": [vp, vp, u64],
    "pz_dev_epoch_count": [vp, vp],
    "pz_dev_epoch_finish": [vp, vp],
    "pz_dev_epoch_gather_compact": [vp, vp, u32, u64, vp, vp],
    "pz_chain_new": [u64, ctypes.c_int, vp],
    "pz_chain_new_comm": [u64, vp, vp],
    "pz_chain_new_from_state": [vp, u64, vp, u64, ctypes.c_int, vp],
    "pz_chain_free": [vp],
    "pz_count_attestations": [vp, vp, u64, c_u64p],
    "pz_chain_process_blocks": [vp, vp, vp, u64, vp, vp, u64],
    "pz_chain_roots": [vp, vp, c_intp],
    "pz_chain_state_bytes": [vp, ctypes.c_int, vp, u64, c_u64p],
    "pz_chain_vote_totals": [vp, vp, vp, u64, c_u64p],
    "pz_chain_phase_times": [vp, vp, ctypes.c_int],
    "pz_dev_vote_tally": [vp, vp],
    "pz_vote_tally": [vp, vp, u64, vp, vp, vp, u64, vp, vp, u64, vp, u64, vp, u64, u64, vp],
    "pz_comm_vote_tally": [vp, vp, vp, u64, vp, vp, vp, u64, vp, vp, u64, vp, u64, vp, u64, u64, vp],
    "pz_wire_validators_bound": [u64, u64],
    "pz_wire_scratch_bytes": [u64],
    "pz_wire_validators": [vp, u64, u32, vp, u64, vp, c_u64p],
    "pz_dev_wire_validators": [vp, u64, u32, vp, vp, vp, vp, vp],
    "pz_check_attestations": [vp],
    "pz_rotate_validator_set": [vp, vp, vp, u64, u64],
    "pz_shuffle_validators_to_committees": [vp, vp, vp, u64, u64, u64, vp, vp, vp, vp, u64, c_u64p],
    "pz_wire_attestations_bound": [u64, u64, u64, u64],
    "pz_wire_attestations_scratch_bytes": [u64],
    "pz_wire_attestations": [vp, u64, u32, vp, u64, vp, c_u64p],
    "pz_dev_wire_attestations": [vp, u64, u32, vp, vp, vp, vp],
    "pz_dev_check_attestations": [vp, vp],
    "pz_shutdown": [],
    "pz_state_new": [u64, ctypes.c_int, vp],
    "pz_state_upload": [vp, vp, vp, vp],
    "pz_state_download": [vp, vp, vp, vp],
    "pz_state_validator_indices": [vp, u64, ctypes.c_int, vp, c_u64p],
    "pz_state_calculate_rewards": [vp, u64, u64, vp, vp, u64, c_intp],
    "pz_state_active_balance": [vp, u64, c_u64p],
    "pz_state_free": [vp],
    "pz_comm_unique_id": [vp],
    "pz_comm_init_rank": [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp],
    "pz_init_devices": [ctypes.c_int, vp, vp],
    "pz_comm_init_loopback": [ctypes.c_int, ctypes.c_int, vp],
    "pz_comm_init_shm": [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32, vp],
    "pz_comm_set_timing": [vp, ctypes.c_int],
    "pz_comm_collective_time": [vp, vp, vp],
    "pz_comm_size": [vp, c_intp, c_intp, c_intp],
    "pz_comm_device": [vp, ctypes.c_int, c_intp],
    "pz_comm_free": [vp],
    "pz_comm_blake2b512_batch": [vp, vp, vp, u64, vp, u32],
    "pz_epoch_state_new": [vp, ctypes.c_int, vp, vp],
    "pz_epoch_state_new_opts": [vp, ctypes.c_int, vp, vp, vp],
    "pz_epoch_state_step": [vp],
    "pz_epoch_state_sync": [vp],
    "pz_epoch_state_shard": [vp, ctypes.c_int, c_u64p, c_u64p, c_intp, vp],
    "pz_epoch_state_bind_stream": [vp, ctypes.c_int, vp],
    "pz_epoch_state_results": [vp, ctypes.c_int, vp, vp, vp, vp, vp],
    "pz_epoch_state_free": [vp],
    "pz_epoch_state_validators": [vp, ctypes.c_int, vp],
    "pz_epoch_state_layout": [vp, c_intp],
    "pz_epoch_state_columns": [vp, vp, vp],
    "pz_epoch_state_tallies": [vp],
    "pz_epoch_plan": [vp, ctypes.c_int, ctypes.c_int, c_u64p, c_u64p, c_intp],
}


class EpochBatch(ctypes.Structure):
    """Mirror of ``pz_epoch_batch`` (include/prysm_hip.h)."""
    _fields_ = [
        ("ninst", ctypes.c_uint32), ("nval", u64), ("val_offset", u64), ("nval_global", u64),
        ("kind", ctypes.c_int), ("balance", vp), ("start", vp), ("end", vp), ("dynasty", vp),
        ("total_deposit", vp), ("natt", ctypes.c_uint32), ("bits", vp), ("boffs", vp),
        ("max_inst_bytes", u64), ("pop_rank", ctypes.c_uint32), ("pop_world", ctypes.c_uint32),
        ("committee", vp), ("coffs", vp), ("att_comm", vp), ("att_shard", vp),
        ("nrec", ctypes.c_uint32), ("rec_dynasty", vp), ("winner", vp), ("vote", vp), ("total", vp),
        ("scal", vp), ("act_mask", vp), ("blk_cnt", vp), ("act_list", vp), ("scal_next", vp),
        ("cpos", vp), ("co_index", vp),
    ]


class EpochHost(ctypes.Structure):
    """Mirror of ``pz_epoch_host`` (include/prysm_hip.h)."""
    _fields_ = [
        ("ninst", ctypes.c_uint32), ("nval", u64), ("balance", vp), ("start", vp), ("end", vp),
        ("dynasty", vp), ("total_deposit", vp), ("natt", ctypes.c_uint32), ("bits", vp), ("boffs", vp),
        ("committee", vp), ("coffs", vp), ("ncomm", u64), ("att_comm", vp), ("att_shard", vp),
        ("nrec", ctypes.c_uint32), ("rec_dynasty", vp), ("layout", ctypes.c_uint32),
    ]


class ChainOptions(ctypes.Structure):
    """Mirror of ``pz_chain_options`` (include/prysm_hip.h)."""
    _fields_ = [("msg_batch", u64), ("tally_forms", u32)]


TALLY_PER_ATTESTATION, TALLY_BITS_ROWS, TALLY_ID_ROWS = 1, 2, 4  # pz_chain_options.tally_forms


class EpochOptions(ctypes.Structure):
    """Mirror of ``pz_epoch_options`` (include/prysm_hip.h)."""
    _fields_ = [("rebase_period", u64), ("window_only", ctypes.c_int)]


class VoteBatch(ctypes.Structure):
    """Mirror of ``pz_vote_batch`` (include/prysm_hip.h)."""
    _fields_ = [
        ("committee", vp), ("coffs", vp), ("att_comm", vp), ("bits", vp), ("boffs", vp),
        ("item_att", vp), ("item_slot", vp), ("nitems", u64), ("balance", vp), ("nval", u64),
        ("bitmaps", vp), ("words_per_slot", u64), ("totals", vp), ("err", vp),
        ("val_offset", u64), ("nval_global", u64),
    ]


class ValidatorCols(ctypes.Structure):
    """Mirror of ``pz_validator_cols`` (include/prysm_hip.h)."""
    _fields_ = [
        ("public_key", vp), ("withdrawal_shard", vp), ("withdrawal_address", vp),
        ("withdrawal_address_offs", vp), ("randao_commitment", vp), ("randao_commitment_offs", vp),
        ("balance", vp), ("start_dynasty", vp), ("end_dynasty", vp),
    ]


class AttestationCols(ctypes.Structure):
    """Mirror of ``pz_attestation_cols`` (include/prysm_hip.h)."""
    _fields_ = [
        ("slot", vp), ("shard_id", vp), ("justified_slot", vp), ("justified_block_hash", vp),
        ("justified_block_hash_offs", vp), ("shard_block_hash", vp), ("shard_block_hash_offs", vp),
        ("attester_bitfield", vp), ("attester_bitfield_offs", vp), ("oblique_parent_hashes", vp),
        ("oblique_offs", vp), ("oblique_first", vp), ("aggregate_sig", vp), ("aggregate_sig_first", vp),
    ]


class AttCheckBatch(ctypes.Structure):
    """Mirror of ``pz_att_check_batch`` (include/prysm_hip.h)."""
    _fields_ = [
        ("natt", u64), ("slot", vp), ("justified_slot", vp), ("shard_id", vp), ("n_oblique", vp),
        ("bits", vp), ("boffs", vp), ("block_slot", vp), ("last_justified_slot", u64),
        ("last_state_recalc", u64), ("n_recent", u64), ("narr", u64), ("arr_offs", vp), ("arr_shard", vp),
        ("arr_comm", vp), ("coffs", vp), ("status", vp), ("committee", vp), ("parents_start", vp),
        ("last_byte", vp),
    ]


SCAL_POP, SCAL_NACT, SCAL_ERR_XL, SCAL_ERR_RWD, SCAL_APPLIED, SCAL_NEXT_BAL, SCAL_MAXIDX1, SCAL_NOMATCH = range(8)
SCAL_COUNT = 8
KIND_ACTIVE, KIND_EXITED, KIND_QUEUED = 0, 1, 2
_RESTYPES = {"pz_last_error": ctypes.c_char_p, "pz_chain_free": None, "pz_set_serial_threshold": u64, "pz_set_host_threads": u32,
             "pz_shutdown": None, "pz_state_free": None, "pz_set_small_batch_threshold": u64, "pz_comm_free": None, "pz_epoch_state_free": None,
             "pz_wire_validators_bound": u64, "pz_wire_scratch_bytes": u64,
             "pz_wire_attestations_bound": u64, "pz_wire_attestations_scratch_bytes": u64}
SERIAL_DEFAULT = 65536        # the library's default serial threshold (bytes)
SERIAL_ON_GPU = (1 << 64) - 1  # pz_set_serial_threshold value that keeps every message on the GPU


class _Lib:
    def __init__(self):
        self._dll = None

    def _load(self):
        if self._dll is None:
            # the in-tree product build; no environment switch selects another one (tests marked
            # `ab` and tools/ point library_path at the A/B library before the first call)
            path = library_path
            if not os.path.exists(path):
                raise PzError(PZ_EDEVICE, "HIP library not built: %s (run __graft_entry__.build())" % path)
            dll = ctypes.CDLL(path)
            for name, args in SIGNATURES.items():
                fn = getattr(dll, name)
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, ctypes.c_int)
            self._dll = dll
        return self._dll

    @property
    def dll(self):
        return self._load()

    def call(self, name, *args):
        rc = getattr(self._load(), name)(*args)
        if rc != PZ_OK:
            raise PzError(rc, self._load().pz_last_error().decode())
        return rc


lib = _Lib()


def ptr(a):
    """Host pointer of a C-contiguous numpy array (None for empty)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data if a.size else None


def as_u8(buf):
    return np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf


def blake2b512_batch(messages, out_bytes=32):
    """Hash a list of byte strings on the GPU; returns a list of ``out_bytes``-byte digests."""
    n = len(messages)
    if n == 0:
        return []
    offsets = np.zeros(n + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(m) for m in messages], dtype=np.uint64)
    data = np.frombuffer(b"".join(bytes(m) for m in messages) + b"\0" * 16, dtype=np.uint8)
    out = np.empty(n * out_bytes, dtype=np.uint8)
    lib.call("pz_blake2b512_batch", ptr(data), ptr(offsets), n, ptr(out), out_bytes)
    raw = out.tobytes()
    return [raw[i * out_bytes:(i + 1) * out_bytes] for i in range(n)]


def blake2b512_csr(data, offsets, out_bytes=32):
    """Hash CSR messages (numpy uint8 data, uint64 offsets[n+1]); returns (n, out_bytes) uint8."""
    n = len(offsets) - 1
    out = np.empty((max(n, 0), out_bytes), dtype=np.uint8)
    if n > 0:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lib.call("pz_blake2b512_batch", ptr(data), ptr(offsets), n, ptr(out), out_bytes)
    return out


def set_serial_threshold(nbytes):
    """Messages of at least ``nbytes`` bytes are hashed on host threads by the batch entry
    points (serial chains); ``SERIAL_ON_GPU`` keeps all of them on the GPU.
    Returns the previous threshold."""
    return int(lib.dll.pz_set_serial_threshold(nbytes))


def serial_threshold_default():
    return SERIAL_DEFAULT


SMALL_BATCH_DEFAULT = 256  # compressions (serial_hash.h PZ_SMALL_BATCH_DEFAULT)


class small_batch_threshold:
    """Context manager: batches of at most ``compressions`` compressions are hashed on the
    calling thread (0: every batch on the GPU)."""

    def __init__(self, compressions):
        self.c = compressions

    def __enter__(self):
        self.old = int(lib.dll.pz_set_small_batch_threshold(self.c))
        return self

    def __exit__(self, *exc):
        lib.dll.pz_set_small_batch_threshold(self.old)


class serial_threshold:
    """Context manager form of :func:`set_serial_threshold`."""

    def __init__(self, nbytes):
        self.nbytes = nbytes

    def __enter__(self):
        self.old = set_serial_threshold(self.nbytes)
        return self

    def __exit__(self, *exc):
        set_serial_threshold(self.old)
