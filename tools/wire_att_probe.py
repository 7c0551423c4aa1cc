"""Times pz_dev_wire_attestations alone on the bench's wire_att workload (the 1,048,576
config-2 AttestationRecords from their SoA columns) with HIP events, and checks the bytes
against synth.attestation_records_512.  Usage: wire_att_probe.py [reps] [n]."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prysm_amd import _lib, synth, wire  # noqa: E402

if os.environ.get("PZ_PROBE_LIB"):  # A/B against another build of the library
    _lib.library_path = os.environ["PZ_PROBE_LIB"]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    cols = synth.attestation_columns_512(n, seed=2)
    t = {k: torch.from_numpy(cols[k].view(np.int64) if cols[k].dtype == np.uint64 else cols[k]).cuda()
         for k in wire.ATT_COLS}
    c = _lib.AttestationCols(*[t[k].data_ptr() for k in wire.ATT_COLS])
    ne, ns = int(cols["oblique_first"][-1]), int(cols["aggregate_sig_first"][-1])
    nbytes = sum(int(cols[k][-1]) for k in ("justified_block_hash_offs", "shard_block_hash_offs",
                                            "attester_bitfield_offs", "oblique_offs"))
    out = torch.zeros(int(_lib.lib.dll.pz_wire_attestations_bound(n, nbytes, ne, ns)) + 16, dtype=torch.uint8,
                      device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    scr = torch.empty(int(_lib.lib.dll.pz_wire_attestations_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    sh = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def run():
        _lib.lib.call("pz_dev_wire_attestations", ctypes.byref(c), n, 0, out.data_ptr(), offs.data_ptr(),
                      scr.data_ptr(), sh)

    for _ in range(200):  # clocks ramp over the first ~100 launches
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    dll = _lib.lib.dll
    if hasattr(dll, "pz_debug_set_att_write_variant"):  # same-process A/B (PZ_PROBE_LIB=build/ab/...)
        # product / byte-loop sig varints / sizing loops (r5 first form) / aligned-dword stage;
        # WATT_VARIANTS=a,b,... another list
        vs = [int(x) for x in os.environ.get("WATT_VARIANTS", "0,8,7,6,0,8,7").split(",")]
        for v in vs:
            dll.pz_debug_set_att_write_variant(v)
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ok_v = bool(np.array_equal(out[:n * 512].cpu().numpy(), synth.attestation_records_512(n, seed=2).reshape(-1)))
            print("  variant %d  encode %.3f ms  parity=%s" % (v, e0.elapsed_time(e1) / reps, ok_v), flush=True)
        dll.pz_debug_set_att_write_variant(0)
        run()
    # the CSR hash kernel over the encoded records (the encode + hash leg's second launch)
    dig = torch.empty(n * 32, dtype=torch.uint8, device="cuda")

    def run_hash():
        _lib.lib.call("pz_dev_blake2b512_batch", out.data_ptr(), offs.data_ptr(), n, dig.data_ptr(), 32, sh)

    for _ in range(20):
        run_hash()
    e0.record()
    for _ in range(reps):
        run_hash()
    e1.record()
    torch.cuda.synchronize()
    hms = e0.elapsed_time(e1) / reps
    print("csr hash: %.3f ms  %.2f G records/s" % (hms, n / hms / 1e6), flush=True)
    want = synth.attestation_records_512(n, seed=2).reshape(-1)
    ok = bool(np.array_equal(out[:want.size].cpu().numpy(), want))
    print("wire_att encode: %d records  %.3f ms  %.1f M records/s  parity=%s" % (n, ms, n / ms / 1e3, ok), flush=True)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
