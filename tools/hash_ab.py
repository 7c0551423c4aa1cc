"""In-process A/B of the fixed-length BLAKE2b kernel variants (interleaved rounds, one
process, same buffers: cdna_hip_programming.md §5.4 rule 24).  GPU only."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import _lib, synth  # noqa: E402


def main(rounds=8, reps=10, n=1 << 20):
    dll = _lib.lib.dll
    dev = torch.device("cuda", 0)
    recs = synth.attestation_records_512(n, seed=2)
    d_in = torch.from_numpy(recs.reshape(-1)).to(dev)
    outs = {v: torch.empty(n * 32, dtype=torch.uint8, device=dev) for v in (0, 1)}
    s = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(s.cuda_stream)
    res = {0: [], 1: []}
    for r in range(rounds):
        for v in (0, 1) if r % 2 == 0 else (1, 0):
            dll.pz_debug_set_hash_variant(v)
            _lib.lib.call("pz_dev_blake2b512_fixed", d_in.data_ptr(), 512, 512, n, outs[v].data_ptr(), 32, sh)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                _lib.lib.call("pz_dev_blake2b512_fixed", d_in.data_ptr(), 512, 512, n, outs[v].data_ptr(), 32, sh)
            e1.record(s)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / reps)
    same = bool(torch.equal(outs[0], outs[1]))
    print(json.dumps({"variant0_plain_ms": sorted(res[0]), "variant1_persistent_dma_ms": sorted(res[1]),
                      "median_ms": {k: float(np.median(v)) for k, v in res.items()}, "identical": same}))


if __name__ == "__main__":
    main()
