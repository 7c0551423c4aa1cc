"""Steady-state timing of the fixed-length hash kernel: 300 back-to-back launches over
1,048,576 x 512 B, average launch time per window of 10 (shows clock ramp / throttling)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from prysm_amd import _lib, synth  # noqa: E402


def main(n=1 << 20, windows=30, per=10):
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(synth.attestation_records_512(n, seed=2).reshape(-1)).to(dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(s.cuda_stream)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(windows + 1)]
    torch.cuda.synchronize()
    evs[0].record(s)
    for w in range(windows):
        for _ in range(per):
            _lib.lib.call("pz_dev_blake2b512_fixed", d_in.data_ptr(), 512, 512, n, d_out.data_ptr(), 32, sh)
        evs[w + 1].record(s)
    torch.cuda.synchronize()
    ms = [evs[w].elapsed_time(evs[w + 1]) / per for w in range(windows)]
    print("per-launch ms by window:", " ".join("%.3f" % x for x in ms))
    print("min %.3f  median %.3f  max %.3f  -> %.2f G hashes/s at median" % (min(ms), sorted(ms)[len(ms) // 2], max(ms),
                                                                            n / sorted(ms)[len(ms) // 2] / 1e6))


if __name__ == "__main__":
    main()
