"""One rank of a multi-process run over the SHM communicator (pz_comm_init_shm): the form the
bench takes under torchrun -- one process per rank, each calling the C ABI and meeting the
others in its collectives -- with every rank on cuda:0.  Started by
tests/test_shm_multiprocess_gpu.py and bench.py's gloo rehearsal checker; writes its results
to an .npz the parent compares with the oracle.

usage: shm_worker.py chain|epoch NAME WORLD RANK IN_DIR OUT_NPZ [extra json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def chain(comm, indir, out, opts):
    from prysm_amd.blockchain import BeaconChain
    data = np.load(os.path.join(indir, "chain_data.npy"))
    offs = np.load(os.path.join(indir, "chain_offs.npy"))
    ch = BeaconChain(int(opts["nval"]), comm=comm)
    br, ar = ch.process_serialized(data, offs)
    roots = ch.roots()
    vt = roots.pop("vote_totals", None)
    np.savez(out, br=br, ar=ar, roots=json.dumps({k: v.hex() for k, v in roots.items()}),
             vote_totals=json.dumps({k.hex(): int(v) for k, v in vt.items()}))


def epoch(comm, indir, out, opts):
    from prysm_amd.native import NativeEpoch
    z = np.load(os.path.join(indir, "epoch_inst.npz"))
    inst = {k: (int(z[k]) if z[k].ndim == 0 else z[k]) for k in z.files}
    ne = NativeEpoch(inst, device=0, comm=comm, layout=opts.get("layout", "auto"))
    res = {"one_pass": np.array(ne.one_pass), "committee_order": np.array(ne.committee_order)}
    lo, hi, _, _ = ne.shard(0)
    res["range"] = np.array([lo, hi], dtype=np.uint64)
    res["idx"] = ne.validators()
    for s in range(int(opts.get("steps", 1))):
        ne.step()
        ne.sync()
        ne.tallies()  # a collective: complete vote/total on every rank
        bal, scal, vote, total, win = ne.results()
        res.update({"bal%d" % s: bal, "scal%d" % s: scal, "vote%d" % s: vote, "total%d" % s: total, "win%d" % s: win})
    ne.free()
    np.savez(out, **res)


def main():
    mode, name, world, rank, indir, out = sys.argv[1:7]
    opts = json.loads(sys.argv[7]) if len(sys.argv) > 7 else {}
    world, rank = int(world), int(rank)
    from prysm_amd import _lib
    from prysm_amd.native import Comm
    _lib.lib.call("pz_init", 0)
    comm = Comm.shm(name, world, rank, 0, timeout_ms=int(opts.get("timeout_ms", 120000)))
    {"chain": chain, "epoch": epoch}[mode](comm, indir, out, opts)
    comm.free()
    print("rank %d of %d: %s done" % (rank, world, mode), flush=True)


if __name__ == "__main__":
    main()
