"""The one-process-per-rank form of the library's sharded paths, run for real: separate
processes, each calling the C ABI (pz_chain_new_comm, pz_epoch_state) and meeting the others
in the communicator's collectives, as bench.py's ranks do under torchrun.  RCCL refuses two
ranks on one device, so on the one-GPU test box the ranks share cuda:0 over the SHM
communicator (pz_comm_init_shm): the same collective call sequence as the RCCL backend
(comm.hip), checked for divergence by the group -- a rank whose host-side decisions differ
from the others' fails loudly instead of hanging (blockchain/core.go:300-345,411-418;
blockchain/service.go:229 run the walk these processes each repeat).

Every rank's results are checked: the chain's against the C restatement of the block
pipeline (oracle/c/replay_ref.c), the epoch's against the numpy oracle."""
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

from prysm_amd import _lib, casper, synth

from epoch_ref_helpers import oracle_epoch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def run_ranks(mode, world, indir, opts, timeout=300):
    """Start `world` worker processes (tests/shm_worker.py) on one SHM group; their result
    files, rank-ordered.  A rank that fails or hangs fails the test with its output."""
    name = "/pz_t_%d_%s" % (os.getpid(), uuid.uuid4().hex[:8])
    outs = [os.path.join(indir, "%s_rank%d.npz" % (mode, r)) for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "shm_worker.py"), mode, name, str(world),
                               str(r), indir, outs[r], json.dumps(opts)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            logs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        # a rank 0 killed between creating the segment and every rank joining leaves it behind
        if os.path.exists("/dev/shm" + name):
            os.unlink("/dev/shm" + name)
    for r, p in enumerate(procs):
        assert p.returncode == 0, "rank %d exited %s:\n%s" % (r, p.returncode, logs[r][-3000:])
    return [np.load(o) for o in outs]


def _chain_files(tmp_path, nval, blocks):
    from prysm_amd.blockchain import serialize_blocks
    data, offs = serialize_blocks(blocks)
    np.save(tmp_path / "chain_data.npy", np.ascontiguousarray(data, dtype=np.uint8))
    np.save(tmp_path / "chain_offs.npy", np.ascontiguousarray(offs, dtype=np.uint64))
    return data, offs


def _roots(z):
    r = {k: bytes.fromhex(v) for k, v in json.loads(str(z["roots"])).items()}
    r["vote_totals"] = {bytes.fromhex(k): v for k, v in json.loads(str(z["vote_totals"])).items()}
    return r


@pytest.mark.parametrize("world", [2, 3])
def test_shm_processes_replay_configs4_chain_vs_c_port(world, tmp_path):
    """BASELINE configs[4] as ONE chain over `world` processes (pz_chain_new_comm over
    pz_comm_init_shm): each process walks the 10,000 blocks itself and holds its validator
    range of the balances, the vote cache and every epoch; the 64 justification totals and the
    epoch's partial sums meet in the collectives.  Every rank's blocks, attestations, four roots
    and vote-cache totals bit-exact against the C restatement."""
    from replay_port_helpers import mismatches, port_replay
    nval = 65536
    data, offs = _chain_files(tmp_path, nval, synth.chain_blocks(nval, 10000, seed=6))
    res = run_ranks("chain", world, str(tmp_path), {"nval": nval})
    z0 = res[0]
    port_out, port_roots = port_replay(data, offs, nval, len(z0["ar"]))
    for r, z in enumerate(res):
        assert int(z["br"]["transition"].sum()) == 156
        assert mismatches(z["br"], z["ar"], _roots(z), port_out, port_roots) == [], "rank %d" % r


def test_shm_processes_golden_chain_world3(tmp_path):
    """The golden 1,024-validator chain (configs[0]) over three processes: 1,024 validators in
    64-aligned ranges gives ranks of 384, 384 and 256 validators."""
    import json as _json
    with open(os.path.join(HERE, "golden", "replay_n1024.json")) as f:
        g = _json.load(f)
    _chain_files(tmp_path, g["nval"], synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"]))
    res = run_ranks("chain", 3, str(tmp_path), {"nval": g["nval"]})
    for z in res:
        roots = _roots(z)
        for k, v in g["roots"].items():
            assert roots[k].hex() == v, k


def _epoch_files(tmp_path, n, B, inactive=False, seed=5):
    shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(n, dtype=np.uint32))
    inst = synth.epoch_batch(n, B, seed=seed, shuffled=shuffled)
    if inactive:  # rank != index: the active masks' all-gather and the global compaction
        rng = np.random.default_rng(1)
        inst["start"][:, rng.random(n) < 0.1] = 7
        inst["end"][:, rng.random(n) < 0.1] = 1
    np.savez(tmp_path / "epoch_inst.npz", **{k: np.asarray(v) for k, v in inst.items()})
    return inst


def _check_epoch(res, inst, steps, world):
    held = []
    for s in range(steps):
        want = [oracle_epoch(inst, b) for b in range(inst["ninst"])]
        for r, z in enumerate(res):
            idx = z["idx"]
            if s == 0:
                held.append(idx)
            for b, (nb, applied, nxt, v, t, w) in enumerate(want):
                assert bool(z["scal%d" % s][b, _lib.SCAL_APPLIED]) == applied, (r, s, b)
                np.testing.assert_array_equal(z["bal%d" % s][b], nb[idx])
                assert int(z["scal%d" % s][b, _lib.SCAL_NEXT_BAL]) == nxt, (r, s, b)
                np.testing.assert_array_equal(z["vote%d" % s][b], v)
                np.testing.assert_array_equal(z["total%d" % s][b], t)
                np.testing.assert_array_equal(z["win%d" % s][b], w)
        for b, (nb, *_rest) in enumerate(want):
            inst["balance"][b] = nb
    np.testing.assert_array_equal(np.sort(np.concatenate(held)), np.arange(inst["nval"]))


def test_shm_processes_epoch_configs3(tmp_path):
    """BASELINE configs[3]: 1,048,576 validators sharded over two processes (committee-aligned
    ranges, the one-pass step, one grouped collective per part), two steps of two instances,
    every rank's balances, next-cycle totals, tallies and winners against the oracle."""
    inst = _epoch_files(tmp_path, 1 << 20, 2)
    res = run_ranks("epoch", 2, str(tmp_path), {"steps": 2})
    assert all(bool(z["one_pass"]) for z in res)
    _check_epoch(res, inst, 2, 2)


@pytest.mark.parametrize("layout", ["auto", "index"])
def test_shm_processes_epoch_inactive_world3(layout, tmp_path):
    """Some validators inactive (rank != index): the two-part pipeline, the active masks'
    all-gather and the global compaction over three processes."""
    inst = _epoch_files(tmp_path, 5000, 3, inactive=True)
    res = run_ranks("epoch", 3, str(tmp_path), {"steps": 2, "layout": layout})
    assert not any(bool(z["one_pass"]) for z in res)
    _check_epoch(res, inst, 2, 3)
