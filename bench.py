#!/usr/bin/env python3
"""Benchmark of the MI355X state-transition hot path (BASELINE.json metric).

Headline (``value``): batched BLAKE2b-512[:32] hashes/s over 1,048,576 synthetic 512-byte
proto3 AttestationRecord encodings per GPU (BASELINE.json configs[1]), inputs resident in
HBM, one ``pz_dev_blake2b512_fixed`` launch per step.  With ``--gpus N`` (torchrun, one
process per GPU) each rank hashes its own batch (message batches shard with no collective:
``scaling`` = "weak"), and ``value`` = all records hashed / max-over-ranks wall time.

Also reported on the same line: ``roofline`` (the hash kernel's VALU roofline fraction,
kernel time from HIP events on the launch stream) and ``cpu_baseline`` (the oracle's C
restatement on this host's cores, rank 0 at N=1 only).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "validator-epoch updates/sec + hashes/sec (1/2/4/8 MI355X) vs Go CPU ref"

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters")
N_CU = 256
CLK_HZ = 2.4e9
LANE_OPS_PER_CU_CLK = 128          # 4 SIMD-32 x 32 lanes (wave64 issues over 2 cycles)
VALU_PEAK = N_CU * LANE_OPS_PER_CU_CLK * CLK_HZ   # 78.6e12 32-bit lane-ops/s
HBM_PEAK = 8.0e12                  # B/s (spec)
# VALU roofline of one BLAKE2b compression on gfx950.  The ISA-minimal G is
# 6 x v_lshl_add_u64 (64-bit add) + 8 x v_xor_b32 + 6 x v_alignbit_b32 (rotr 24/16/63; rotr 32
# is a register swap), and the compression adds 32 v_xor_b32 for h ^= v[i] ^ v[i+8].  On
# gfx950 these do not issue at one rate: measured throughput relative to v_xor_b32 (full rate,
# tools/valu_rates.hip -> profiles/r01/valu_rates.txt) is 0.304 for v_lshl_add_u64 and 0.602
# for v_alignbit_b32.  Work is therefore counted in full-rate issue slots (lane-ops a
# full-rate instruction would retire) and priced against the spec full-rate peak.
REL_COST = {"v_lshl_add_u64": 1 / 0.304, "v_xor_b32": 1.0, "v_alignbit_b32": 1 / 0.602}
SLOTS_PER_G = 6 * REL_COST["v_lshl_add_u64"] + 8 * REL_COST["v_xor_b32"] + 6 * REL_COST["v_alignbit_b32"]
OPS_PER_COMPRESSION = 96 * SLOTS_PER_G + 32            # ~3652 full-rate slots


def warm_clocks(step, torch, dev, ms):
    """Run ``step`` back to back for ``ms`` milliseconds of wall time (untimed): from idle the
    GPU clock ramps over ~100 ms of sustained load (first launches of the hash kernel take
    0.40 ms, steady state 0.24 ms), so W short warmup steps alone would time the ramp."""
    if ms <= 0:
        return
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            step()
        torch.cuda.synchronize(dev)


def host_info():
    """The host the CPU baselines ran on (print nproc and the CPU model)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model)
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return {"nproc": os.cpu_count(), "affinity": aff, "model": model,
            "threads_all_cores": max(1, min(16, aff)),
            "note": "all-cores lines use min(16, affinity) threads: the CPU share of one GPU on the bench boxes"}


def max_over_ranks(x, torch, dist, dev):
    """MAX of a host float over the ranks (a device tensor for RCCL, a host one for gloo)."""
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([x], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--clock-warm-ms", type=float, default=400.0,
                   help="untimed back-to-back launches before the warmup steps: MI355X clocks ramp "
                        "from idle over ~100 launches of this kernel (tools/hash_steady.py)")
    p.add_argument("--records", type=int, default=1 << 20)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="collective backend at N > 1 (gloo: rehearsal with ranks sharing a GPU)")
    p.add_argument("--cpu-replay-blocks", type=int, default=1040,
                   help="blocks of the replay chain the CPU baseline (oracle/c/replay_ref.c) processes (~6 s)")
    p.add_argument("--no-epoch", action="store_true")
    p.add_argument("--epoch-layout", default="auto", choices=["auto", "twopass", "index"],
                   help="auto: committee order when every validator is active and the committees partition "
                        "the set, one-pass step (pz_epoch_host.layout); twopass: that layout, two-pass step; "
                        "index: validator-index order")
    p.add_argument("--no-epoch-cold", action="store_true",
                   help="skip the epoch legs' cold-data rotation over 4 instance sets")
    p.add_argument("--no-replay", action="store_true")
    p.add_argument("--no-wire", action="store_true")
    p.add_argument("--no-attcheck", action="store_true")
    p.add_argument("--replay-blocks", type=int, default=10000,
                   help="blocks per sync replay (BASELINE configs[4]; 65,536 validators)")
    p.add_argument("--epoch-validators", type=int, default=0,
                   help="validators per epoch instance (default: 65,536 at N=1, 1,048,576 at N>1)")
    p.add_argument("--epoch-instances", type=int, default=0,
                   help="independent epoch instances per step (default: 16.7M validator-epochs/step)")
    p.add_argument("--single-process", action="store_true",
                   help="one process drives --gpus devices through pz_init_devices (ncclCommInitAll, grouped "
                        "RCCL calls over per-device streams): the form a Go node links (service.go:229)")
    p.add_argument("--no-single-process-leg", action="store_true",
                   help="at N > 1 under torchrun, skip rank 0's --single-process child run after the main legs")
    p.add_argument("--single-process-timeout", type=float, default=300.0)
    p.add_argument("--launch-selftest", action="store_true",
                   help="launcher check: every rank prints its RANK/WORLD_SIZE and exits before any GPU call")
    return p.parse_args()


def launch_ranks(args):
    """``--gpus N`` (N > 1) without a launcher around this process (WORLD_SIZE unset): start
    ``torch.distributed.run`` with N ranks as a CHILD process, forward its output and return
    its exit code.  Nothing GPU-related has been imported or touched here (argparse only), so
    the ranks are the only processes that initialise the GPUs; the parent just waits."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    env["PZ_BENCH_LAUNCH"] = "torchrun child of bench.py --gpus %d" % args.gpus
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench: %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


# Algorithmic HBM bytes per validator-epoch: 16 B start/end
# dynasty + 16 B balance read-modify-write + 1/8 B last-bitfield bit + 1/8 B committee bitfield
# popcount + 12 B crosslink committee gather (u32 member + u64 balance).
EPOCH_BYTES_PER_VALIDATOR = 44.25
COLD_STATE_BYTES = 800_000_000  # the epoch cold leg's streamed state, >= 3x the 256 MiB Infinity Cache


def epoch_layout_bytes(inst, de):
    """Bytes per validator-epoch the one-pass committee-order step must move, from
    the widths the state actually uploaded (pz_epoch_state_columns): the balance read and
    written (2 x 4 B as u32 offsets from a per-instance base, or 2 x 8 B), the {start, end}
    dynasties (4 B in the 16-bit saturated column, 8 B in the 32-bit one, else 16 B), and the
    instance's bitfields once (their bytes / nval); co_index is shared by the instances (L2).
    None for the other layouts (SURVEY.md §8d's 44.25 B stays their model)."""
    if de is None or not getattr(de, "one_pass", False):
        return None
    bits = float(inst["boffs"][-1]) / (inst["ninst"] * inst["nval"])
    return 2 * de.balance_bytes + de.dynasty_bytes + bits


def epoch_bytes_model(de, bpv):
    if bpv is None:
        return "SURVEY.md §8d: 44.25 B per validator-epoch"
    return ("the one-pass committee-order layout's bytes: %.2f B per validator-epoch (balance read + write "
            "2 x %d, {start, end} %d, bitfields %.2f; DESIGN.md §3)"
            % (bpv, de.balance_bytes, de.dynasty_bytes, bpv - 2 * de.balance_bytes - de.dynasty_bytes))


HASH_KERNEL = "pz_b2b_fixed_persistent_kernel"
CPU_SAMPLE_S = 8.0  # seconds of CPU work per cpu_baseline leg (three legs: ~25 s in all)


def native_comm(dist, rank, world, local, shm=False):
    """The library's own communicator over the torchrun ranks.  RCCL: rank 0's ncclUniqueId
    (pz_comm_unique_id) reaches the others through the launcher's TCP store.  ``shm`` (the
    gloo rehearsal, ranks sharing one GPU, which RCCL refuses): pz_comm_init_shm -- the same
    collective call sequence staged through host memory, checked for divergence -- on a
    shared-memory group whose name rank 0 passes through the store."""
    from prysm_amd.native import Comm
    store = dist.distributed_c10d._get_default_store()
    if shm:
        if rank == 0:
            store.set("pz_shm_name", "/pz_bench_%d_%d" % (os.getpid(), int(time.time() * 1e3) % 1000000))
        name = store.get("pz_shm_name").decode()
        if rank == 0:  # (the library unlinks it once every rank has joined; this covers a failed join)
            import atexit
            atexit.register(lambda: os.path.exists("/dev/shm" + name) and os.unlink("/dev/shm" + name))
        return Comm.shm(name, world, rank, local, timeout_ms=300000)
    if rank == 0:
        store.set("pz_comm_uid", Comm.unique_id())
    uid = store.get("pz_comm_uid")
    return Comm.rank(uid, world, rank, local)


def all_ranks(ok, torch, dist, dev):
    """True iff ``ok`` holds on every rank (MIN all-reduce; every rank must call it)."""
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item() > 0.5)


def hash_spot_check(records_np, d_out, k=65536):
    """This rank's digests of its first and last ``k`` records against the C port (the
    checker at N > 1, where the full-batch check of the N = 1 cpu_baseline leg does not run)."""
    from oracle import cport
    n = records_np.shape[0]
    k = min(k, n)
    got = d_out.view(n, 32)
    ok = True
    for lo in sorted({0, n - k}):
        want = cport.hash_fixed(np.ascontiguousarray(records_np[lo:lo + k]), 512, 32)
        ok &= bool(np.array_equal(got[lo:lo + k].cpu().numpy(), want))
    return ok, "records [0, %d) and [%d, %d)" % (k, n - k, n)


def epoch_leg(args, torch, dist, dev, rank, world, nval=None, ninst=None, baseline=True, comm=None):
    """BASELINE configs[2] (N=1: 65,536 validators, B instances per step) / configs[3]
    (N>1: 1,048,576 validators sharded over the ranks, RCCL all-reduce of the sums).

    The step is pz_epoch_state_step: kernels and RCCL collectives enqueued by the C ABI on
    the library's streams (the path a cgo caller links)."""
    from prysm_amd import casper, synth
    from prysm_amd.native import NativeEpoch

    nval = nval or args.epoch_validators or (65536 if world == 1 else 1 << 20)
    # throughput mode: 16.7 M validator-epochs per GPU per step at every N (weak scaling; at
    # N > 1 each rank holds 1/N of every 1M-validator instance and B grows with N)
    ninst = ninst or args.epoch_instances or max(1, (1 << 24) * world // nval)
    seed_a = b"A" + bytes(31)  # common.Hash{'A'} (casper/sharding_test.go:57)
    shuffled = casper.shuffle_indices(seed_a, np.arange(nval, dtype=np.uint32))
    inst = synth.epoch_batch(nval, ninst, seed=3, shuffled=shuffled)
    native = True
    de = NativeEpoch(inst, device=dev.index, comm=comm if world > 1 else None, layout=args.epoch_layout)
    lo, hi, _, sp = de.shard(0)
    stream = torch.cuda.ExternalStream(sp, device=dev)
    step = de.step
    # a fixed count (not a time budget): at N > 1 every step holds collectives, so all ranks
    # must run the same number of them
    for _ in range(args.warmup + (30 if args.clock_warm_ms > 0 else 0)):
        step()
    torch.cuda.synchronize(dev)
    stream.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # one event pair around the K back-to-back steps: the average launch duration without
    # per-step event packets between the launches (what rocprofv3's kernel trace averages)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    stream.synchronize()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        wall = max_over_ranks(wall, torch, dist, dev)
    units = nval * ninst * args.steps
    local_units = (hi - lo) * ninst
    one_pass = native and de.one_pass
    lay = epoch_layout_bytes(inst, de if native else None)
    bpv = lay if lay is not None else EPOCH_BYTES_PER_VALIDATOR
    achieved = local_units * bpv / (step_ms * 1e-3)
    survey = local_units * EPOCH_BYTES_PER_VALIDATOR / (step_ms * 1e-3)
    workload = {(65536, 256): "epoch65k", (1 << 20, 16): "epoch1m"}.get((nval, ninst)) if world == 1 else None
    traffic = pmc_traffic(["pz_epoch_*"], workload) if workload else None
    out = {
        "metric": "validator-epoch updates/s",
        "value": units / wall,
        "unit": "validator-epochs/s",
        "ms_per_step": wall / args.steps * 1e3,
        "scaling": "weak",
        "config": {"workload": "stateRecalc data-parallel part: crosslink tallies+winners, attester "
                               "popcount, CalculateRewards, next-cycle balance (BASELINE configs[%d])"
                               % (2 if (world == 1 and nval != 1 << 20) else 3),
                   "validators": nval, "instances_per_step": ninst, "attestations_per_instance": inst["natt"],
                   "parallelism": (("committee-aligned validator shard x%d + one grouped RCCL collective per "
                                    "part (sum of scalars, min of winners)" % world) if (world > 1 and native and
                                                                                       de.one_pass)
                                   else ("validator-shard x%d + RCCL all-reduce" % world) if world > 1
                                   else "single GPU"),
                   "layout": (("committee order, one-pass step" if de.one_pass else
                               "committee order, two-pass step" if de.committee_order else "index order")
                              if native else "index order"),
                   "path": ("pz_epoch_state_step (C ABI: HIP kernels + the library's RCCL communicator)"
                            if native else "")},
        "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK,
                     "bytes_model": epoch_bytes_model(de, lay),
                     "survey_model": {"bytes_per_validator_epoch": EPOCH_BYTES_PER_VALIDATOR,
                                      "achieved": survey / 1e9, "frac": survey / HBM_PEAK,
                                      "note": "SURVEY.md §8d's figure prices a 12 B committee gather and 16 B of "
                                              "start/end the committee-order layout does not move"},
                     "traffic": traffic,
                     "traffic_source": ("%s (every pz_epoch_* kernel of the %d x %d step)"
                                        % (pmc_summary_path(workload), nval, ninst)) if workload else None,
                     "traffic_frac": (traffic / (step_ms * 1e-3) / HBM_PEAK) if traffic else None,
                     "kernel": ("epoch step: pz_epoch_window_b32_s16 (ONE launch: the bit count shared by an "
                                "instance's blocks, the last bitfield into LDS by DMA, per-instance committee pieces "
                                "with their vote bits read beside the stream, classify, crosslink tallies per "
                                "committee in LDS, winners, rewards on the u32 balance offsets, next-cycle sum); "
                                "device time of the whole step" if one_pass else
                                "epoch step (count+winner+compact+reward, device time of the whole step)"),
                     "step_device_ms": step_ms,
                     "algorithmic_bytes_per_launch": local_units * bpv},
    }
    if world > 1 and native and comm is not None:
        out["collectives"] = epoch_collective_time(args, de, comm, stream)
    del de
    if world == 1 and native and workload and not args.no_epoch_cold:
        out["cold"] = epoch_cold(args, torch, dev, nval, ninst, shuffled, workload, bpv=bpv)
    if rank == 0 and world == 1:
        out["parity"] = epoch_parity(inst, dev)
    elif world > 1 and native:
        ok, what = epoch_parity_sharded(inst, dev, comm)
        out["parity"] = "%s, on every rank: %s" % (what, all_ranks(ok, torch, dist, dev))
    if world == 1 and baseline:
        out["single_instance"] = epoch_single_instance(args, torch, dev, nval, shuffled)
    if rank == 0 and world == 1 and not args.no_cpu_baseline and baseline:
        out["cpu_baseline"] = epoch_cpu_baseline(inst)
    return out


def epoch_collective_time(args, de, comm, stream):
    """After the timed loop: ``args.steps`` more steps with the communicator's collectives
    bracketed by HIP events on its stream (pz_comm_set_timing), so the timed loop itself
    carries no extra event packets.  The collectives' own device time per step; the step's
    device time beside it (the part of the collectives the two-part pipeline does not hide is
    at most their sum)."""
    import torch
    for _ in range(2):
        de.step()
    stream.synchronize()
    comm.set_timing(True)
    comm.collective_time()  # restart the sum
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        de.step()
    e1.record(stream)
    stream.synchronize()
    ms, count = comm.collective_time()
    comm.set_timing(False)
    return {"ms_per_step": ms / args.steps, "per_step": count / args.steps,
            "step_device_ms_same_pass": e0.elapsed_time(e1) / args.steps,
            "what": "device time of the communicator's collectives (HIP events on its stream of this rank, "
                    "rank 0 reported), %d steps after the timed loop" % args.steps}


def epoch_parity_sharded(inst, dev, comm):
    """The checker at N > 1: instance 0 of the timed workload, one fresh step through a
    sharded pz_epoch_state over the same communicator (a collective: every rank builds and
    steps it), each rank's validator range (balances, next-cycle total, applied flag) and the
    complete tallies and winners against oracle/epoch_np."""
    from prysm_amd import _lib, synth
    from prysm_amd.native import NativeEpoch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from epoch_ref_helpers import oracle_epoch

    one = synth.epoch_instances(inst, 1)
    de = NativeEpoch(one, device=dev.index, comm=comm)
    de.step()
    de.sync()
    de.tallies()
    bal, scal, vote, total, win = de.results()
    idx = de.validators()
    de.free()
    nb, applied, nxt, v, t, w = oracle_epoch(one, 0)
    ok = (np.array_equal(bal[0], nb[idx]) and bool(scal[0, _lib.SCAL_APPLIED]) == applied
          and int(scal[0, _lib.SCAL_NEXT_BAL]) == nxt and np.array_equal(vote[0], v)
          and np.array_equal(total[0], t) and np.array_equal(win[0], w))
    return ok, ("instance 0 of the timed workload, one step sharded over the %d ranks, each rank's %d validators "
                "bit-exact vs oracle/epoch_np" % (comm.world, len(idx)))


def epoch_cold(args, torch, dev, nval, ninst, shuffled, workload, nsets=4, bpv=None):
    """The same step with the timed steps rotated over ``nsets`` distinct instance sets (each
    ~400 MB; together far above the 256 MiB Infinity Cache), all bound to one stream, so every
    step reads its state from HBM: the epoch against HBM, not against the cache the
    back-to-back steps of one set enjoy."""
    from prysm_amd import synth
    from prysm_amd.native import NativeEpoch

    stream = torch.cuda.Stream(device=dev)  # a real stream: a null handle means "the state's own"
    sets = []
    k = 0
    while k < nsets:
        inst_k = synth.epoch_batch(nval, ninst, seed=3 + k, shuffled=shuffled)
        de = NativeEpoch(inst_k, device=dev.index)
        de.bind_stream(stream.cuda_stream)
        sets.append(de)
        if k == 0:  # enough sets that the streamed state is >= 3x the 256 MiB Infinity Cache
            if bpv is None:
                bpv = epoch_layout_bytes(inst_k, de) or EPOCH_BYTES_PER_VALIDATOR
            sets_bb = de.balance_bytes
            state_bytes = nval * ninst * (de.balance_bytes + de.dynasty_bytes)
            nsets = max(nsets, -(-COLD_STATE_BYTES // state_bytes))
        k += 1
    steps = max(nsets, (args.steps + nsets - 1) // nsets * nsets)
    for _ in range(2):
        for de in sets:
            de.step()
    stream.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(steps):
        sets[i % nsets].step()
    ev1.record(stream)
    stream.synchronize()
    wall = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / steps
    for de in sets:
        de.free()
    units = nval * ninst
    alg = units * bpv
    traffic = pmc_traffic(["pz_epoch_*"], workload + "_cold")
    yard = cold_stream_yardstick(torch, dev, units, nsets, steps)
    yard_layout = cold_layout_yardstick(torch, dev, units, nsets, steps, sets_bb)
    return {"what": "%d steps rotated over %d distinct %d x %d instance sets (%.2f GB of streamed validator "
                    "state: balances and the {start, end} column), one stream"
                    % (steps, nsets, nval, ninst, nsets * state_bytes / 1e9),
            "value": units * steps / wall, "unit": "validator-epochs/s", "step_device_ms": step_ms,
            "frac": alg / (step_ms * 1e-3) / HBM_PEAK,
            "survey_frac": units * EPOCH_BYTES_PER_VALIDATOR / (step_ms * 1e-3) / HBM_PEAK,
            "traffic": traffic, "traffic_source": pmc_summary_path(workload + "_cold") if traffic else None,
            "traffic_frac": (traffic / (step_ms * 1e-3) / HBM_PEAK) if traffic else None,
            "yardstick": yard, "yardstick_layout": yard_layout}


def cold_stream_yardstick(torch, dev, units, nsets, steps):
    """What a stock elementwise kernel reaches on the same traffic shape, cold: per element 3
    reads + 1 write of 8 B (the epoch's balance/start/end in, balance out) -- torch's
    ``addcmul_`` on float64, rotated over ``nsets`` distinct sets on one stream.  The epoch's
    counter-byte fraction is read against this, not only against the 8 TB/s spec."""
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        sets = [[torch.rand(units, dtype=torch.float64, device=dev) for _ in range(3)] for _ in range(nsets)]
        for x, y, z in sets:
            x.addcmul_(y, z)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(steps):
            x, y, z = sets[i % nsets]
            x.addcmul_(y, z)
        e1.record(s)
    s.synchronize()
    ms = e0.elapsed_time(e1) / steps
    del sets
    torch.cuda.empty_cache()
    return {"what": "torch addcmul_ float64 (3 x 8 B read + 8 B written per element), %d elements, %d sets, "
                    "cold" % (units, nsets),
            "ms": ms, "frac": units * 32 / (ms * 1e-3) / HBM_PEAK}


def cold_layout_yardstick(torch, dev, units, nsets, steps, balance_bytes):
    """A stock elementwise kernel on the epoch layout's own traffic shape, cold: torch's in-place
    ``x.add_(y)`` with x the balance column's width (int32 for the u32 offsets, int64) and y
    int32 (the {start, end} column's 4 B), i.e. read 2 columns, write one, per element."""
    dt = torch.int32 if balance_bytes == 4 else torch.int64
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        sets = [(torch.zeros(units, dtype=dt, device=dev), torch.ones(units, dtype=torch.int32, device=dev))
                for _ in range(nsets)]
        for x, y in sets:
            x.add_(y)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for i in range(steps):
            x, y = sets[i % nsets]
            x.add_(y)
        e1.record(s)
    s.synchronize()
    ms = e0.elapsed_time(e1) / steps
    del sets
    torch.cuda.empty_cache()
    per = 2 * balance_bytes + 4
    return {"what": "torch in-place add_ (%s += int32: %d B read + %d B written per element), %d elements, %d "
                    "sets, cold" % (str(dt).replace("torch.", ""), balance_bytes + 4, balance_bytes, units, nsets),
            "ms": ms, "frac": units * per / (ms * 1e-3) / HBM_PEAK}


def epoch_parity(inst, dev):
    """The checker for the timed workload: one fresh step of the same B instances through
    pz_epoch_state (the timed loop has already stepped the balances many times), instance 0
    compared bit-exactly with the numpy oracle (oracle/epoch_np.py): balances, tallies,
    winners, next-cycle total."""
    from prysm_amd import _lib
    from prysm_amd.native import NativeEpoch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from epoch_ref_helpers import oracle_epoch

    de = NativeEpoch(inst, device=dev.index)
    de.step()
    bal, scal, vote, total, win = de.results()
    idx = de.validators()  # the validator index of each balance column (committee order)
    de.free()
    nb, applied, nxt, v, t, w = oracle_epoch(inst, 0)
    ok = (np.array_equal(bal[0], nb[idx]) and bool(scal[0, _lib.SCAL_APPLIED]) == applied
          and int(scal[0, _lib.SCAL_NEXT_BAL]) == nxt and np.array_equal(vote[0], v)
          and np.array_equal(total[0], t) and np.array_equal(win[0], w))
    return "instance 0 of the timed %d x %d workload, one step, bit-exact vs oracle/epoch_np: %s" % (
        inst["ninst"], inst["nval"], ok)


def epoch_single_instance(args, torch, dev, nval, shuffled):
    """the latency of ONE epoch instance (B = 1) at configs[2]'s size
    (2.9 MB of algorithmic traffic): the single-launch step (pz_epoch_one_kernel), device time
    by HIP events, median over the steps; beside it the window pass (the multi-instance one-pass
    kernel, pz_epoch_options.window_only) on the same instance."""
    from prysm_amd import _lib, synth
    from prysm_amd.native import NativeEpoch

    def measure(window_only=False):
        de = NativeEpoch(synth.epoch_batch(nval, 1, seed=3, shuffled=shuffled), device=dev.index,
                         window_only=window_only)
        stream = torch.cuda.ExternalStream(de.shard(0)[3], device=dev)
        for _ in range(args.warmup + 20):
            de.step()
        stream.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(max(args.steps, 20))]
        t0 = time.perf_counter()
        for e0, e1 in evs:
            e0.record(stream)
            de.step()
            e1.record(stream)
        stream.synchronize()
        wall = time.perf_counter() - t0
        # back to back: one event pair around K steps (each step's launch overhead hidden
        # behind the previous step, as a node stepping epochs in a row would see it)
        b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        b0.record(stream)
        for _ in range(len(evs)):
            de.step()
        b1.record(stream)
        stream.synchronize()
        de.free()
        return (float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])), wall / len(evs) * 1e3,
                b0.elapsed_time(b1) / len(evs))

    ms, wall_ms, b2b = measure()
    floor = event_pair_floor(args, torch, dev)
    ms3, wall3, b2b3 = measure(window_only=True)
    return {"validators": nval, "instances_per_step": 1, "path": "pz_epoch_one_kernel (single launch)",
            "device_ms_median": ms, "wall_ms_per_step": wall_ms, "back_to_back_ms_per_step": b2b,
            "device_ms_net_of_event_floor": ms - floor["empty_ms"], "event_floor": floor,
            "validator_epochs_per_s": nval / (ms * 1e-3),
            "window_pass": {"device_ms_median": ms3, "wall_ms_per_step": wall3, "back_to_back_ms_per_step": b2b3}}


def event_pair_floor(args, torch, dev):
    """What the event-pair clock of epoch_single_instance reads with nothing between the two
    events, and around one one-element torch kernel, on a fresh stream (tools/launch_floor.py:
    ~4.8 and ~8.6 us on an MI355X): the floor under any single-launch latency measured so."""
    s = torch.cuda.Stream(device=dev)
    x = torch.zeros(1, device=dev)

    def med(fn, k=max(args.steps, 50)):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        with torch.cuda.stream(s):
            for _ in range(10):
                fn()
            for e0, e1 in evs:
                e0.record(s)
                fn()
                e1.record(s)
        s.synchronize()
        return float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))

    return {"empty_ms": med(lambda: None), "tiny_kernel_ms": med(lambda: x.add_(1)),
            "what": "median HIP-event pair around nothing / one 1-element torch kernel"}


def epoch_cpu_baseline(inst):
    """The oracle's C restatement of the same epoch (AoS, 1 thread), on one instance."""
    try:
        from oracle import cport
        reps, dt = cport.epoch_instance_timed(inst, 0, min_seconds=CPU_SAMPLE_S)
        host = cport.host_info()
        T = host["threads_all_cores"]
        ra, da = cport.epoch_all_cores_timed(inst, T, CPU_SAMPLE_S / 2)
        return {"value": reps * inst["nval"] / dt, "unit": "validator-epochs/s", "cores": 1, "kind": "port",
                "sample": "%d x one %d-validator epoch instance (AoS records, 1 thread, oracle/c/epoch_ref.c), "
                          "%.2f s" % (reps, inst["nval"], dt),
                "all_cores": {"value": ra * inst["nval"] / da, "cores": T,
                              "sample": "%d transitions of %d independent %d-validator instances, one per thread, "
                                        "%.2f s" % (ra, T, inst["nval"], da)}}
    except Exception as e:  # pragma: no cover
        return {"value": None, "unit": "validator-epochs/s", "cores": 0, "kind": "port",
                "sample": "unavailable: %s" % e}


WIRE_KERNELS = ("pz_wire_val_size_kernel", "pz_wire_scan_kernel", "pz_wire_val_write_kernel")


def wire_leg(args, torch, dist, dev, rank, world):
    """the CrystallizedState's ValidatorRecords proto3-encoded on the
    device from the resident SoA columns (pz_dev_wire_validators).  One step encodes 16
    states of 1,048,576 validators (configs[3]'s size; the columns of the 16 states back to
    back, which is the same bytes as 16 separate calls).  Algorithmic bytes per record: the
    three u64 columns read once (24 B) + the encoded record written once."""
    from prysm_amd import _lib, pb, wire

    nval, nst = 1 << 20, 16
    n = nval * nst
    rng = np.random.default_rng(7 + rank)
    bal = rng.integers(16, 49, size=n, dtype=np.uint64)
    start = np.zeros(n, dtype=np.uint64)
    end = np.full(n, 9999999999999999999, dtype=np.uint64)
    cols_t = [torch.from_numpy(a.view(np.int64)).to(dev) for a in (bal, start, end)]
    bound = int(_lib.lib.dll.pz_wire_validators_bound(n, 0))
    d_out = torch.empty(bound, dtype=torch.uint8, device=dev)
    d_scr = torch.empty(int(_lib.lib.dll.pz_wire_scratch_bytes(n)) // 8, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    cols = _lib.ValidatorCols(None, None, None, None, None, None, *[t.data_ptr() for t in cols_t])
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)

    def step():
        _lib.lib.call("pz_dev_wire_validators", ctypes.byref(cols), n, 11, d_out.data_ptr(), None,
                      d_scr.data_ptr(), d_tot.data_ptr(), sh)

    for _ in range(args.warmup + 20):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # one event pair around the K back-to-back steps: the average launch duration without
    # per-step event packets between the launches (what rocprofv3's kernel trace averages)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        wall = max_over_ranks(wall, torch, dist, dev)
    total = int(d_tot.item())
    alg = n * 24 + total
    out = {
        "metric": "ValidatorRecords proto3-encoded/s",
        "value": n * world * args.steps / wall,
        "unit": "records/s",
        "ms_per_step": wall / args.steps * 1e3,
        "scaling": "weak",
        "config": {"workload": "CrystallizedState.validators (field 11) encoding of %d states x %d validators "
                               "(configs[3] size) from device-resident balance/start/end columns" % (nst, nval),
                   "records_per_gpu": n, "encoded_bytes_per_gpu": total,
                   "parallelism": "independent states per rank" if world > 1 else "single GPU"},
        "roofline": {"bound": "hbm", "achieved": alg / (step_ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": alg / (step_ms * 1e-3) / HBM_PEAK,
                     "traffic": pmc_traffic(["pz_wire_val_kernel"]), "traffic_source": PMC_SUMMARY,
                     "kernel": "pz_wire_val_kernel (device time of the step, tile-status memset included)", "step_device_ms": step_ms,
                     "algorithmic_bytes_per_launch": alg},
    }
    # the checker (every rank): the first state's bytes against the C port
    from oracle import cport
    one = pb.Validators(nval, balance=bal[:nval], start_dynasty=start[:nval], end_dynasty=end[:nval])
    want = cport.wire_validators(one)
    got = d_out[:len(want)].cpu().numpy().tobytes()
    ok = got == want if world == 1 else all_ranks(got == want, torch, dist, dev)
    out["parity"] = "byte-exact vs the C port on the first state's %d bytes%s: %s" % (
        len(want), "" if world == 1 else " of every rank", ok)
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            reps, dt = cport.wire_validators_timed(one, min_seconds=CPU_SAMPLE_S / 2)
            out["cpu_baseline"] = {"value": reps * nval / dt, "unit": "records/s", "cores": 1, "kind": "port",
                                   "sample": "%d encodings of one %d-validator state (AoS records, size + marshal "
                                             "pass, 1 thread, oracle/c/wire_ref.c), %.2f s" % (reps, nval, dt)}
    return out


def wire_att_leg(args, torch, dist, dev, rank, world, d_digests):
    """SURVEY.md §8f row 1 for attestations: the hash bench's 1M AttestationRecords (configs[1])
    proto3-encoded on the device from their SoA columns (pz_dev_wire_attestations), then
    hashed (pz_dev_blake2b512_batch, CSR).  The encode is timed alone and as encode + hash;
    the digests are checked against the main leg's, whose records are the same bytes."""
    from prysm_amd import _lib, synth, wire

    n = args.records
    cols = synth.attestation_columns_512(n, seed=2 + rank)
    t = {k: torch.from_numpy(cols[k].view(np.int64) if cols[k].dtype == np.uint64 else cols[k]).to(dev)
         for k in wire.ATT_COLS}
    c = _lib.AttestationCols(*[t[k].data_ptr() for k in wire.ATT_COLS])
    ne, ns = int(cols["oblique_first"][-1]), int(cols["aggregate_sig_first"][-1])
    nbytes = sum(int(cols[k][-1]) for k in ("justified_block_hash_offs", "shard_block_hash_offs",
                                            "attester_bitfield_offs", "oblique_offs"))
    d_out = torch.empty(int(_lib.lib.dll.pz_wire_attestations_bound(n, nbytes, ne, ns)) + 16, dtype=torch.uint8,
                        device=dev)
    d_offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_scr = torch.empty(int(_lib.lib.dll.pz_wire_attestations_scratch_bytes(n)), dtype=torch.uint8, device=dev)
    d_dig = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)

    def encode():
        _lib.lib.call("pz_dev_wire_attestations", ctypes.byref(c), n, 0, d_out.data_ptr(), d_offs.data_ptr(),
                      d_scr.data_ptr(), sh)

    def encode_hash():
        encode()
        _lib.lib.call("pz_dev_blake2b512_batch", d_out.data_ptr(), d_offs.data_ptr(), n, d_dig.data_ptr(), 32, sh)

    def timed(fn):
        for _ in range(args.warmup + 5):
            fn()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        if world > 1:
            wall = max_over_ranks(wall, torch, dist, dev)
        return wall, e0.elapsed_time(e1) / args.steps

    wall_e, ms_e = timed(encode)
    wall_eh, ms_eh = timed(encode_hash)
    in_bytes = sum(int(cols[k].nbytes) for k in wire.ATT_COLS)
    alg = in_bytes + n * 512 + (n + 1) * 8
    out = {
        "metric": "AttestationRecords proto3-encoded (+ hashed) /s from device columns",
        "value": n * world * args.steps / wall_eh,
        "unit": "records/s",
        "ms_per_step": wall_eh / args.steps * 1e3,
        "scaling": "weak",
        "config": {"workload": "the %d x 512-B AttestationRecords of configs[1], encoded from SoA columns then "
                               "BLAKE2b-512[:32] (CSR)" % n, "parallelism": "record-shard x%d" % world},
        "encode_only": {"value": n * world * args.steps / wall_e, "ms_per_step": wall_e / args.steps * 1e3},
        "roofline": {"bound": "hbm", "achieved": alg / (ms_e * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                     "frac": alg / (ms_e * 1e-3) / HBM_PEAK,
                     "traffic": pmc_traffic(["pz_wire_att_size_kernel", "pz_wire_att_write_kernel"]),
                     "traffic_source": PMC_SUMMARY,
                     "kernel": ("pz_wire_att_size_kernel (sizes, tile scan, decoupled look-back) + "
                                "pz_wire_att_write_kernel (device time of the encode)"),
                     "step_device_ms": ms_e, "encode_hash_device_ms": ms_eh, "algorithmic_bytes_per_launch": alg},
    }
    if d_digests is not None:
        out["parity"] = "digests of the encoded records equal the hash leg's on all %d records: %s" % (
            n, bool(torch.equal(d_dig, d_digests)))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cport
        port = cport.WireAtt(cols, n)
        try:
            reps, t1 = 0, time.perf_counter()
            while reps == 0 or time.perf_counter() - t1 < CPU_SAMPLE_S / 4:
                port.run()
                reps += 1
            dt = time.perf_counter() - t1
        finally:
            port.close()
        out["cpu_baseline"] = {"value": reps * n / dt, "unit": "records/s (encode only)", "cores": 1, "kind": "port",
                               "sample": "%d marshals of the %d records (AoS, Size + MarshalTo per record, 1 thread, "
                                         "oracle/c/wire_ref.c), %.2f s" % (reps, n, dt)}
    return out


ATT_BYTES = 65  # per attestation: 5 u64 columns + its boffs entry + the bitfield's last byte (its own column) + 16 B out


def attcheck_columns(natt, seed):
    """Synthetic processAttestation inputs at configs[2]'s committee shape (65,536 validators:
    5 committees of 204-205 per slot, 256 ShardAndCommitteesForSlots arrays), blocks of slots
    64-127 after a recalc at 0; 5 % of the attestations fail one of the checks."""
    rng = np.random.default_rng(seed)
    narr, per = 256, 5
    arr_offs = np.arange(narr + 1, dtype=np.uint64) * per
    arr_shard = ((np.arange(narr * per) // per % 64) * per + np.arange(narr * per) % per).astype(np.uint64) % 1024
    arr_comm = ((np.arange(narr * per) // per % 64) * per + np.arange(narr * per) % per).astype(np.uint32)
    sizes = np.full(64 * per, 204, dtype=np.uint64)
    sizes[: 65536 - 204 * 64 * per] += 1
    coffs = np.zeros(64 * per + 1, dtype=np.uint64)
    coffs[1:] = np.cumsum(sizes)
    bslot = rng.integers(64, 128, size=natt, dtype=np.uint64)
    slot = bslot - rng.integers(0, 65, size=natt, dtype=np.uint64)
    j = rng.integers(0, per, size=natt)
    shard = arr_shard[slot.astype(np.int64) * per + j]
    k = sizes[arr_comm[slot.astype(np.int64) * per + j]]
    blen = (k + np.uint64(7)) // np.uint64(8)
    bad = rng.random(natt) < 0.05
    js = np.where(bad & (rng.random(natt) < 0.5), np.uint64(9), np.uint64(0)).astype(np.uint64)
    blen = np.where(bad & (js == 0), blen + np.uint64(1), blen)
    boffs = np.zeros(natt + 1, dtype=np.uint64)
    boffs[1:] = np.cumsum(blen)
    bits = rng.integers(0, 256, size=int(boffs[-1]) + 1, dtype=np.uint8)
    last = (boffs[1:] - np.uint64(1)).astype(np.int64)
    rem = (k % np.uint64(8)).astype(np.int64)
    bits[last] &= np.where(rem > 0, (0xFF << (8 - rem)) & 0xFF, 0xFF).astype(np.uint8)
    nob = np.zeros(natt, dtype=np.uint64)
    cols = dict(slot=slot, justified_slot=js, shard_id=shard, n_oblique=nob, bits=bits, boffs=boffs, block_slot=bslot)
    tab = dict(arr_offs=arr_offs, arr_shard=arr_shard, arr_comm=arr_comm, coffs=coffs)
    return cols, tab


def attcheck_batch(torch, dev, cols, tab, natt, last_byte=True):
    """The pz_att_check_batch over device copies of ``attcheck_columns`` (and the tensors it
    points into, which the caller keeps alive).  ``last_byte``: the caller-side column of each
    bitfield's last byte (bits[boffs[i+1]-1]), so the trailing-bits check reads 1 B per
    attestation instead of touching every bitfield line."""
    from prysm_amd import _lib

    cols = dict(cols)
    if last_byte:
        cols["last_byte"] = cols["bits"][(cols["boffs"][1:].astype(np.int64) - 1) % max(1, cols["bits"].size)]
    t = {k: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v.view(np.int32) if v.dtype == np.uint32
                             else v).to(dev) for k, v in list(cols.items()) + list(tab.items())}
    t["status"] = torch.empty(natt, dtype=torch.int32, device=dev)
    t["committee"] = torch.empty(natt, dtype=torch.int32, device=dev)
    t["pstart"] = torch.empty(natt, dtype=torch.int64, device=dev)
    b = _lib.AttCheckBatch(natt, t["slot"].data_ptr(), t["justified_slot"].data_ptr(), t["shard_id"].data_ptr(),
                           t["n_oblique"].data_ptr(), t["bits"].data_ptr(), t["boffs"].data_ptr(),
                           t["block_slot"].data_ptr(), 0, 0, 128, 256, t["arr_offs"].data_ptr(),
                           t["arr_shard"].data_ptr(), t["arr_comm"].data_ptr(), t["coffs"].data_ptr(),
                           t["status"].data_ptr(), t["committee"].data_ptr(), t["pstart"].data_ptr(),
                           t["last_byte"].data_ptr() if last_byte else None)
    return b, t


def attcheck_leg(args, torch, dist, dev, rank, world):
    """processAttestation's checks for a batch of 4M attestations on the
    GPU (pz_dev_check_attestations, one lane each); attestations shard over the ranks."""
    from prysm_amd import _lib

    natt = 1 << 22
    cols, tab = attcheck_columns(natt, seed=11 + rank)
    b, t = attcheck_batch(torch, dev, cols, tab, natt)
    status = t["status"]
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)

    def step():
        _lib.lib.call("pz_dev_check_attestations", ctypes.byref(b), sh)

    for _ in range(args.warmup + 20):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # one event pair around the K back-to-back steps: the average launch duration without
    # per-step event packets between the launches (what rocprofv3's kernel trace averages)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    step_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        wall = max_over_ranks(wall, torch, dist, dev)
    alg = natt * ATT_BYTES
    out = {
        "metric": "attestations checked/s (processAttestation, core.go:240-297)",
        "value": natt * world * args.steps / wall,
        "unit": "attestations/s",
        "ms_per_step": wall / args.steps * 1e3,
        "scaling": "weak",
        "config": {"workload": "%d attestations per GPU at configs[2]'s committee shape (65,536 validators), "
                               "5%% failing a check" % natt, "parallelism": "attestation-shard x%d" % world},
        "roofline": {"bound": "hbm", "achieved": alg / (step_ms * 1e-3) / 1e9, "peak": HBM_PEAK / 1e9,
                     "unit": "GB/s", "frac": alg / (step_ms * 1e-3) / HBM_PEAK,
                     "traffic": pmc_traffic(["pz_att_check_p_kernel"]), "traffic_source": PMC_SUMMARY,
                     "kernel": "pz_att_check_p_kernel", "step_device_ms": step_ms,
                     "algorithmic_bytes_per_launch": alg},
    }
    from oracle import cport
    ns = 1 << 20
    sub = {k: (v[:ns + 1] if k == "boffs" else v[:ns]) for k, v in cols.items() if k != "bits"}
    port = cport.AttCheck(sub["slot"], sub["justified_slot"], sub["shard_id"], sub["n_oblique"], cols["bits"],
                          sub["boffs"], sub["block_slot"])
    try:
        want = port.run(0, 0, 128, tab["arr_offs"], tab["arr_shard"], tab["arr_comm"], tab["coffs"])
        got = status[:ns].cpu().numpy()
        ok = bool(np.array_equal(got, want))
        ok = ok if world == 1 else all_ranks(ok, torch, dist, dev)
        out["parity"] = "status of the first %d attestations%s equal to the C port: %s" % (
            ns, "" if world == 1 else " of every rank", ok)
        if rank == 0 and world == 1:
            if not args.no_cpu_baseline:
                reps, t1 = 0, time.perf_counter()
                while reps == 0 or time.perf_counter() - t1 < CPU_SAMPLE_S / 4:
                    port.run(0, 0, 128, tab["arr_offs"], tab["arr_shard"], tab["arr_comm"], tab["coffs"])
                    reps += 1
                dt = time.perf_counter() - t1
                out["cpu_baseline"] = {"value": reps * ns / dt, "unit": "attestations/s", "cores": 1, "kind": "port",
                                       "sample": "%d passes over %d attestations (AoS records, 1 thread, "
                                                 "oracle/c/attcheck_ref.c), %.2f s" % (reps, ns, dt)}
    finally:
        port.close()
    return out


def replay_sharded_leg(args, torch, dist, dev, rank, world, comm):
    """BASELINE configs[4] as ONE chain batch-sharded over the N GPUs:
    every rank replays the same 10,000 blocks (the walk is sequential host work, done by each
    process), and the device work is split by validator range -- each GPU holds 1/N of the
    balances, of every vote-cache voter bitmap and of every epoch; a transition all-reduces the
    64 justification totals, the epoch's partial sums and the previous epoch's next-cycle
    partial in ONE collective over RCCL (pz_chain_new_comm; the call's final flush carries the
    last one)."""
    from prysm_amd import synth
    from prysm_amd.blockchain import BeaconChain, serialize_blocks

    nval, nb = 65536, args.replay_blocks
    blocks = synth.chain_blocks(nval, nb, seed=6)
    data, offs = serialize_blocks(blocks)
    w_data, w_offs = serialize_blocks(blocks[:min(nb, 130)])
    BeaconChain(nval, comm=comm).process_serialized(w_data, w_offs)  # warm-up
    torch.cuda.synchronize(dev)
    dist.barrier()
    ch = BeaconChain(nval, comm=comm)
    torch.cuda.synchronize(dev)
    dist.barrier()
    comm.set_timing(True)  # event pairs on the communicator's stream (the walk is host-bound)
    comm.collective_time()
    t0 = time.perf_counter()
    br, ar = ch.process_serialized(data, offs)
    wall = time.perf_counter() - t0
    wall = max_over_ranks(wall, torch, dist, dev)
    cms, cn = comm.collective_time()
    comm.set_timing(False)
    roots = ch.roots()
    # the checker, on every rank: its copy of the one chain against the C restatement of
    # blockProcessing (every rank walks the same blocks, so every rank's results must be exact)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from replay_port_helpers import mismatches, port_replay
    t1 = time.perf_counter()
    p_out, p_roots = port_replay(data, offs, nval, len(ar))
    bad = mismatches(br, ar, roots, p_out, p_roots)
    ok = all_ranks(not bad, torch, dist, dev)
    out = {"metric": "sync-replay blocks/s (one chain over N GPUs)", "value": nb / wall, "unit": "blocks/s",
           "ms_per_block": wall / nb * 1e3,
           "config": {"workload": "the configs[4] chain (10,000 blocks, 65,536 validators) as ONE chain",
                      "parallelism": "validator-range shard x%d of the vote cache and the epoch; ONE all-reduce "
                                     "per transition: the 64 justification totals, the epoch's partial sums and the "
                                     "previous epoch's next-cycle partial (%s)"
                                     % (world, "RCCL" if dist.get_backend() == "nccl" else "SHM rehearsal")},
           "processed": int((br["status"] == 0).sum()), "transitions": int(br["transition"].sum()),
           "collectives": {"count": cn, "device_ms": cms, "per_transition": cn / max(1, int(br["transition"].sum())),
                           "what": "rank 0's collectives over the timed replay, HIP events on the communicator stream"},
           "parity": ("all %d blocks, %d attestations, the 4 state roots and %d vote-cache totals of every rank's copy "
                      "vs oracle/c/replay_ref.c (%.1f s): %s" % (nb, len(ar), len(p_roots["vote_totals"]),
                                                                 time.perf_counter() - t1,
                                                                 "bit-exact on every rank" if ok else
                                                                 "MISMATCH " + (", ".join(bad) or "on another rank"))),
           "cand_crystallized_root": roots.get("cand_crystallized", b"").hex()}
    return out


PROF_PHASES = ("parse", "digest_batch", "checks", "vote_queue", "vote_flush", "state_recalc", "msg_digests", "walk",
               "process", "count_atts", "flush_arena_wait", "msg_send", "msg_hash_log", "msg_wait",
               "totals_wait", "poll_fallbacks", "vote_id_rows")  # the last two are counts (tally-total polls that
#               fell back to the event wait; queued attestations whose parent ids needed an explicit row)


def chain_phases_ms(ch):
    """The chain engine's always-on phase clocks (pz_chain_phase_times; the per-attestation
    ones, checks and vote_queue, run only under PZ_CHAIN_PROFILE and read 0 here)."""
    import ctypes
    from prysm_amd import _lib
    n = len(PROF_PHASES)
    pv = (ctypes.c_double * n)()
    fn = _lib.lib.dll.pz_chain_phase_times
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    k = fn(ch._h, pv, n)
    out = {PROF_PHASES[i]: round(pv[i] * 1e3, 3) for i in range(min(k, n - 2)) if pv[i] > 0}
    for i in range(n - 2, min(k, n)):
        out[PROF_PHASES[i]] = int(pv[i])  # the counts, always reported, 0 included
    return out


def _compressions(nbytes):
    return max(1, -(-int(nbytes) // 128))


def replay_roofline(blocks, offs, ar, wall, ch):
    """configs[4]'s roofline.  The device work per block, priced at the chip's peaks: the
    BLAKE2b compressions of its digests (block encoding, and per attestation its encoding, its
    Key() preimage and the 64-byte signed-message digest) at OPS_PER_COMPRESSION on the VALU
    model of the hash leg, and the vote-cache tally's bytes (per queued attestation: the
    bitfield, 63 parent ids, the k members' 8-byte balances, and per signed parent and member a
    4-byte voter-bitmap word read and written) at HBM peak.  ``peak`` is the blocks/s that device work alone would
    allow; the walk itself is sequential host work, so ``bound`` is "host" and
    the phase clocks say where the wall time goes."""
    from prysm_amd import wire
    nb = len(blocks)
    comp = sum(_compressions(int(offs[i + 1]) - int(offs[i])) for i in range(nb))
    tally_b = 0
    for b in blocks:
        for a in b.attestations:
            comp += _compressions(len(wire.attestation_record(a)))
            comp += _compressions(10 + len(a.shard_block_hash) + 32 * len(a.oblique_parent_hashes))
            k = 8 * len(a.attester_bitfield)
            tally_b += len(a.attester_bitfield) + 63 * 4 + 8 * k + 63 * k * 8
    comp += sum(_compressions(int(m)) for m in ar["msg_len"] if m)
    dev_s = comp * OPS_PER_COMPRESSION / VALU_PEAK + tally_b / HBM_PEAK
    achieved = nb / wall
    peak = nb / dev_s
    return {"bound": "host", "achieved": achieved, "peak": peak, "unit": "blocks/s", "frac": achieved / peak,
            "traffic": None,
            "model": {"compressions_per_block": comp / nb, "valu_slots_per_compression": OPS_PER_COMPRESSION,
                      "tally_bytes_per_block": tally_b / nb, "device_floor_ms": dev_s * 1e3,
                      "wall_ms": wall * 1e3},
            "host_phases_ms": chain_phases_ms(ch),
            "note": "device floor = compressions x VALU slots / 78.6 T + tally bytes / 8 TB/s; the rest of the "
                    "wall is the sequential host walk (parse, checks, vote queue, stateRecalc's round trip)"}


def replay_leg(args, torch, dist, dev, rank, world):
    """BASELINE configs[4]: sync replay of a synthetic 10,000-block chain through the block
    pipeline (blockchain/service.go:229-363): per block the block digest, 5 attestations'
    Hash / Key / 64-byte message digests, the vote-cache tally of 5 x 204-205 members x 63
    signed parent hashes, and a stateRecalc every 64 blocks.  The control flow is sequential
    (host walk); the hashing, tallies and epochs are batched on the GPU.  At N > 1 every rank
    replays its own chain (seed + rank): block batches shard with no collective.  Also
    BASELINE configs[0]: the 1,024-validator chain of tests/golden/replay_n1024.json, its
    roots checked against the fixture."""
    from prysm_amd import synth
    from prysm_amd.blockchain import BeaconChain

    from prysm_amd.blockchain import serialize_blocks

    nval, nb = 65536, args.replay_blocks
    blocks = synth.chain_blocks(nval, nb, seed=6 + rank)
    data, offs = serialize_blocks(blocks)  # sync delivers serialized blocks (sync/service.go:147-164)
    # warm-up: the same chain on a throwaway BeaconChain (kernels loaded; the library's pinned
    # staging pool, which a long-running node keeps, holds buffers of this size)
    w = BeaconChain(nval, dev)
    w.process_serialized(data, offs)
    del w  # (pz_chain_free: its pinned buffers go back to the pool)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # five replays, each of the whole chain on a fresh chain (genesis -- shuffle + uploads -- is
    # not part of a replay): the median, so one descheduled host thread or a slow first replay
    # (the box's host warming up: 12.7 / 11.5 / 10.9 ms in profiles/r04/bench_r4ap.json) does not
    # make the line
    walls, reps_agree = [], True
    NREP = 5
    for k in range(NREP):
        ch = BeaconChain(nval, dev)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        br, ar = ch.process_serialized(data, offs)
        torch.cuda.synchronize(dev)
        w_k = time.perf_counter() - t0
        walls.append(max_over_ranks(w_k, torch, dist, dev) if world > 1 else w_k)
        # every timed replay's records equal the last one's, which the checker below compares
        # with the C restatement (the first four were never checked)
        if k == 0:
            br0, ar0 = br, ar
        else:
            reps_agree = reps_agree and np.array_equal(br, br0) and np.array_equal(ar, ar0)
        if k < NREP - 1:
            del ch
    wall = float(np.median(walls))
    # State roots (types/state.go:138-149, 237-248) of the replayed chain: the 1.7 MB
    # CrystallizedState is one serial BLAKE2b chain of 13,416 compressions.  Timed on both
    # routes: host threads (the default for messages >= 64 KiB) and a single GPU lane.
    from prysm_amd import _lib
    root_ms, root_vals = {}, {}
    for label, thr in (("host_serial", _lib.serial_threshold_default()), ("gpu_lane", _lib.SERIAL_ON_GPU)):
        with _lib.serial_threshold(thr):
            t1 = time.perf_counter()
            r = ch.roots()
            root_ms[label] = (time.perf_counter() - t1) * 1e3
            root_vals[label] = r
    state_roots = {"ms_per_roots_call": root_ms, "routes_agree": root_vals["host_serial"] == root_vals["gpu_lane"],
                   "what": "4 state roots (chain + candidate Active/Crystallized), serialization included"}
    recs = [{"status": "processed" if s == 0 else "other", "transition": bool(t)}
            for s, t in zip(br["status"], br["transition"])]
    out = {"metric": "sync-replay blocks/s", "value": nb * world / wall, "unit": "blocks/s",
           "ms_per_block": wall / nb * 1e3, "replay_walls_ms": [round(x * 1e3, 3) for x in walls],
           "timing": "median of 5 replays of the whole chain, each on a fresh chain",
           "config": {"workload": "sync replay: block + 5 x (attestation Hash, Key, message digest) + vote "
                                  "tally per block, stateRecalc every 64 blocks (BASELINE configs[4])",
                      "validators": nval, "blocks_per_gpu": nb, "attestations_per_block": 5,
                      "parallelism": "%d independent chain(s), one per GPU (replicas; not one batch-sharded "
                                     "chain: DESIGN.md §6)" % world},
           "input": "serialized canonical BeaconBlock encodings, %.1f MB" % (int(offs[-1]) / 1e6),
           "processed": sum(r["status"] == "processed" for r in recs),
           "transitions": sum(r["transition"] for r in recs),
           "state_roots": state_roots,
           "cand_crystallized_root": root_vals["host_serial"].get("cand_crystallized", b"").hex(),
           "roofline": replay_roofline(blocks, offs, ar, wall, ch)}
    # the checker (every rank, its own replica): the whole timed chain through the C
    # restatement of the block pipeline (checker mode), compared with the GPU engine's records
    # and roots
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from replay_port_helpers import mismatches, port_replay
    t1 = time.perf_counter()
    p_out, p_roots = port_replay(data, offs, nval, len(ar))
    bad = mismatches(br, ar, root_vals["host_serial"], p_out, p_roots)
    if not reps_agree:
        bad = list(bad) + ["the %d timed replays' records differ" % NREP]
    ok = not bad if world == 1 else all_ranks(not bad, torch, dist, dev)
    out["parity"] = ("all %d blocks and %d attestations (digests, statuses, transitions; identical in all 5 timed "
                     "replays), the 4 state roots and %d vote-cache totals vs the C restatement of blockProcessing (oracle/c/replay_ref.c), "
                     "%.1f s%s: %s" % (nb, len(ar), len(p_roots["vote_totals"]), time.perf_counter() - t1,
                                       "" if world == 1 else ", each rank's own chain",
                                       "bit-exact" + ("" if world == 1 else " on every rank") if ok else
                                       "MISMATCH " + (", ".join(bad) or "on another rank")))
    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            from oracle import cport
            sd, so = serialize_blocks(blocks[:args.cpu_replay_blocks])
            nsa = sum(len(b.attestations) for b in blocks[:args.cpu_replay_blocks])
            r = cport.Replay(nval)  # Go's algorithms: linear scan of VoterIndices (core.go:333-337)
            t0 = time.perf_counter()
            r.process(sd, so, nsa)
            dt = time.perf_counter() - t0
            r.close()
            out["cpu_baseline"] = {"value": (len(so) - 1) / dt, "unit": "blocks/s", "cores": 1,
                                   "kind": "port",
                                   "sample": "first %d blocks of the same serialized chain through the C restatement of "
                                             "blockProcessing (oracle/c/replay_ref.c: decode, Marshal + BLAKE2b, "
                                             "processAttestation, the vote cache with Go's O(k^2) voter scan, "
                                             "stateRecalc over heap records), 1 thread, %.2f s" % (len(so) - 1, dt)}
    # configs[0]: the golden 1,024-validator chain (parity of the final roots on this box)
    with open(os.path.join(ROOT, "tests", "golden", "replay_n1024.json")) as f:
        g = json.load(f)
    sim_blocks = synth.chain_blocks(g["nval"], g["nblocks"], seed=g["seed"])
    t0 = time.perf_counter()
    sc = BeaconChain(g["nval"], dev)
    sc.process_blocks(sim_blocks)
    roots = sc.roots()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    out["simulator"] = {"config": "BASELINE configs[0]: %d validators, %d blocks (2 cycle transitions)"
                                  % (g["nval"], g["nblocks"]),
                        "blocks_per_s": g["nblocks"] / dt,
                        "roots_match_golden": all(roots[k].hex() == v for k, v in g["roots"].items()),
                        "cand_crystallized_root": roots["cand_crystallized"].hex()}
    return out


def shuffle_leg(args):
    """utils.ShuffleIndices at configs[3]'s 1,048,576 validators
    (host by design: a sequential swap chain, shuffle.go:14-33), and the whole
    ShuffleValidatorsToCommittees (sharding.go:11-53: the device active filter, the swap chain,
    splitBySlotShard into the committee CSR), which updateHead runs on every head
    (blockchain/service.go:185-190).  Parity: the permutation against the C restatement."""
    from oracle import cport
    from prysm_amd import casper

    n = 1 << 20
    seed = b"A" + bytes(31)
    base = np.arange(n, dtype=np.uint32)
    ts = []
    for _ in range(max(3, min(args.steps, 20))):
        lst = base.copy()
        t0 = time.perf_counter()
        got = casper.shuffle_indices(seed, lst)  # in place, like the Go function
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts)) * 1e3
    start = np.zeros(n, dtype=np.uint64)
    end = np.full(n, 9999999999999999999, dtype=np.uint64)
    comm = casper.shuffle_validators_to_committees(seed, start, end, 1, 0)
    # the C-ABI call alone, into preallocated CSR buffers
    from prysm_amd import _lib
    cap = 64 * (n // (64 * 128 * 2) + 1)
    seed_a = np.frombuffer(seed, dtype=np.uint8).copy()
    members, coffs = np.empty(n, np.uint32), np.empty(cap + 1, np.uint64)
    shard, slot_offs, nc = np.empty(cap, np.uint64), np.empty(65, np.uint64), ctypes.c_uint64(0)
    tc = []
    for _ in range(5):
        t0 = time.perf_counter()
        _lib.lib.call("pz_shuffle_validators_to_committees", _lib.ptr(seed_a), _lib.ptr(start), _lib.ptr(end), n,
                      1, 0, _lib.ptr(members), _lib.ptr(coffs), _lib.ptr(shard), _lib.ptr(slot_offs), cap,
                      ctypes.byref(nc))
        tc.append(time.perf_counter() - t0)
    out = {"metric": "ShuffleIndices on 1,048,576 validators", "ms_per_call": ms,
           "value": n / (ms * 1e-3), "unit": "validators/s",
           "committees_ms_per_call": float(np.median(tc)) * 1e3,
           "committees": "%d slots x %d committees" % (len(comm), len(comm[0])),
           "path": "host swap chain without division (sw < 256 <= n - i: the swap targets are the fixed "
                   "offsets i + sw[k]); seed stream BLAKE2b on the calling thread (small batch)",
           "parity": "permutation equal to the C restatement (oracle/c/shuffle_ref.c): %s"
                     % bool(np.array_equal(got, cport.shuffle_indices(seed, base)))}
    if not args.no_cpu_baseline:
        reps, dt = cport.shuffle_timed(seed, n, min_seconds=CPU_SAMPLE_S / 4)
        out["cpu_baseline"] = {"value": reps * n / dt, "unit": "validators/s", "cores": 1, "kind": "port",
                               "ms_per_call": dt / reps * 1e3,
                               "sample": "%d ShuffleIndices calls on 1,048,576 indices (shuffle.go's modulo per swap, "
                                         "1 thread, oracle/c/shuffle_ref.c), %.2f s" % (reps, dt)}
    return out


PMC_DIRS = (os.path.join("profiles", "r06"),)  # (this round's tree only: kernel names change between rounds)
PMC_SUMMARY = os.path.join(PMC_DIRS[0], "pmc_main.json")


def pmc_summary_path(workload):
    """The newest round's committed summary of ``workload`` (tools/gpu_pmc.sh)."""
    for d in PMC_DIRS:
        path = os.path.join(d, "pmc_%s.json" % workload)
        if os.path.exists(os.path.join(ROOT, path)):
            return path
    return os.path.join(PMC_DIRS[0], "pmc_%s.json" % workload)


def pmc_traffic(kernels, workload="main"):
    """HBM bytes per launch of ``kernels`` (summed; a name ending in '*' takes every kernel of
    the workload with that prefix) from the committed rocprofv3 --pmc summary of tools/
    pmc_workload.py's ``workload`` (tools/gpu_pmc.sh + tools/pmc_summary.py: FETCH_SIZE doubled
    per the gfx950 correction, WRITE_SIZE as is).  PMC counters cannot be read inside this
    process, so the figure comes from a separate profiled run of the same workload; None if
    the summary is absent or lacks a kernel."""
    path = os.path.join(ROOT, pmc_summary_path(workload))
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    names = []
    for k in kernels:
        names += sorted(n for n in d if n.startswith(k[:-1])) if k.endswith("*") else [k]
    try:
        return float(sum(d[k]["hbm_bytes_per_launch"] for k in names)) if names else None
    except KeyError:
        return None


def host_api_rate(records_np, reps=3):
    """The PCIe-inclusive rate (never `value`): the host-pointer C-ABI a cgo caller would use,
    pz_blake2b512_batch, over the same records from host memory (H2D of the batch, kernel,
    D2H of the digests), wall clock, median of `reps` calls."""
    from prysm_amd import _lib

    n = records_np.shape[0]
    flat = np.ascontiguousarray(records_np).reshape(-1)
    offs = np.arange(n + 1, dtype=np.uint64) * records_np.shape[1]
    out = np.empty(n * 32, dtype=np.uint8)
    ts = []
    for _ in range(reps + 1):
        t0 = time.perf_counter()
        _lib.lib.call("pz_blake2b512_batch", _lib.ptr(flat), _lib.ptr(offs), n, _lib.ptr(out), 32)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts[1:]))
    return {"value": n / dt, "unit": "hashes/s", "ms_per_call": dt * 1e3,
            "input_GBps": flat.nbytes / dt / 1e9,
            "what": "pz_blake2b512_batch (host pointers): H2D of the %d x %d-B batch + kernel + D2H, "
                    "median of %d calls" % (n, records_np.shape[1], reps)}


def avx2_host_rate(records_np, want, seconds):
    """The library's AVX2 host hasher (prysm_amd/csrc/serial_hash.cpp: the row-vector BLAKE2b
    compression, the stand-in for Go's x/crypto/blake2b assembly, blake2bAVX2_amd64.s) over the
    same records on 1 thread (pz_blake2b512_batch with the small-batch threshold above the batch,
    so the whole batch is hashed on the calling thread).  Digests checked against the portable
    C port's ``want``."""
    from prysm_amd import _lib
    n = records_np.shape[0]
    flat = np.ascontiguousarray(records_np).reshape(-1)
    offs = np.arange(n + 1, dtype=np.uint64) * records_np.shape[1]
    out = np.empty(n * 32, dtype=np.uint8)
    dll = _lib.lib.dll
    dll.pz_set_small_batch_threshold.restype = ctypes.c_uint64
    dll.pz_set_small_batch_threshold.argtypes = [ctypes.c_uint64]
    dll.pz_set_serial_threshold.restype = ctypes.c_uint64
    dll.pz_set_serial_threshold.argtypes = [ctypes.c_uint64]
    dll.pz_set_host_threads.restype = ctypes.c_uint32
    dll.pz_set_host_threads.argtypes = [ctypes.c_uint32]

    def call():
        _lib.lib.call("pz_blake2b512_batch", _lib.ptr(flat), _lib.ptr(offs), n, _lib.ptr(out), 32)

    def timed():
        t0 = time.perf_counter()
        call()
        ok = bool(np.array_equal(out.reshape(n, 32), want.reshape(n, 32)))
        passes = 1
        while time.perf_counter() - t0 < seconds:
            call()
            passes += 1
        return passes, time.perf_counter() - t0, ok

    old = dll.pz_set_small_batch_threshold(1 << 62)
    try:
        p1, d1, ok1 = timed()
    finally:
        dll.pz_set_small_batch_threshold(old)
    return {"value": p1 * n / d1, "cores": 1, "digests_match_port": ok1,
            "sample": "%d pass(es) over the %d x 512-B records, 1 thread, the library's AVX2 BLAKE2b "
                      "(serial_hash.cpp, row-vector compression; the stand-in for Go's x/crypto/blake2b AVX2 "
                      "assembly), %.2f s" % (p1, n, d1)}


def cpu_baseline(records_np):
    """The reference's hash on this host's cores over the same records: the AVX2 hasher on 1
    core (the honest stand-in for Go's x/crypto/blake2b, which runs AVX2 assembly),
    beside the oracle's portable C restatement (oracle/c) on 1 core and on all cores."""
    try:
        from oracle import cport
    except Exception as e:  # pragma: no cover - reported, not fatal
        return {"value": None, "unit": "hashes/s", "cores": 0, "kind": "port",
                "sample": "unavailable: %s" % e}, None
    n = records_np.shape[0]
    t0 = time.perf_counter()
    digests = cport.hash_fixed(records_np, 512, 32)
    passes = 1
    while time.perf_counter() - t0 < CPU_SAMPLE_S / 2:
        cport.hash_fixed(records_np, 512, 32)
        passes += 1
    dt = time.perf_counter() - t0
    T = cport.host_info()["threads_all_cores"]
    na, da = cport.hash_all_cores_timed(records_np, 512, T, CPU_SAMPLE_S / 4)
    portable = {"value": passes * n / dt, "cores": 1,
                "sample": "%d pass(es) over the %d x 512-B records of the per-GPU batch, 1 thread, portable C "
                          "BLAKE2b (oracle/c/blake2b_ref.c), %.2f s" % (passes, n, dt),
                "all_cores": {"value": na / da, "cores": T,
                              "sample": "the same records split over %d threads, %.2f s" % (T, da)}}
    try:
        avx = avx2_host_rate(records_np, digests, CPU_SAMPLE_S / 2)
    except Exception as e:  # pragma: no cover - reported, not fatal
        avx = None
        portable["avx2_error"] = str(e)
    # value: the faster of the two 1-core restatements (the baseline the reference's own
    # assembly would at least reach); both lines kept, the all-cores line the portable one's
    out = dict(portable, unit="hashes/s", kind="port", which="portable C")
    if avx is not None:
        out["avx2"] = avx
        if avx["value"] > portable["value"]:
            out.update(value=avx["value"], sample=avx["sample"], which="AVX2")
    out["note"] = ("value = the faster 1-core CPU restatement of the same hash over the same records (the AVX2 "
                   "row-vector hasher or the portable C one; Go's x/crypto/blake2b runs AVX2 assembly); both "
                   "lines are reported")
    return out, digests


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.single_process:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_selftest:  # one write(2) per line: lines of concurrent ranks never interleave
        os.write(1, (json.dumps({"rank": rank, "world": world, "gpus": args.gpus,
                                 "launch": os.environ.get("PZ_BENCH_LAUNCH", "external launcher")}) + "\n").encode())
        return
    if args.single_process:
        return single_process_main(args)
    if world > 1 and args.gpus not in (1, world):
        print("bench: --gpus %d but WORLD_SIZE %d: reporting the %d ranks that run" % (args.gpus, world, world),
              file=sys.stderr, flush=True)
    import torch
    import torch.distributed as dist

    from prysm_amd import _lib, synth

    if world > 1:
        # "nccl" is RCCL over xGMI; "gloo" only rehearses the N > 1 code path with several
        # ranks sharing one GPU (collectives through host copies; not a measurement)
        dist.init_process_group(args.backend)
    if args.backend == "gloo":
        local %= max(1, torch.cuda.device_count())
        if world > 1:
            # RCCL refuses two ranks on one device ("Duplicate GPU"): the rehearsal's library
            # communicator is the SHM one (pz_comm_init_shm), which issues the RCCL backend's
            # collective sequence through host memory and fails loudly if the ranks diverge
            args.epoch_path_note = ("gloo rehearsal: ranks share a GPU, the library's collectives over "
                                    "pz_comm_init_shm (host-staged; a code-path check, not a speed)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    _lib.lib.call("pz_init", local)

    n = args.records
    recs = synth.attestation_records_512(n, seed=2 + rank)
    d_in = torch.from_numpy(recs.reshape(-1)).to(dev)
    d_out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sh = ctypes.c_void_p(stream.cuda_stream)

    def step():
        _lib.lib.call("pz_dev_blake2b512_fixed", d_in.data_ptr(), 512, 512, n, d_out.data_ptr(), 32, sh)

    warm_clocks(step, torch, dev, args.clock_warm_ms)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    # one event pair around the K back-to-back steps: the average launch duration without
    # per-step event packets between the launches (what rocprofv3's kernel trace averages)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        wall = max_over_ranks(wall, torch, dist, dev)

    # the checker at N > 1 (and at N = 1 without the cpu_baseline leg, whose full-batch check
    # it replaces): this rank's first and last 65,536 digests against the C port
    spot = None
    if world > 1 or args.no_cpu_baseline:
        ok, what = hash_spot_check(recs, d_out)
        spot = "%s%s vs the C port (oracle/c/blake2b_ref.c): %s" % (
            what, "" if world == 1 else " of every rank", ok if world == 1 else all_ranks(ok, torch, dist, dev))

    comm = None
    if world > 1 and not args.no_epoch:
        # every rank must take the same path: agree on whether the communicator came up; a
        # failure ends the run (non-zero exit), it never switches to another path
        err = None
        try:
            comm = native_comm(dist, rank, world, local, shm=args.backend == "gloo")
        except Exception as e:
            err = "%s: %s" % (type(e).__name__, e)
        ok = torch.tensor([0.0 if err else 1.0], device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if ok.item() < 1.0:
            print("bench: rank %d: the library's RCCL communicator did not come up: %s"
                  % (rank, err or "another rank failed"), file=sys.stderr, flush=True)
            dist.destroy_process_group()
            sys.exit(3)
    epoch = None if args.no_epoch else epoch_leg(args, torch, dist, dev, rank, world, comm=comm)
    # configs[3]'s instance size (1,048,576 validators) on this one GPU: the N = 1 point of
    # the 1/2/4/8-GPU series that the N > 1 epoch leg runs (16 instances per GPU per step)
    epoch_1m = None
    if epoch is not None and world == 1 and not args.epoch_validators:
        epoch_1m = epoch_leg(args, torch, dist, dev, rank, world, nval=1 << 20, ninst=16, baseline=False)
    replay = None if args.no_replay else replay_leg(args, torch, dist, dev, rank, world)
    replay_sh = (replay_sharded_leg(args, torch, dist, dev, rank, world, comm)
                 if (world > 1 and comm is not None and not args.no_replay) else None)
    wire_out = None if args.no_wire else wire_leg(args, torch, dist, dev, rank, world)
    att_out = None if args.no_attcheck else attcheck_leg(args, torch, dist, dev, rank, world)
    watt_out = None if args.no_wire else wire_att_leg(args, torch, dist, dev, rank, world, d_out)
    shuf = shuffle_leg(args) if (rank == 0 and not args.no_epoch) else None

    if rank == 0:
        total = n * world * args.steps
        value = total / wall
        ops = n * 4 * OPS_PER_COMPRESSION
        achieved = ops / (kern_ms * 1e-3)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "hashes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": "batched BLAKE2b-512[:32] of 512-B proto3 AttestationRecord "
                                   "encodings (BASELINE configs[1])",
                       "records_per_gpu": n, "record_bytes": 512, "global_batch": n * world,
                       "parallelism": "batch-shard x%d" % world},
            "roofline": {
                "bound": "valu",
                "achieved": achieved / 1e12,
                "peak": VALU_PEAK / 1e12,
                "unit": "T full-rate-slot lane-ops/s",
                "frac": achieved / VALU_PEAK,
                "cost_model": "per compression 96 G x (6 add64 @1/0.304 + 8 xor + 6 alignbit @1/0.602) + 32 xor "
                              "= %.0f full-rate slots" % OPS_PER_COMPRESSION,
                "traffic": pmc_traffic([HASH_KERNEL]) if n == 1 << 20 else None,
                "traffic_source": PMC_SUMMARY,
                "kernel": HASH_KERNEL,
                "kernel_ms": kern_ms,
                "algorithmic_ops_per_launch": ops,
                "hbm_view": {"bytes_per_launch": n * (512 + 32),
                             "achieved_GBps": n * 544 / (kern_ms * 1e-3) / 1e9,
                             "peak_GBps": HBM_PEAK / 1e9},
            },
        }
        if world == 1:
            line["host_api"] = host_api_rate(recs)
        line["host"] = host_info()
        if world == 1 and not args.no_cpu_baseline:
            cb, digests = cpu_baseline(recs)
            line["cpu_baseline"] = cb
            if digests is not None:  # the checker: GPU digests of the timed batch vs the C port
                gpu = d_out.cpu().numpy().reshape(n, 32)
                line["parity"] = "bit-exact vs cpu_baseline on all %d digests: %s" % (
                    n, bool(np.array_equal(gpu, digests)))
        if spot is not None:
            line["parity"] = spot
        line["launch"] = (os.environ.get("PZ_BENCH_LAUNCH", "torchrun (external launcher)") if world > 1
                          else "single process, one GPU")
        line["rccl_world"] = comm.world if comm is not None else None
        if epoch is not None:
            if getattr(args, "epoch_path_note", None):
                epoch["config"]["path_note"] = args.epoch_path_note
            line["epoch"] = epoch
        if epoch_1m is not None:
            line["epoch_1m_single_gpu"] = epoch_1m
        if replay is not None:
            if replay_sh is not None:
                # the replicas' chains are the same seed-6 chain only on rank 0; its root is
                # the one the sharded chain must reproduce
                replay_sh["root_matches_rank0_replica"] = (
                    replay_sh["cand_crystallized_root"] == replay.get("cand_crystallized_root", ""))
                replay["sharded"] = replay_sh
            line["replay"] = replay
        if wire_out is not None:
            line["wire"] = wire_out
        if att_out is not None:
            line["attcheck"] = att_out
        if watt_out is not None:
            line["wire_att"] = watt_out
        if shuf is not None:
            line["shuffle"] = shuf
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if comm is not None:
        comm.free()
    if rank == 0:
        if world > 1 and args.backend == "nccl" and not args.no_single_process_leg:
            # the other ranks have left the process group (and exit); rank 0 runs the
            # one-process form over all the node's GPUs in a child process with a time limit
            del d_in, d_out
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
            line["single_process"] = single_process_child(args, world)
        print(json.dumps(line), flush=True)


def single_process_child(args, ndev):
    """Rank 0's child run of ``bench.py --single-process --gpus ndev`` (hash + epoch legs),
    under a time limit; its JSON line, or the reason it has none."""
    import subprocess

    cmd = [sys.executable, os.path.abspath(__file__), "--single-process", "--gpus", str(ndev), "--steps",
           str(args.steps), "--warmup", str(args.warmup), "--records", str(args.records), "--no-cpu-baseline",
           "--replay-blocks", str(args.replay_blocks)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                           "GROUP_RANK", "ROLE_RANK", "MASTER_PORT")}
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=args.single_process_timeout)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after %.0f s" % args.single_process_timeout, "cmd": " ".join(cmd)}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": "exit %d" % r.returncode, "stderr_tail": r.stderr[-2000:], "cmd": " ".join(cmd)}
    return json.loads(lines[-1])


def single_process_main(args):
    """``--single-process --gpus N``: ONE process drives N GPUs, the form a Go node links (one
    beacon-chain process, ``blockchain/service.go:229``).  The communicator is
    ``pz_init_devices(N)`` (ncclCommInitAll; every collective is a grouped RCCL call over the
    per-device streams, comm.hip), and:

    * hash: each device hashes its own 1M-record batch (configs[1] per GPU, no collective);
    * epoch: configs[3], B = 16 N instances of 1,048,576 validators sharded over the N
      devices by ``pz_epoch_state`` (one-pass step, one grouped collective per part).

    Wall clock over K steps on all devices; device time by HIP events on every shard's stream."""
    import torch

    from prysm_amd import _lib, casper, synth
    from prysm_amd.native import Comm, NativeEpoch

    N = args.gpus
    comm = Comm.devices(N)
    devs = [torch.device("cuda", i) for i in range(N)]
    n = args.records
    d_in, d_out, streams = [], [], []
    for i, dv in enumerate(devs):
        torch.cuda.set_device(dv)
        _lib.lib.call("pz_init", i)
        d_in.append(torch.from_numpy(synth.attestation_records_512(n, seed=2 + i).reshape(-1)).to(dv))
        d_out.append(torch.empty(n * 32, dtype=torch.uint8, device=dv))
        streams.append(torch.cuda.current_stream(dv))

    def hash_step():
        for i, dv in enumerate(devs):
            torch.cuda.set_device(dv)
            _lib.lib.call("pz_dev_blake2b512_fixed", d_in[i].data_ptr(), 512, 512, n, d_out[i].data_ptr(), 32,
                          ctypes.c_void_p(streams[i].cuda_stream))

    def sync_all():
        for dv in devs:
            torch.cuda.synchronize(dv)

    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < args.clock_warm_ms:
        for _ in range(8):
            hash_step()
        sync_all()
    for _ in range(args.warmup):
        hash_step()
    sync_all()
    evs = []
    for i, dv in enumerate(devs):
        torch.cuda.set_device(dv)
        evs.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        evs[-1][0].record(streams[i])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        hash_step()
    for i, dv in enumerate(devs):
        torch.cuda.set_device(dv)
        evs[i][1].record(streams[i])
    sync_all()
    wall = time.perf_counter() - t0
    kern_ms = max(e0.elapsed_time(e1) for e0, e1 in evs) / args.steps
    spots = [hash_spot_check(synth.attestation_records_512(n, seed=2 + i), d_out[i]) for i in range(N)]
    hash_out = {"value": n * N * args.steps / wall, "unit": "hashes/s", "ms_per_step": wall / args.steps * 1e3,
                "kernel_ms_max_over_devices": kern_ms,
                "roofline_frac": n * 4 * OPS_PER_COMPRESSION / (kern_ms * 1e-3) / VALU_PEAK,
                "parity": "%s of every device vs the C port: %s" % (spots[0][1], all(ok for ok, _ in spots))}
    del d_in, d_out
    torch.cuda.set_device(devs[0])

    nval = 1 << 20
    ninst = 16 * N
    shuffled = casper.shuffle_indices(b"A" + bytes(31), np.arange(nval, dtype=np.uint32))
    inst = synth.epoch_batch(nval, ninst, seed=3, shuffled=shuffled)
    one = synth.epoch_instances(inst, 1)  # the checker's instance
    de = NativeEpoch(inst, device=0, comm=comm)
    bpv = epoch_layout_bytes(inst, de) or EPOCH_BYTES_PER_VALIDATOR
    del inst
    for _ in range(args.warmup + 30):
        de.step()
    de.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        de.step()
    de.sync()
    wall_e = time.perf_counter() - t0
    comm.set_timing(True)
    comm.collective_time()
    for _ in range(args.steps):
        de.step()
    cms, cn = comm.collective_time()
    comm.set_timing(False)
    epoch_out = {"value": nval * ninst * args.steps / wall_e, "unit": "validator-epochs/s",
                 "ms_per_step": wall_e / args.steps * 1e3,
                 "config": {"validators": nval, "instances_per_step": ninst,
                            "layout": "committee order, one-pass step" if de.one_pass else
                                      "committee order, two-pass step" if de.committee_order else "index order",
                            "shards": [list(de.shard(i)[:3]) for i in range(de.nlocal)]},
                 "bytes_per_validator_epoch": bpv,
                 "algorithmic_GBps_per_gpu": nval * 16 * bpv / (wall_e / args.steps) / 1e9,
                 "collectives": {"ms_per_step": cms / args.steps, "per_step": cn / args.steps,
                                 "what": "device time of the grouped collectives (max over the devices), HIP events "
                                         "on the communicator's streams, %d steps after the timed loop" % args.steps}}
    de.free()
    # the checker: instance 0, one fresh sharded step, every device's range vs oracle/epoch_np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from epoch_ref_helpers import oracle_epoch
    pe = NativeEpoch(one, device=0, comm=comm)
    pe.step()
    pe.sync()
    pe.tallies()
    nb, applied, nxt, v, t, w = oracle_epoch(one, 0)
    ok = True
    for i in range(pe.nlocal):
        bal, scal, vote, total, win = pe.results(i)
        idx = pe.validators(i)
        ok &= (np.array_equal(bal[0], nb[idx]) and bool(scal[0, _lib.SCAL_APPLIED]) == applied
               and int(scal[0, _lib.SCAL_NEXT_BAL]) == nxt and np.array_equal(vote[0], v)
               and np.array_equal(total[0], t) and np.array_equal(win[0], w))
    pe.free()
    epoch_out["parity"] = ("instance 0, one sharded step, every device's validator range bit-exact vs "
                           "oracle/epoch_np: %s" % ok)
    # configs[4] as one chain over the N devices of this process (pz_chain_new_comm)
    from prysm_amd.blockchain import BeaconChain, serialize_blocks
    blocks = synth.chain_blocks(65536, args.replay_blocks, seed=6)
    data, offs = serialize_blocks(blocks)
    BeaconChain(65536, comm=comm).process_serialized(*serialize_blocks(blocks[:130]))
    ch = BeaconChain(65536, comm=comm)
    t0 = time.perf_counter()
    br, ar = ch.process_serialized(data, offs)
    wall_r = time.perf_counter() - t0
    roots = ch.roots()
    from replay_port_helpers import mismatches, port_replay
    p_out, p_roots = port_replay(data, offs, 65536, len(ar))
    bad = mismatches(br, ar, roots, p_out, p_roots)
    replay_out = {"value": args.replay_blocks / wall_r, "unit": "blocks/s", "transitions": int(br["transition"].sum()),
                  "processed": int((br["status"] == 0).sum()),
                  "parity": "every block, attestation, root and vote-cache total vs oracle/c/replay_ref.c: %s" % (
                      "bit-exact" if not bad else "MISMATCH " + ", ".join(bad)),
                  "cand_crystallized_root": roots.get("cand_crystallized", b"").hex()}
    del ch
    line = {"metric": METRIC, "mode": "single process, %d GPUs (pz_init_devices -> ncclCommInitAll)" % N,
            "n_gpus": N, "rccl_world": comm.world, "rccl_nlocal": comm.nlocal, "steps": args.steps,
            "warmup": args.warmup, "hash": hash_out, "epoch": epoch_out, "replay_one_chain": replay_out}
    comm.free()
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
