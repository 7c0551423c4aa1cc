"""bench.py's multi-GPU launch (VERDICT r2 "next" 1): ``--gpus N`` without a launcher starts
``torch.distributed.run`` with N ranks as a child process, forwards its output and exits with
its code; ``--single-process`` drives N devices from one process through ``pz_init_devices``.

CPU: the launcher itself (ranks report RANK/WORLD_SIZE before any GPU call) and the exit-code
propagation.  GPU: the whole bench at world 2 over gloo on the one-GPU test box (the ranks
share cuda:0, so the epoch runs the torch.distributed orchestration, labelled), and the
single-process form at one device (ncclCommInitAll over one GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, timeout):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=ROOT)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-selftest"], 180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert sorted(x["rank"] for x in lines) == list(range(n))
    assert all(x["world"] == n and x["launch"].startswith("torchrun child") for x in lines)


def test_gpus_1_stays_in_process():
    r = _run(["--gpus", "1", "--launch-selftest"], 120)
    assert r.returncode == 0, r.stderr[-2000:]
    (x,) = _json_lines(r.stdout)
    assert (x["rank"], x["world"]) == (0, 1)


def test_rank_failure_is_the_exit_code():
    """Ranks that fail (``--records -1`` raises in every rank; on a CPU-only host the device
    selection fails first) make the launcher exit non-zero, with no bench line printed."""
    r = _run(["--gpus", "2", "--backend", "gloo", "--records", "-1"], 240)
    assert r.returncode != 0
    assert not any(x.get("n_gpus") for x in _json_lines(r.stdout))


@pytest.mark.gpu
def test_bench_world2_gloo_rehearsal():
    r = _run(["--gpus", "2", "--backend", "gloo", "--no-cpu-baseline", "--records", "4096", "--replay-blocks", "130",
              "--steps", "2", "--warmup", "1", "--clock-warm-ms", "0", "--epoch-validators", "65536",
              "--epoch-instances", "4", "--no-wire", "--no-attcheck"], 600)
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = [x for x in _json_lines(r.stdout) if "metric" in x]
    assert line["n_gpus"] == 2 and line["launch"].startswith("torchrun child")
    assert line["epoch"]["config"]["path_note"].startswith("gloo rehearsal")
    assert line["replay"]["processed"] == 130 * 2 // 2  # blocks per rank (every block processed)


@pytest.mark.gpu
def test_bench_single_process_one_device():
    r = _run(["--single-process", "--gpus", "1", "--records", "4096", "--steps", "2", "--warmup", "1", "--replay-blocks", "130",
              "--clock-warm-ms", "0"], 600)
    assert r.returncode == 0, r.stderr[-3000:]
    (line,) = _json_lines(r.stdout)
    assert line["rccl_world"] == 1 and line["rccl_nlocal"] == 1
    assert line["epoch"]["config"]["layout"] == "committee order, one-pass step"
    assert line["hash"]["value"] > 0 and line["epoch"]["value"] > 0
    assert line["replay_one_chain"]["transitions"] == 2


def test_bench_traffic_summaries_present_and_shipped():
    """Every kernel whose counted HBM traffic the bench line quotes has it in the committed PMC
    summaries of this round (a kernel renamed since the counter passes reads None), and those
    summaries are not excluded from the tree gpurun ships to the GPU box (.gpurunignore)."""
    import fnmatch

    sys.path.insert(0, ROOT)
    import bench

    quoted = [([bench.HASH_KERNEL], "main"), (["pz_wire_val_kernel"], "main"), (["pz_att_check_p_kernel"], "main"),
              (["pz_wire_att_size_kernel", "pz_wire_att_write_kernel"], "main")]
    quoted += [(["pz_epoch_*"], w) for w in ("epoch65k", "epoch1m", "epoch65k_cold", "epoch1m_cold")]
    for kernels, workload in quoted:
        assert bench.pmc_traffic(kernels, workload), (kernels, workload)
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        pats = [ln.strip() for ln in f if ln.strip()]
    for workload in {w for _, w in quoted}:
        rel = "./" + bench.pmc_summary_path(workload).replace(os.sep, "/")
        for pat in pats:
            parts = rel.split("/")
            prefixes = ["/".join(parts[:i]) for i in range(2, len(parts) + 1)]
            assert not any(fnmatch.fnmatch(p, pat) or fnmatch.fnmatch(p[2:], pat) for p in prefixes), (rel, pat)
