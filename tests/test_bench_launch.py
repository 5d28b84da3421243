"""bench.py --gpus N owns its rank setup (the reference's program
sets up its own ranks, mpi-horz-driver.cpp:14-32).

CPU (-m "not gpu"): the launch decision (bench.launch_plan) for every combination of
--gpus, $WORLD_SIZE, visible devices and --share-gpu; the refusals end bench.py with
status 2 and a message before any GPU call; the one-host check of the per-fill clock
over a world-2 gloo group.
GPU (-m gpu): `python bench.py --gpus 2 --share-gpu` with NO launcher starts its two
ranks itself and prints one line with n_gpus 2 and a golden score.
"""
import datetime
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

sys.path.insert(0, ROOT)
sys.path.insert(0, PKG)
import bench  # noqa: E402
import nw_bands  # noqa: E402


@pytest.mark.parametrize("gpus,world,ndev,share,want", [
    (1, None, 0, False, "single"),
    (1, None, 1, False, "single"),
    (1, "1", 1, False, "single"),
    (2, None, 8, False, "spawn"),
    (8, None, 8, False, "spawn"),
    (2, None, 1, True, "spawn"),
    (8, "8", 8, False, "ranks"),
    (2, "2", 1, True, "ranks"),
    (3, "3", 1, True, "ranks"),
])
def test_launch_plan(gpus, world, ndev, share, want):
    assert bench.launch_plan(gpus, world, ndev, share) == (want, "")


@pytest.mark.parametrize("gpus,world,ndev,share,needle", [
    (2, None, 1, False, "visible GPU"),      # too few devices, no --share-gpu
    (8, None, 4, False, "visible GPU"),
    (2, None, 0, True, "no visible GPU"),    # sharing needs one device
    (8, "4", 8, False, "WORLD_SIZE=4"),      # launcher rank count != --gpus
    (1, "8", 8, False, "WORLD_SIZE=8"),      # 8 ranks, each believing it is alone
    (2, "2", 1, False, "visible GPU"),       # launched, but one GPU for two ranks
    (2, "x", 8, False, "not an integer"),
    (0, None, 8, False, "at least 1"),
])
def test_launch_plan_refusals(gpus, world, ndev, share, needle):
    plan, why = bench.launch_plan(gpus, world, ndev, share)
    assert plan == "refuse" and needle in why


def _run_bench(args, **env_over):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over)
    env["PYTHONPATH"] = PKG
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True,
                          text=True, timeout=300, env=env, cwd=ROOT)


def test_bench_refuses_rank_mismatch_before_any_gpu_call():
    out = _run_bench(["--gpus", "8", "--steps", "1", "--warmup", "0"], WORLD_SIZE="2")
    assert out.returncode == 2
    assert "refusing" in out.stderr and "WORLD_SIZE=2 but --gpus 8" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.skipif(__import__("torch").cuda.device_count() > 0,
                    reason="this host has a GPU: the no-device refusal is a CPU-host case")
def test_bench_refuses_without_devices_instead_of_spawning():
    out = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert out.returncode == 2 and "visible GPU" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


def test_same_host():
    assert nw_bands.same_host(["a", "a", "a"]) and nw_bands.same_host([])
    assert not nw_bands.same_host(["a", "b"])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _host_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, PKG)
    import nw_bands as nb
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    try:
        nb.check_one_host(world)
        q.put((rank, "ok"))
    except RuntimeError as e:  # pragma: no cover (one host here)
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_check_one_host_gloo_world2():
    """The ranks' host names over a real world-2 gloo group: one host passes."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_host_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    assert res == {0: "ok", 1: "ok"}


@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.mark.gpu
def test_bench_self_launches_two_ranks(torch_gpu):
    """No launcher: bench.py starts 2 ranks itself (sharing the GPU), rank 0's line is
    the command's line: n_gpus 2, requested_gpus 2, the one-GPU rehearsal table
    (524288 x 65536, two bands of 32768 rows) with its golden score."""
    out = _run_bench(["--gpus", "2", "--share-gpu", "--steps", "2", "--warmup", "1", "--band-rows", "32768",
                      "--alt-partition", "none", "--no-cpu-baseline"])
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["requested_gpus"] == 2 and res["launcher"] == "self"
    assert res["config"]["n1"] == 524288 and res["config"]["n2"] == 65536
    assert res["score_ok"] is True, (res["score"], res["score_golden"])
