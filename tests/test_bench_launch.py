"""bench.py's launch logic on the CPU: how `--gpus N` becomes ranks with and
without an external launcher, and that too few visible
GPUs end the run with a non-zero status instead of a silent one-GPU line."""
import os
import subprocess
import sys
import threading

import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _count(n):
    calls = []

    def f():
        calls.append(1)
        return n

    f.calls = calls
    return f


def test_single_gpu_default():
    p = bench.plan_launch(1, {}, _count(0))
    assert p["mode"] == "single" and p["world"] == 1 and p["devices"] == [0] and p["ranks"] == [0]


def test_single_gpu_honours_krylov_device():
    assert bench.plan_launch(1, {"KRYLOV_DEVICE": "3"}, _count(8))["devices"] == [3]


def test_plain_gpus_n_drives_n_devices_in_one_process():
    c = _count(8)
    p = bench.plan_launch(8, {}, c)
    assert p["mode"] == "threads" and p["world"] == 8
    assert p["devices"] == list(range(8)) and p["ranks"] == list(range(8))
    assert c.calls  # the device count was checked


@pytest.mark.parametrize("gpus,have", [(2, 1), (8, 4), (4, 0)])
def test_too_few_devices_exit_nonzero(gpus, have):
    with pytest.raises(SystemExit) as e:
        bench.plan_launch(gpus, {}, _count(have))
    assert f"only {have} GPU" in str(e.value.code)


def test_torchrun_env_wins():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    p = bench.plan_launch(4, env, _count(4))
    assert p["mode"] == "torchrun" and p["world"] == 4 and p["rank"] == 2 and p["devices"] == [2]
    assert p["ranks"] == [2] and p["note"] is None
    p = bench.plan_launch(1, env, _count(4))
    assert p["world"] == 4 and "WORLD_SIZE 4" in p["note"]


def test_torchrun_rank_without_its_device_exits():
    with pytest.raises(SystemExit):
        bench.plan_launch(2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}, _count(1))


def test_zero_gpus_rejected():
    with pytest.raises(SystemExit):
        bench.plan_launch(0, {}, _count(8))


def test_run_all_runs_every_rank_concurrently_and_raises_the_first_error():
    job = bench.Job({"mode": "threads", "world": 3, "rank": 0, "devices": [0, 1, 2], "ranks": [0, 1, 2]})
    gate = threading.Barrier(3, timeout=10)  # only passes if all three run at once

    def fn(i):
        gate.wait()
        return i * 10

    assert job.run_all(fn) == [0, 10, 20]

    def bad(i):
        if i == 1:
            raise ValueError("rank 1")
        return i

    with pytest.raises(ValueError, match="rank 1"):
        job.run_all(bad)


def test_bench_gpus_2_without_devices_fails_loudly():
    """The plain `python bench.py --gpus 2` the driver may run: on a host with
    fewer GPUs it must not print a one-GPU line."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""  # no device, also on a GPU host
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--quick", "--steps", "2"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert '"value"' not in r.stdout


def test_threads_launch_forced_at_one_gpu():
    p = bench.plan_launch(1, {}, _count(1), "threads")
    assert p["mode"] == "threads" and p["world"] == 1 and p["devices"] == [0]
