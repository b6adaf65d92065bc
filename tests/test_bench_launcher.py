"""bench.py's multi-GPU launcher (`python bench.py --gpus N` with no
torch.distributed.run around it): argument/environment logic and the
spawn-and-wait of the rank processes, on the CPU."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _no_count():
    raise AssertionError("device_count() must not be called here")


def test_single_gpu_runs_in_process():
    b = _bench()
    assert b.launch_plan(1, {}, _no_count) == ("run", None)


def test_world_size_set_must_match_gpus():
    b = _bench()
    assert b.launch_plan(4, {"WORLD_SIZE": "4"}, _no_count) == ("run", None)
    what, msg = b.launch_plan(8, {"WORLD_SIZE": "1"}, _no_count)
    assert what == "error" and "WORLD_SIZE=1" in msg and "--gpus 8" in msg
    what, _ = b.launch_plan(1, {"WORLD_SIZE": "2"}, _no_count)
    assert what == "error"


def test_nccl_needs_one_gpu_per_rank():
    b = _bench()
    what, msg = b.launch_plan(2, {}, lambda: 1)
    assert what == "error" and "needs 2 GPUs" in msg and "has 1" in msg
    what, msg = b.launch_plan(8, {"GDSP_DIST_BACKEND": "nccl"}, lambda: 0)
    assert what == "error"


def test_spawn_environments():
    b = _bench()
    what, ranks = b.launch_plan(8, {"PATH": "/bin"}, lambda: 8)
    assert what == "spawn" and len(ranks) == 8
    ports = {e["MASTER_PORT"] for e in ranks}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, e in enumerate(ranks):
        assert e["RANK"] == str(r) and e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == "8" and e["MASTER_ADDR"] == "127.0.0.1"
        assert e["PATH"] == "/bin"


def test_gloo_rehearsal_spawns_without_counting():
    b = _bench()
    what, ranks = b.launch_plan(2, {"GDSP_DIST_BACKEND": "gloo", "MASTER_PORT": "29555"},
                                _no_count)
    assert what == "spawn" and [e["MASTER_PORT"] for e in ranks] == ["29555", "29555"]


def test_bad_gpu_count():
    b = _bench()
    assert b.launch_plan(0, {}, _no_count)[0] == "error"


CHILD = r"""
import json, os, sys
r = int(os.environ["RANK"])
print(f"[Gloo] Rank {r} is connected to 2 peer ranks.", flush=True)  # stdout noise
if os.environ.get("FAIL_RANK") == str(r):
    sys.exit(3)
if os.environ.get("HANG_RANK") == str(r):
    import time; time.sleep(600)
if r == 0:
    print(json.dumps({"n_gpus": int(os.environ["WORLD_SIZE"]), "rank": r}), flush=True)
"""


def _run_launch(tmp_path, n, extra=None):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    code = (
        "import importlib.util, os, sys\n"
        f"spec = importlib.util.spec_from_file_location('b', {os.path.join(REPO, 'bench.py')!r})\n"
        "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
        f"what, ranks = b.launch_plan({n}, dict(os.environ), lambda: 0)\n"
        "assert what == 'spawn', (what, ranks)\n"
        f"sys.exit(b.launch([sys.executable, {str(script)!r}], ranks, poll_s=0.05))\n")
    env = dict(os.environ, GDSP_DIST_BACKEND="gloo", **(extra or {}))
    env.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                          timeout=60)


def test_launch_forwards_rank0_line(tmp_path):
    p = _run_launch(tmp_path, 3)
    assert p.returncode == 0, p.stderr
    # only rank 0's JSON line reaches stdout; the ranks' other stdout lines
    # go to stderr
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1 and json.loads(lines[0]) == {"n_gpus": 3, "rank": 0}
    assert p.stderr.count("[Gloo] Rank") == 3


def test_launch_fails_loud_and_ends_the_others(tmp_path):
    # rank 1 fails while rank 2 would sleep for 10 minutes: the launcher must
    # return rank 1's status promptly, having ended rank 2
    p = _run_launch(tmp_path, 3, {"FAIL_RANK": "1", "HANG_RANK": "2"})
    assert p.returncode == 3, (p.returncode, p.stderr)


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "must agree" in p.stderr


def test_bench_nccl_without_enough_gpus_exits_nonzero():
    # this container has no GPU: `bench.py --gpus 2` (nccl) must refuse
    # instead of timing one rank and printing an n_gpus = 1 line
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GDSP_DIST_BACKEND"):
        env.pop(k, None)
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("node has two GPUs")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "needs 2 GPUs" in p.stderr, (p.returncode, p.stderr)
    assert p.stdout.strip() == ""


def _fake_kfd(root, nodes):
    # nodes: list of (gpu_id, simd_count); node 0 of a real topology is the CPU
    for i, (gid, simd) in enumerate(nodes):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "gpu_id").write_text(f"{gid}\n")
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\nmax_waves_per_simd 8\n")
    return str(root)


def test_kfd_gpu_count_reads_sysfs(tmp_path):
    b = _bench()
    root = _fake_kfd(tmp_path / "nodes", [(0, 0)] + [(1000 + i, 1024) for i in range(8)])
    assert b.kfd_gpu_count(root, env={}) == 8
    assert b.kfd_gpu_count(root, env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert b.kfd_gpu_count(root, env={"ROCR_VISIBLE_DEVICES": "3", "HIP_VISIBLE_DEVICES": "0,1"}) == 1
    assert b.kfd_gpu_count(root, env={"CUDA_VISIBLE_DEVICES": ""}) == 0
    assert b.kfd_gpu_count(str(tmp_path / "missing"), env={}) is None


def test_launcher_count_loads_no_gpu_runtime(tmp_path):
    # the launcher parent counts devices from sysfs: no torch / HIP module is
    # imported by the count itself when the topology is readable
    root = _fake_kfd(tmp_path / "nodes", [(0, 0), (7, 256)])
    code = ("import importlib.util, sys\n"
            f"spec = importlib.util.spec_from_file_location('b', {os.path.join(REPO, 'bench.py')!r})\n"
            "b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)\n"
            f"b.KFD_NODES = {root!r}\n"
            "n = b._device_count()\n"
            "assert n == 1, n\n"
            "assert 'torch' not in sys.modules, 'torch imported by the launcher count'\n")
    env = {k: v for k, v in os.environ.items() if not k.endswith("VISIBLE_DEVICES")}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       env=env)
    assert p.returncode == 0, p.stderr


def test_rank_device_check():
    b = _bench()
    # one GPU per local rank
    assert b.rank_device_check(8, 3, "nccl", {"LOCAL_WORLD_SIZE": "8"}, 8) is None
    # a two-node job of 16 ranks, 8 per node: only the node's ranks count
    assert b.rank_device_check(8, 7, "nccl", {"LOCAL_WORLD_SIZE": "8"}, 16) is None
    # a launcher that gives each rank one GPU through HIP_VISIBLE_DEVICES
    assert b.rank_device_check(1, 5, "nccl", {"LOCAL_WORLD_SIZE": "8",
                                              "HIP_VISIBLE_DEVICES": "5"}, 8) is None
    # too few GPUs for the node's ranks
    msg = b.rank_device_check(1, 1, "nccl", {"LOCAL_WORLD_SIZE": "2"}, 2)
    assert msg and "need 2 GPUs" in msg
    assert b.rank_device_check(4, 0, "nccl", {}, 8) is not None
    # the gloo rehearsal shares one GPU
    assert b.rank_device_check(1, 1, "gloo", {"LOCAL_WORLD_SIZE": "2"}, 2) is None
