"""bench.py's multi-rank launcher on CPU (gloo): `bench.py --gpus N` started without torchrun must
start N ranks itself (one process per GPU on the driver's node, RCCL there) and report n_gpus = N;
a process group whose size differs from --gpus must fail instead of printing a mislabelled line.
--launch-check stops each rank right after the process-group check, before any GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(GS_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1", **kw)
    return env


def _json_lines(text):
    return [json.loads(x) for x in text.splitlines() if x.startswith("{")]


def test_bench_gpus2_starts_two_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["backend"] == "gloo"


def test_bench_refuses_world_size_mismatch():
    # launched as one rank of a world of 1 while claiming 2 GPUs: exit non-zero, no JSON line
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--launch-check"], cwd=ROOT,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    assert not _json_lines(r.stdout)
    assert "WORLD_SIZE=1" in r.stderr


def test_bench_single_gpu_needs_no_launcher():
    r = subprocess.run([sys.executable, "bench.py", "--launch-check"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json_lines(r.stdout)[0]["n_gpus"] == 1
