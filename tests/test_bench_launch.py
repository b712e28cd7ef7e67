"""CPU: ``python bench.py --gpus N`` starts its own N ranks (torch.distributed.run as a child
process, 127.0.0.1 rendezvous) and every rank sees WORLD_SIZE = N; inside a launcher a world size
that differs from --gpus is a hard error.  ``--rank-check`` makes each rank report and exit before
any GPU call."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=120)


def test_bench_starts_its_own_ranks():
    r = _run(["--gpus", "2", "--rank-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["n_gpus"] == 2 for x in lines)


def test_single_gpu_default_runs_one_rank_in_process():
    r = _run(["--rank-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip()) == {"rank": 0, "local_rank": 0, "n_gpus": 1}


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--rank-check"], env={"WORLD_SIZE": "3", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
