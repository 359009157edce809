"""bench.py's rank launcher (CPU): `bench.py --gpus N` started without
torchrun runs N rank processes as its children and returns their status;
a launcher world that disagrees with --gpus is refused.  The ranks run the
launch probe (UNIPEAK_BENCH_LAUNCH_PROBE: a gloo all-reduce, no GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    e.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True,
                          timeout=240)


def last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = run(["--gpus", str(n), "--steps", "3"], UNIPEAK_BENCH_LAUNCH_PROBE="0")
    assert r.returncode == 0, r.stderr[-2000:]
    d = last_json(r.stdout)
    assert d["n_gpus"] == n
    assert d["rank_sum"] == n * (n - 1) // 2  # every rank joined one world
    assert d["local_world"] == n              # one node, one process per GPU
    assert f"launching {n} ranks" in r.stderr


def test_failing_rank_fails_the_launch():
    r = run(["--gpus", "2"], UNIPEAK_BENCH_LAUNCH_PROBE="3")
    assert r.returncode != 0
    assert "rank processes failed" in r.stderr


def test_world_mismatch_refused():
    r = run(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    r = run(["--gpus", "1"], WORLD_SIZE="8", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2


def test_bad_gpus_and_one_gpu_workload():
    assert run(["--gpus", "0"]).returncode != 0
    r = run(["--gpus", "2", "--workload", "hg19-shift"])
    assert r.returncode != 0 and "one GPU" in r.stderr
