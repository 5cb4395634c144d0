"""bench.py's multi-rank launch (VERDICT r05 Next 1), on the CPU.

`python bench.py --gpus N` without a launcher must start N ranks itself (fresh
processes, before any GPU call), report `n_gpus: N`, and a WORLD_SIZE that
disagrees with --gpus must fail instead of silently measuring one GPU.
`--launcher-selftest` stops each rank right after it joined the gloo group, so
nothing here loads librsketch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=timeout)


def test_launcher_spawns_three_ranks_into_one_group():
    p = _run(["--gpus", "3", "--launcher-selftest"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # only rank 0's line reaches the caller
    d = json.loads(lines[0])
    assert d["launcher_selftest"] is True and d["n_gpus"] == 3
    assert [e["rank"] for e in d["ranks"]] == [0, 1, 2]
    assert [e["local_rank"] for e in d["ranks"]] == [0, 1, 2]
    assert len({e["pid"] for e in d["ranks"]}) == 3  # three distinct processes


def test_single_gpu_runs_in_process():
    p = _run(["--gpus", "1", "--launcher-selftest"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["ranks"][0]["rank"] == 0


def test_world_size_mismatch_is_refused():
    p = _run(["--gpus", "3", "--launcher-selftest"],
             _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29555"))
    assert p.returncode != 0
    assert "refusing" in p.stderr
    # the reverse: a launcher with 2 ranks around a --gpus 1 command
    p = _run(["--launcher-selftest"], _env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1"))
    assert p.returncode != 0 and "refusing" in p.stderr


def test_a_failing_rank_fails_the_launch():
    # rank 1 exits with 3 after joining; ranks 0 and 2 would wait for it in a
    # collective forever, so the launcher must stop them and fail
    p = _run(["--gpus", "3", "--launcher-selftest"], _env(RSK_SELFTEST_FAIL_RANK="1"), timeout=120)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert "rank 1 exited with 3" in p.stderr
    assert p.stdout.strip() == ""
    p = _run(["--gpus", "0", "--launcher-selftest"], _env())
    assert p.returncode != 0
