"""bench.py's launcher contract (CPU, no GPU touched): `--gpus N` without a launcher starts N ranks
itself; under a launcher whose WORLD_SIZE differs from N it exits non-zero before any work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


def test_bench_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["world"] == 2 and d["ranks_seen"] == 2 and d["local_world"] == 2


def test_bench_mismatched_launcher_exits_nonzero():
    r = _run(["--gpus", "4", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
