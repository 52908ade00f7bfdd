"""bench.py's multi-rank entry without an external launcher (CPU, gloo).

``python bench.py --gpus N`` with no WORLD_SIZE spawns the N rank processes itself; under a
launcher WORLD_SIZE must equal --gpus.  ``--selftest`` runs the launcher, barrier, timed
region and MAX-over-ranks reduction with a CPU stand-in step, so the plumbing is checked here
without a GPU (the real forward path is the same code after the rank setup)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus2_spawns_two_ranks_one_line():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--selftest", "--steps", "3", "--warmup", "1",
                        "--batch", "16"], capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]   # gloo logs a line too
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["slots_total"] == 2 * 16 * 3
    assert d["ranks_spawned_by"] == "bench.py"
    assert d["value"] > 0


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--selftest", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=120,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
