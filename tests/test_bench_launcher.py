"""bench.py's multi-rank launch on the CPU (gloo, --dry: the launcher, process group, barriers and
max-over-ranks timing with no HIP work): `--gpus N` without WORLD_SIZE starts N ranks itself, every
rank joins, rank 0 alone prints one line with n_gpus = N; a WORLD_SIZE that disagrees with --gpus
is refused."""
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def _lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_gpus_2_starts_two_ranks_and_prints_one_line():
    p = _run(["--gpus", "2", "--dry", "--backend", "gloo", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _lines(p.stdout)
    assert len(lines) == 1, p.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["ranks_joined"] == 2 and d["backend"] == "gloo"
    assert d["config"]["parallelism"] == "dp2"


def test_gpus_4_ranks():
    p = _run(["--gpus", "4", "--dry", "--backend", "gloo", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    (d,) = _lines(p.stdout)
    assert d["n_gpus"] == 4 and d["ranks_joined"] == 4 and d["config"]["parallelism"] == "dp4"


def test_gpus_1_is_a_single_process():
    p = _run(["--dry", "--steps", "2", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    (d,) = _lines(p.stdout)
    assert d["n_gpus"] == 1 and d["backend"] is None and d["config"]["parallelism"] == "single"


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--dry", "--backend", "gloo"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=4" in p.stderr
    assert not _lines(p.stdout)


def test_gloo_needs_dry():
    p = _run(["--backend", "gloo"])
    assert p.returncode != 0 and "--dry" in p.stderr


def test_rank_that_never_joins_ends_every_rank_nonzero():
    """A rank that never reaches the rendezvous (test hook) must not hang the run until the driver's
    limit: the others time out after --pg-timeout with a message, exit non-zero, the parent stops the
    absent one and exits non-zero, listing every rank's status."""
    t0 = time.time()
    p = _run(["--gpus", "2", "--dry", "--backend", "gloo", "--steps", "2", "--warmup", "1", "--pg-timeout", "8",
              "--dry-absent-rank", "1"], timeout=120)
    elapsed = time.time() - t0
    assert p.returncode != 0, p.stdout + p.stderr[-2000:]
    assert not _lines(p.stdout)
    assert "did not form within 8 s" in p.stderr, p.stderr[-2000:]
    m = re.search(r"rank exit statuses \[([^\]]*)\]", p.stderr)
    assert m, p.stderr[-2000:]
    statuses = [int(x) for x in m.group(1).split(",")]
    assert len(statuses) == 2 and all(s != 0 for s in statuses), statuses
    assert elapsed < 60, elapsed
