"""bench.py's launch contract on the CPU: `bench.py --gpus N` with no launcher starts N ranks
itself and reports n_gpus = N; a launcher's WORLD_SIZE that disagrees with --gpus is an error, not a silent
one-GPU run.  The ranks run the hidden --launch-check body (gloo all-reduce, no GPU)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                          env=env, timeout=timeout)


def _json_lines(out):
    return [json.loads(s) for s in out.splitlines() if s.strip().startswith("{")]


def test_gpus_2_self_launches_two_ranks():
    p = _run(["--gpus", "2", "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout          # exactly one JSON line on stdout, re-printed by the parent
    assert lines[0]["n_gpus"] == 2 and lines[0]["value"] == 2.0 and lines[0]["launched_by_bench"]


def test_gpus_1_runs_in_process():
    p = _run(["--gpus", "1", "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 1 and not line["launched_by_bench"]


def test_world_size_mismatch_fails_loudly():
    p = _run(["--gpus", "1", "--launch-check"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0
    assert "must agree" in p.stderr
    assert not _json_lines(p.stdout)


def test_watchdog_prints_the_headline_when_a_secondary_line_hangs():
    """Both ranks stall in a 'secondary line' for 60 s; the 3 s watchdog prints rank 0's line and every rank exits 0."""
    p = _run(["--gpus", "2", "--launch-check", "--hang-check", "60", "--secondary-timeout", "3"], timeout=50)
    assert p.returncode == 0, p.stderr[-3000:]
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 2 and "watchdog" in line["secondary_lines"]
