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
    """Both ranks stall in a 'secondary line' for 60 s; the 3 s watchdog prints rank 0's line and every rank exits
    with the watchdog status (a hang in a multi-rank line must fail the run visibly, not exit 0), which
    the self-launching parent passes through."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    p = _run(["--gpus", "2", "--launch-check", "--hang-check", "60", "--secondary-timeout", "3"], timeout=50)
    assert p.returncode == bench.WATCHDOG_EXIT != 0, p.stderr[-3000:]
    (line,) = _json_lines(p.stdout)
    assert line["n_gpus"] == 2 and "watchdog" in line["secondary_lines"]


def test_multi_rank_line_carries_no_unlabelled_one_gpu_profile_figures():
    """the committed rocprofv3 / PMC figures are this command's own only at N = 1; at N > 1 the
    roofline must not carry them as if measured (kernel_trace_*, traffic) -- they sit under profile_1gpu, with a
    note."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    N, L, B = 1 << 16, 8, 1024
    alg = 16.0 * N * L * B
    one = bench.profile_figures(N, L, B, alg, 1)
    assert "traffic" in one and "kernel_trace_frac" in one   # the committed profiles of the default command
    for world in (2, 4, 8):
        many = bench.profile_figures(N, L, B, alg, world)
        assert set(many) == {"profile_1gpu"}
        assert not any(k.startswith("kernel_trace") or k.startswith("traffic") for k in many)
        assert "not measured in this" in many["profile_1gpu"]["note"]
