"""bench.py as the driver runs it: ``python bench.py --gpus N`` without a launcher spawns the N rank
processes itself (gloo on the CPU here), rank 0 prints ONE JSON line for the whole job, and a
launcher whose WORLD_SIZE disagrees with --gpus, or a failing rank, makes the command fail."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=600, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=e,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)


def test_bench_spawns_ranks_and_reports_dp_line():
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--sensors", "8", "--days", "3"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 256 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    ig = out["ig"]
    assert ig["n_ranks"] == 2 and ig["value"] > 0 and ig["sharding"].startswith("round-robin")


def test_bench_world_size_mismatch_fails():
    r = _bench(["--gpus", "2", "--steps", "1"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_bench_failing_rank_fails_the_job():
    """Rank 1 fails right after joining the process group; rank 0 would wait in its first collective
    forever - the parent must stop it and exit with the failing rank's code."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--sensors", "8", "--days", "3"], timeout=300,
               GNNQC_BENCH_FAIL_RANK="1")
    assert r.returncode == 3, r.stderr[-2000:]
    assert "rank 1 exited with 3" in r.stderr
