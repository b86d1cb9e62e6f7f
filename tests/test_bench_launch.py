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
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--sensors", "8", "--days", "3",
                "--cv-folds", "2", "--cv-epochs", "1"], timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 256 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    ig = out["ig"]
    assert ig["n_ranks"] == 2 and ig["value"] > 0 and ig["sharding"].startswith("round-robin")
    cv = out["cv"]                              # the headline's ROC-AUC half: every fold run exactly once
    assert cv["folds"] == 2 and cv["epochs"] == 1 and cv["fold_per_rank"] is True
    for m in ("gcn", "baseline"):
        assert cv[f"{m}_folds_run"] == [0, 1]
        assert len(cv[f"{m}_fold_auc"]) == 2 and 0.0 <= cv[f"{m}_mean_auc"] <= 1.0
    assert cv["seconds"] > 0 and cv["dtype"] == "bf16"
    assert len(cv["gcn_minus_baseline_fold_auc"]) == 2 and cv["paper_parity"].startswith("unpinned")
    assert "vs_reference_gcn_auc" not in cv
    soil = out["soilnet"]                       # the headline's second dataset: throughput + its own CV
    assert soil["global_batch"] == 64 and soil["seq_len"] == 337 and soil["value"] > 0 and soil["ms_per_step"] > 0
    scv = soil["cv"]
    assert scv["folds"] == 2 and scv["fold_per_rank"] is True and "spatial_fault_frac=0.5" in scv["data"]
    for m in ("gcn", "baseline"):
        assert scv[f"{m}_folds_run"] == [0, 1] and 0.0 <= scv[f"{m}_mean_auc"] <= 1.0
    assert scv["paper_mean_auc"] == {"gcn": 0.858, "baseline": 0.816}


def test_bench_eight_ranks_cv_and_ig_cover_every_fold_once():
    """The driver's 8-GPU form rehearsed on gloo: 8 rank processes, 5 CV folds dealt over 8 ranks (3
    ranks idle), IG batches round-robin over 8 ranks, ONE JSON line, every fold run exactly once."""
    r = _bench(["--gpus", "8", "--steps", "1", "--warmup", "0", "--sensors", "8", "--days", "3",
                "--cv-folds", "5", "--cv-epochs", "1", "--cv-days", "4", "--no-soil-line"], timeout=1500)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 1024
    assert out["ig"]["n_ranks"] == 8 and out["ig"]["value"] > 0
    cv = out["cv"]
    assert cv["folds"] == 5 and cv["fold_per_rank"] is True
    for m in ("gcn", "baseline"):
        assert cv[f"{m}_folds_run"] == [0, 1, 2, 3, 4]
        assert len(cv[f"{m}_fold_auc"]) == 5


def test_bench_parent_never_initialises_hip():
    """The spawning parent must not call torch.cuda at all (on ROCm device_count() falls back to
    hipGetDeviceCount without amdsmi, initialising HIP in a process that then forks its ranks): run
    the parent with every such entry point poisoned; the children are fresh interpreters."""
    boot = ("import sys, runpy, torch\n"
            "def boom(*a, **k):\n"
            "    raise RuntimeError('parent touched torch.cuda')\n"
            "for name in ('device_count', '_lazy_init', 'is_available', 'init', 'set_device'):\n"
            "    setattr(torch.cuda, name, boom)\n"
            "torch._C._cuda_getDeviceCount = boom\n"
            "sys.argv = [sys.argv[1]] + sys.argv[2:]\n"
            "runpy.run_path(sys.argv[0], run_name='__main__')\n")
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-c", boot, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--sensors", "8", "--days", "3", "--no-ig-line", "--no-cv-line",
                        "--no-knn-line", "--no-soil-line"], cwd=ROOT, env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2


def test_bench_world_size_mismatch_fails():
    r = _bench(["--gpus", "2", "--steps", "1"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_bench_failing_rank_fails_the_job():
    """Rank 1 fails right after joining the process group; rank 0 would wait in its first collective
    forever - the parent must stop it and exit with the failing rank's code."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--sensors", "8", "--days", "3", "--no-soil-line"],
               timeout=300,
               GNNQC_BENCH_FAIL_RANK="1")
    assert r.returncode == 3, r.stderr[-2000:]
    assert "rank 1 exited with 3" in r.stderr
