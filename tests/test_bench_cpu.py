"""bench.py launch contract on CPU (gloo): `--gpus N` without a torchrun
environment starts N ranks itself and rank 0 reports the whole job."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    res = _run(["--plumbing", "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "256"])
    assert res["n_gpus"] == 2
    assert res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 512
    assert res["steps"] == 3
    # the cohort-statistics all-reduce (dist.allreduce_sums) ran on both ranks
    chk = res["rccl_allreduce_check"]
    assert chk["ok"] and chk["world"] == 2 and chk["backend"] == "gloo"
    # value = all ranks' utterances / max-over-ranks time (rank 1 sleeps longer)
    assert abs(res["value"] - 512 * 3 / (res["ms_per_step"] * 3e-3)) / res["value"] < 0.02


def test_bench_single_rank_default():
    res = _run(["--plumbing", "--steps", "2", "--warmup", "0"])
    assert res["n_gpus"] == 1 and res["config"]["parallelism"] == "dp1"


def test_bench_world_mismatch_is_an_error():
    env = {k: v for k, v in os.environ.items()}
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--plumbing", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
