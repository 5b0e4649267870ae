"""bench.py's multi-GPU entry point (the driver's `python bench.py --gpus N`): without a launcher in
the environment it starts the N ranks itself (torch.distributed.run on 127.0.0.1) and rank 0 reports
the world they formed; a launcher that started a different number of ranks is refused.  Rehearsed
on the CPU with --dry-run (gloo all_reduce of a flat gradient of the model's size)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                               "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_gpus_n_starts_n_ranks():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "2",
                        "--warmup", "1"], cwd=REPO, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["allreduce_ok"] is True        # mean of ranks 1 and 2 everywhere
    # the reference model has 3,307,270 parameters; base.output_heads (514) is unused by the Hetero forward
    # (train.py:579-586) and has no slot in the flat gradient
    assert out["config"]["grad_elems"] == 3307270 - 514
    assert out["value"] > 0 and out["steps"] == 2


def test_world_size_mismatch_is_refused():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"], cwd=REPO,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_launcher_counts_gpus_without_touching_hip():
    """The self-launch path counts devices in a child interpreter: the launching process itself never
    initialises HIP (a process that did must not start another program on this pool)."""
    code = ("import sys; sys.argv = ['bench.py']; sys.path.insert(0, %r); import bench, torch; "
            "n = bench._visible_gpus(); print(n, torch.cuda.is_initialized())" % REPO)
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    n, init = r.stdout.split()[-2:]
    assert init == "False"
    import torch
    assert int(n) == (torch.cuda.device_count() if torch.cuda.is_available() else 0)
