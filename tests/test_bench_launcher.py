"""bench.py's multi-rank launcher: ``python bench.py --gpus N`` must run N
ranks and report n_gpus = N, never silently one.  CPU only: the --dry-run mode goes through the
same launch (torch.distributed.run child), rendezvous (gloo), barrier and max-over-ranks timing as
the GPU run, around a CPU stand-in step."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                             "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=240)


def _line(out):
    return json.loads([ln for ln in out.strip().splitlines() if ln.startswith("{")][-1])


def test_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["dry_run"] and d["ranks_launched_by_bench"]
    assert d["steps"] == 3 and d["value"] > 0


def test_gpus1_runs_in_process():
    r = _run(["--gpus", "1", "--dry-run", "--steps", "2", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and not d["ranks_launched_by_bench"]


def test_world_size_must_agree_with_gpus():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "disagrees with WORLD_SIZE" in r.stderr


def test_too_few_gpus_refused():
    # this container has no GPU: a real (non dry-run) --gpus 2 must refuse before launching anything
    r = _run(["--gpus", "2"])
    assert r.returncode != 0 and "GPU(s) visible" in r.stderr
