"""bench.py's multi-rank entry point on the CPU: `--gpus 2` without a launcher
spawns two ranks itself (the path the driver's N-GPU runs and the 1/2/4/8
curve go through), and a launcher whose WORLD_SIZE differs from --gpus is
refused.  LNL_BENCH_DRYRUN=1 runs the plumbing (spawn, gloo barrier, MIN/MAX/
SUM and the per-rank gather) with no kernel, since this container has no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=240):
    env = dict(os.environ, LNL_BENCH_DRYRUN="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    if extra_env:
        env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--packets", "1000"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["steps"] == 3 and line["warmup"] == 1
    assert len(line["roofline"]["kernel_ms_per_rank"]) == 2
    assert line["config"]["payload_bytes_per_gpu"] == 1000 * 1400
    assert line["config"]["parallelism"].startswith("shard2")
    assert "dry_run" in line


def test_gpus_8_names_config4():
    r = _run(["--gpus", "8", "--steps", "2", "--warmup", "0", "--packets", "64"])
    assert r.returncode == 0, r.stderr
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert line["n_gpus"] == 8
    assert line["config"]["workload"].startswith("config4")


def test_dead_rank_ends_the_run():
    """A rank that dies before rendezvous: the spawner stops its siblings (which
    would wait for it forever) and returns the dead rank's status."""
    import time
    t0 = time.time()
    r = _run(["--gpus", "4", "--steps", "2", "--warmup", "0", "--packets", "64"],
             extra_env={"LNL_BENCH_DRYRUN_FAIL_RANK": "2"}, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "rank 2 exited with status 3" in r.stderr
    assert time.time() - t0 < 90


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "2", "--steps", "1"], extra_env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_every_workload_names_its_metric():
    """Each --workload prints one line with its own metric and workload name
    (dry run: the plumbing, no kernel)."""
    seen = set()
    for wl in ("fixed", "csr", "filter", "xor", "xor_csr", "dispatch", "append", "filter_dispatch",
               "filter_then_dispatch"):
        r = _run(["--workload", wl, "--steps", "1", "--warmup", "0", "--packets", "64"])
        assert r.returncode == 0, (wl, r.stderr)
        line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert line["n_gpus"] == 1 and line["unit"] == "GB/s" and line["higher_is_better"]
        seen.add((line["metric"], line["config"]["workload"]))
    assert len(seen) == 9


def test_force_dist_at_one_rank():
    """--force-dist at --gpus 1 initialises the process group and runs every
    collective of the N-rank path (here gloo, dry run; RCCL on the GPU box:
    tests/test_gpu_config4.py), then tears it down."""
    r = _run(["--gpus", "1", "--force-dist", "--steps", "2", "--warmup", "0", "--packets", "64"])
    assert r.returncode == 0, r.stderr
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert line["n_gpus"] == 1
    assert line["distributed"]["forced"] is True and line["distributed"]["world_size"] == 1
    r = _run(["--gpus", "1", "--steps", "2", "--warmup", "0", "--packets", "64"])
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert line["distributed"] is None
