"""Config 4 (BASELINE.json configs[3]: 8 x 2^20 x 1400 B, one shard per GPU, no
collectives) through the HIP path at its full size, on the box's one GPU.

bench.py --gpus 8 spawns eight fresh ranks before any GPU call; each owns a
contiguous 2^20-datagram shard (shard_range), generates it in HBM, runs the
lane-run kernel on it, and compares its first datagrams with the oracle.
LNL_BENCH_BACKEND=gloo + LNL_BENCH_ONE_GPU=1 put all eight ranks on GPU 0
(the driver's 8-GPU run uses RCCL and one GPU per rank, through the same
spawn / shard / gather / aggregate code).  8 x 1.47 GB = 11.7 GB of HBM.
"""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config4_eight_shards_full_size():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, LNL_BENCH_BACKEND="gloo", LNL_BENCH_ONE_GPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LNL_BENCH_DRYRUN"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3",
                        "--warmup", "1", "--no-host-path", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 8
    assert line["config"]["workload"].startswith("config4")
    assert line["config"]["packets_per_gpu"] == 1 << 20
    assert line["config"]["payload_bytes_per_gpu"] == (1 << 20) * 1400
    assert line["parity_on_sample"].startswith("bit-exact"), line["parity_on_sample"]
    assert "of 8 rank(s)" in line["parity_on_sample"]
    assert len(line["roofline"]["kernel_ms_per_rank"]) == 8
    assert all(k > 0 for k in line["roofline"]["kernel_ms_per_rank"])
    assert line["value"] > 0


def test_bench_rccl_branch_on_one_gpu():
    """bench.py --gpus 1 --force-dist: the RCCL branch the driver's multi-GPU
    run takes -- init_process_group("nccl", device_id=...), barrier with
    device_ids, MAX / SUM / all_gather on device tensors, destroy_process_group
    -- in a fresh process on the box's one GPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LNL_BENCH_DRYRUN", "LNL_BENCH_BACKEND", "LNL_BENCH_ONE_GPU",
              "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-dist",
                        "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--no-host-path", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    d = line["distributed"]
    assert d["backend"] == "nccl" and d["world_size"] == 1 and d["forced"] is True
    assert "device tensors" in d["collectives"]
    assert line["n_gpus"] == 1 and line["parity_on_sample"].startswith("bit-exact")
    assert line["value"] > 0 and len(line["roofline"]["kernel_ms_per_rank"]) == 1
