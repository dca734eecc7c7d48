#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric: CRC32C GB/s (device-resident) over
2^20 x 1400 B datagrams, bit-exact.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload fixed|csr]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

A step is one launch of the batched CRC-32C kernel over the rank's resident
shard (config 2: 2^20 x 1400 B per GPU at stride 1400; config 4 = the same per
GPU at N = 8: weak scaling, packets sharded by contiguous ranges, no
collective on the data path -- the only collectives are the timing barrier and
a MAX over per-rank times).  Inputs are generated on the device before the
timed region.  Rank 0 prints ONE JSON line.

roofline: algorithmic bytes per launch = sum(L) + 4 N (datagram bytes read +
CRC words written; CSR adds 8 N offset bytes; the xor workload reads and writes
2 sum(L)) over the average launch duration
measured with one HIP event pair around the K launches on the launch stream;
peak 8.0 TB/s (MI355X HBM3E nameplate).  traffic: HBM bytes per launch from the rocprofv3 PMC pass
(profiles/traffic_<workload>.json, FETCH_SIZE x2 gfx950 correction +
WRITE_SIZE) when present, else null.
cpu_baseline: the oracle's batch CRC (SSE4.2 crc32 instruction, OpenMP) timed
on this host's cores over a bounded sample of the same batch (rank 0, N = 1).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from litenetlibpp_amd.shard import max_over_ranks, shard_range, sum_over_ranks  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E nameplate, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "CRC32C GB/s (device-resident) over 1M×1400B packets; bit-exact"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["fixed", "csr", "filter", "xor", "dispatch"], default="fixed",
                    help="fixed: config 2 (the headline); csr: config 3; filter: the batched inbound "
                         "filter (CRC check + net_packet::verify) over the config-3 batch as wire "
                         "datagrams; xor: the XOR-encryption layer in place over the config-2 batch; "
                         "dispatch: lnl_dispatch_csr_dev over accepted MERGED containers of 256-B "
                         "messages (the config-1 traffic shape)")
    ap.add_argument("--packets", type=int, default=1 << 20, help="per GPU")
    ap.add_argument("--length", type=int, default=1400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-path", action="store_true",
                    help="also time lnl_crc32c_batch_host (PCIe-inclusive, config 5)")
    return ap.parse_args()


def make_workload(args, rank, world, device):
    """Device-resident synthetic shard (generated on the GPU, untimed): rank r
    owns datagrams shard_range(N * world, r, world) of the job's batch."""
    g = torch.Generator(device=device)
    g.manual_seed(42 + rank)
    _, n = shard_range(args.packets * world, rank, world)
    if args.workload == "xor":  # read + write every byte in place
        L = args.length
        data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=device, generator=g)
        return dict(data=data, n=n, L=L, off=None, payload=n * L, algo=2 * n * L, xor=True)
    if args.workload == "dispatch":
        return make_dispatch_workload(n, device, g)
    if args.workload == "fixed":
        L = args.length
        data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=device, generator=g)
        return dict(data=data, n=n, L=L, off=None, payload=n * L, algo=n * L + 4 * n)
    # config 3: lengths 64 + U[0, 1337), packed CSR with int64 offsets (filter: the
    # same bytes read as wire datagrams, each ending in its 4-byte CRC field)
    lens = torch.randint(64, 1401, (n,), dtype=torch.int64, device=device, generator=g)
    off = torch.zeros(n + 1, dtype=torch.int64, device=device)
    off[1:] = torch.cumsum(lens, 0)
    total = int(off[-1].item())
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=device, generator=g)
    if args.workload == "filter":  # status byte out instead of a CRC word
        return dict(data=data, n=n, L=None, off=off, payload=total, algo=total + n + 8 * (n + 1), filter=True)
    return dict(data=data, n=n, L=None, off=off, payload=total, algo=total + 4 * n + 8 * (n + 1))


XOR_KEY = b"LiteNetLibPP-bench-key"
DISPATCH_SUBS = 5          # 256-B user messages per MERGED container (config 1's payload size)
DISPATCH_SUB = 2 + 1 + 256  # [u16 LE size][UNRELIABLE header byte][256 B payload]
DISPATCH_STRIDE = 1 + DISPATCH_SUBS * DISPATCH_SUB + 4


def make_dispatch_workload(n, device, g):
    """MERGED containers as net_peer::send_merged lays them out
    (/root/reference/src/lnl/net_peer.cpp:446-486), each carrying five 257-B
    UNRELIABLE packets and ending in its CRC-32C field; filtered once
    (untimed) so every status is LNL_INBOUND_ACCEPT."""
    import litenetlibpp_amd as P
    S = DISPATCH_STRIDE
    data = torch.randint(0, 256, (n * S,), dtype=torch.uint8, device=device, generator=g)
    d = data.view(n, S)
    d[:, 0] = 0x0C
    for j in range(DISPATCH_SUBS):
        b = 1 + j * DISPATCH_SUB
        d[:, b] = (DISPATCH_SUB - 2) & 0xFF
        d[:, b + 1] = (DISPATCH_SUB - 2) >> 8
        d[:, b + 2] = 0x00
    crc = P.batch_fixed(data, S, S - 4, n)
    d[:, S - 4:] = crc.view(torch.uint8).view(n, 4)
    off = torch.arange(0, (n + 1) * S, S, dtype=torch.int64, device=device)
    status = P.inbound_filter(data, off)
    assert bool((status == 1).all()), "dispatch workload: filter rejected a container"
    k = n * DISPATCH_SUBS
    # algorithmic bytes: offset, status and container header byte per datagram;
    # u16 size + header byte read and {start, len, parent} (16 B) written per packet
    # the walk's HBM floor: every 64-B sector holding a byte it must read (header
    # byte, each entry's u16 size + header byte), once per container
    need = np.array([0] + [b for j in range(DISPATCH_SUBS) for b in range(1 + j * DISPATCH_SUB, 4 + j * DISPATCH_SUB)])
    starts = np.arange(n, dtype=np.int64)[:, None] * S
    lines = (starts + need[None, :]) // 64
    per = 1 + (np.diff(lines, axis=1) != 0).sum(axis=1)
    line_bytes = int(per.sum()) * 64 + n * (8 + 1) + k * 16
    return dict(data=data, n=n, L=None, off=off, payload=n * S, algo=n * (8 + 1 + 1) + k * (3 + 16),
                line_bytes=line_bytes,
                dispatch=True, status=status, pkts=k,
                pkt_start=torch.empty(k, dtype=torch.int64, device=device),
                pkt_len=torch.empty(k, dtype=torch.int32, device=device),
                pkt_parent=torch.empty(k, dtype=torch.int32, device=device),
                total=torch.zeros(1, dtype=torch.int32, device=device))


def launch(P, w, out, stream):
    if w.get("dispatch"):
        P._lib.check(P.lib().lnl_dispatch_csr_dev(
            w["data"].data_ptr(), w["off"].data_ptr(), w["n"], w["status"].data_ptr(),
            w["pkt_start"].data_ptr(), w["pkt_len"].data_ptr(), w["pkt_parent"].data_ptr(), w["pkts"],
            w["total"].data_ptr(), stream.cuda_stream), "lnl_dispatch_csr_dev")
    elif w.get("xor"):
        P.xor_layer_fixed(w["data"], w["L"], w["L"], w["n"], XOR_KEY, stream=stream)
    elif w.get("filter"):
        P.inbound_filter(w["data"], w["off"], out=w["status"], stream=stream)
    elif w["off"] is None:
        P.batch_fixed(w["data"], w["L"], w["L"], w["n"], out=out, stream=stream)
    else:
        P.batch_csr(w["data"], w["off"], out=out, stream=stream)


def hbm_probe_peak(data, device):
    """Measured read-only streaming rate over the same buffer (context for the
    nameplate peak)."""
    so = os.path.join(ROOT, "litenetlibpp_amd", "libhbm_probe.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    L.lnl_probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(4, dtype=torch.int32, device=device)
    s = torch.cuda.current_stream()
    nbytes = data.numel() // 16 * 16
    for _ in range(3):
        L.lnl_probe_stream_read(data.data_ptr(), nbytes, sink.data_ptr(), s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        L.lnl_probe_stream_read(data.data_ptr(), nbytes, sink.data_ptr(), s.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


def cpu_baseline(w, gpu_out):
    """Oracle batch CRC on this host over a bounded sample of the same batch;
    also checks the GPU output on that sample (bit-exact)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    n_s = min(w["n"], 1 << 17)
    if w["off"] is None:
        L = w["L"]
        sample = w["data"][: n_s * L].cpu().numpy()
        def run(th):
            return oracle.batch_fixed(sample, L, L, n_s, threads=th)
        sbytes = n_s * L
        desc = f"{n_s} x {L} B datagrams (first {sbytes / 1e6:.1f} MB of the GPU batch)"
    else:
        off = w["off"][: n_s + 1].cpu().numpy().astype(np.uint64)
        sample = w["data"][: int(off[-1])].cpu().numpy()
        def run(th):
            return oracle.batch_csr(sample, off, threads=th)
        sbytes = int(off[-1] - off[0])
        desc = f"first {n_s} mixed-length datagrams ({sbytes / 1e6:.1f} MB) of the GPU batch"
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    res = {}
    for th in (1, threads):
        best, ref = None, None
        t_end = time.perf_counter() + 5.0
        while True:
            t0 = time.perf_counter()
            ref = run(th)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
            if time.perf_counter() > t_end:
                break
        res[th] = (sbytes / best / 1e9, ref)
    exact = bool(np.array_equal(gpu_out[:n_s], res[threads][1]))
    return res, threads, desc, exact


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs (the driver never sets them): LNL_BENCH_BACKEND=gloo and
    # LNL_BENCH_ONE_GPU=1 run N ranks on one GPU to exercise the N > 1 path.
    backend = os.environ.get("LNL_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("LNL_BENCH_ONE_GPU") == "1" else local
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    red_dev = device if backend == "nccl" else None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    import litenetlibpp_amd as P
    P.lib()

    w = make_workload(args, rank, world, device)
    out = torch.empty(w["n"], dtype=torch.int32, device=device)
    if w.get("filter") and "status" not in w:
        w["status"] = torch.empty(w["n"], dtype=torch.uint8, device=device)
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        launch(P, w, out, stream)
    torch.cuda.synchronize()

    # K back-to-back launches bracketed by barrier + synchronize; one HIP event
    # pair on the launch stream gives the average launch duration (per-launch
    # event pairs would insert ~11 us of idle between launches)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier(device_ids=[gpu]) if backend == "nccl" else dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        launch(P, w, out, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier(device_ids=[gpu]) if backend == "nccl" else dist.barrier()
    wall = t1 - t0
    kern_ms = e0.elapsed_time(e1) / args.steps
    wall = max_over_ranks(wall, red_dev)          # the job takes as long as its slowest rank
    kern_ms = max_over_ranks(kern_ms, red_dev)
    ms_per_step = wall / args.steps * 1e3
    total_payload = sum_over_ranks(w["payload"], red_dev)
    value = total_payload / (ms_per_step * 1e-3) / 1e9
    achieved = w["algo"] / (kern_ms * 1e-3) / 1e9

    if rank == 0:
        traffic = None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
        if os.path.exists(tf):
            with open(tf) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        line = {
            "metric": {"fixed": METRIC,
                       "csr": "CRC32C GB/s (device-resident) over 1M mixed-length (64-1400B) packets; bit-exact",
                       "filter": "inbound filter GB/s (CRC check + verify, device-resident) over 1M mixed-length (64-1400B) datagrams",
                       "xor": "XOR-layer GB/s (device-resident, in place) over 1M x 1400B packets",
                       "dispatch": "dispatch GB/s (MERGED containers cut on device) over 1M x 1300B datagrams"}[args.workload],
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint on device, seed 42+rank), resident in HBM before timing",
            "config": {
                "workload": {"fixed": "config2: 2^20 x 1400 B datagrams per GPU, fixed stride 1400, device-resident",
                             "csr": "config3: 2^20 mixed-length datagrams (64..1400 B uniform) per GPU, CSR int64 offsets",
                             "filter": "config-3 batch as wire datagrams through lnl_inbound_filter_csr_dev",
                             "xor": "XOR layer over the config-2 batch, in place (22-byte key)",
                             "dispatch": "2^20 accepted MERGED containers x 5 UNRELIABLE 256-B messages (1300 B wire), lnl_dispatch_csr_dev"}[args.workload],
                "packets_per_gpu": w["n"],
                "payload_bytes_per_gpu": w["payload"],
                "parallelism": f"shard{world} (contiguous packet ranges, no data-path collectives)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": w["algo"],
                "kernel_ms": round(kern_ms, 5),
            },
        }
        if "line_bytes" in w:  # random narrow reads: HBM moves whole 64-B sectors
            lb = w["line_bytes"] / (kern_ms * 1e-3) / 1e9
            line["roofline"]["sector_granular_bytes_per_launch"] = w["line_bytes"]
            line["roofline"]["sector_granular_achieved"] = round(lb, 1)
            line["roofline"]["sector_granular_frac"] = round(lb / HBM_PEAK_GBS, 4)
        probe = hbm_probe_peak(w["data"], device)
        if probe:
            line["roofline"]["measured_stream_read_peak_gbs"] = round(probe, 1)
        if world == 1 and not args.no_cpu_baseline and not (w.get("xor") or w.get("filter") or w.get("dispatch")):
            gpu_out = out.cpu().numpy().view(np.uint32)
            res, threads, desc, exact = cpu_baseline(w, gpu_out)
            line["cpu_baseline"] = {
                "value": round(res[threads][0], 3),
                "unit": "GB/s",
                "cores": threads,
                "kind": "port",
                "sample": desc + f"; oracle SSE4.2 crc32 loop, OpenMP {threads} threads, best of repeats over ~5 s",
                "single_core_value": round(res[1][0], 3),
            }
            line["parity_on_sample"] = "bit-exact" if exact else "MISMATCH"
        if args.host_path and world == 1:
            line["host_path"] = host_path_rate(P, w)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_path_rate(P, w):
    """Config 5: host-resident pinned batch -> lnl_crc32c_batch_host (H2D +
    kernel + D2H over 2 streams).  PCIe-inclusive; never the headline value."""
    if w["off"] is None:
        n, L = w["n"], w["L"]
        host = w["data"].cpu().pin_memory()
        off = np.arange(0, (n + 1) * L, L, dtype=np.uint64)
    else:
        host = w["data"].cpu().pin_memory()
        off = w["off"].cpu().numpy().astype(np.uint64)
    arr = host.numpy()
    P.batch_host(arr, off, torch.cuda.current_device())
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        P.batch_host(arr, off, torch.cuda.current_device())
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(w["payload"] / dt / 1e9, 2), "unit": "GB/s",
            "what": "pinned host batch, lnl_crc32c_batch_host, H2D+kernel+D2H, 2 streams"}


if __name__ == "__main__":
    main()
