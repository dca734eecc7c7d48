#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric: CRC32C GB/s (device-resident) over
2^20 x 1400 B datagrams, bit-exact.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload fixed|csr|...]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

With --gpus N > 1 and no launcher (WORLD_SIZE unset), this process starts N
child processes itself -- one per GPU, RANK / LOCAL_RANK / WORLD_SIZE set --
before anything touches the GPU, and exits with the worst child's status.
Under a launcher, WORLD_SIZE must equal --gpus.

A step is one launch of the batched CRC-32C kernel over the rank's resident
shard (config 2: 2^20 x 1400 B per GPU at stride 1400; config 4 = the same per
GPU at N = 8: weak scaling, packets sharded by contiguous ranges, no
collective on the data path -- the only collectives are the timing barrier,
MIN/MAX/SUM over per-rank times and bytes, and a gather of per-rank figures).
Inputs are generated on the device before the timed region.  `value` = the
bytes all ranks checksummed / (last rank's finish - first rank's start), on
the host wall clock, bracketed by a barrier + synchronize on both sides.
Rank 0 prints ONE JSON line.

roofline: algorithmic bytes per launch = sum(L) + 4 N (datagram bytes read +
CRC words written; CSR adds 8 N offset bytes; the xor workload reads and writes
2 sum(L)) over the average launch duration measured with one HIP event pair
around the K launches on the launch stream; peak 8.0 TB/s (MI355X HBM3E
nameplate).  traffic: HBM bytes per launch from the builder's rocprofv3 PMC
passes (profiles/traffic_<workload>.json; FETCH_SIZE x its access shape's
factor -- x2 for wide streaming reads, x1 for the dispatch walk's random
sectors, calibrated in profiles/fetch_calibration.json -- + WRITE_SIZE),
labelled as such -- it is not measured inside this run.
cpu_baseline: the oracle's batch CRC (SSE4.2 crc32 instruction, OpenMP) timed
on this host over the WHOLE batch (copied to host memory, untimed), on one
core and on every core this process may run on (rank 0, N = 1); the checker
also compares the GPU's output for the whole batch with it.
host_path: config 5 -- the same batch from pinned host memory through
lnl_crc32c_batch_host_ex (H2D + kernel + D2H on 2 HIP streams, BASELINE
configs[4]; the 4-stream default beside it), PCIe-inclusive.
"""
from __future__ import annotations

import argparse
import ctypes
import datetime
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from litenetlibpp_amd.shard import gather_over_ranks, max_over_ranks, shard_range, sum_over_ranks  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E nameplate, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "CRC32C GB/s (device-resident) over 1M×1400B packets; bit-exact"
DRY = os.environ.get("LNL_BENCH_DRYRUN") == "1"  # CPU plumbing test: no kernels, no device


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed: run the step for this long before the warmup steps, so that the timed "
                         "steps see the GPU's sustained clocks (compute-heavy steps run ~3 %% (config 2) to "
                         "~15 %% (config 3) slower in the first milliseconds after idle; DESIGN 5); reported "
                         "in the line as settle_ms / settle_steps")
    ap.add_argument("--workload", choices=["fixed", "csr", "filter", "xor", "xor_csr", "dispatch", "append",
                                           "filter_dispatch", "filter_then_dispatch"], default="fixed",
                    help="fixed: config 2 (the headline; config 4 at N = 8); csr: config 3; filter: the "
                         "batched inbound filter (CRC check + net_packet::verify) over the config-3 batch as "
                         "wire datagrams; xor: the XOR-encryption layer in place over the config-2 batch "
                         "(xor_csr: over the config-3 batch); "
                         "dispatch: lnl_dispatch_csr_dev over accepted MERGED containers of 256-B "
                         "messages (the config-1 traffic shape); filter_dispatch: the same containers as wire "
                         "datagrams through lnl_inbound_filter_dispatch_csr_dev (one pass: the walk in the "
                         "filter's span kernel); filter_then_dispatch: the two calls, for comparison")
    ap.add_argument("--packets", type=int, default=1 << 20, help="per GPU")
    ap.add_argument("--length", type=int, default=1400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the config-5 (PCIe-inclusive) measurement")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed (backend nccl = RCCL on the GPU box) even at --gpus 1 and "
                         "run every collective the N-rank path runs (barrier with device_ids, MAX / SUM / gather "
                         "on device tensors, destroy_process_group): a one-GPU rehearsal of the driver's "
                         "multi-GPU run (DESIGN 6)")
    return ap.parse_args()


# ------------------------------------------------------------------ launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """One child process per GPU, started before this process makes any GPU
    call (children are fresh interpreters, never an exec of this one).  Every
    child is polled: the first one to exit non-zero ends the run -- its
    siblings (which would otherwise wait in rendezvous or a barrier forever)
    are terminated, then killed -- and its status is returned."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                for q in live:
                    q.terminate()
                t_end = time.time() + 10.0
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, t_end - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                sys.stderr.write(f"bench.py: rank {procs.index(p)} exited with status {c}; "
                                 f"stopped the other {len(live)} rank(s)\n")
                return c
        time.sleep(0.05)
    return 0


# ------------------------------------------------------------------ workloads
def make_workload(args, rank, world, device):
    """Device-resident synthetic shard (generated on the GPU, untimed): rank r
    owns datagrams shard_range(N * world, r, world) of the job's batch."""
    _, n = shard_range(args.packets * world, rank, world)
    if DRY:  # plumbing only: nothing is launched
        return dict(data=None, n=n, L=args.length, off=None, payload=n * args.length,
                    algo=n * (args.length + 4))
    g = torch.Generator(device=device)
    g.manual_seed(42 + rank)
    if args.workload == "xor":  # read + write every byte in place
        L = args.length
        data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=device, generator=g)
        return dict(data=data, n=n, L=L, off=None, payload=n * L, algo=2 * n * L, xor=True)
    if args.workload in ("dispatch", "filter_dispatch", "filter_then_dispatch"):
        w = make_dispatch_workload(n, device, g)
        if args.workload != "dispatch":  # statuses written by the timed call; every byte read
            w.update(dispatch=False, fused=args.workload == "filter_dispatch", filter_dispatch=True,
                     status=torch.empty(n, dtype=torch.uint8, device=device),
                     algo=w["payload"] + 8 * (n + 1) + n + w["pkts"] * 16)
            w.pop("line_bytes")
        return w
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
    if args.workload == "xor_csr":  # read + write every byte in place, per-datagram key phase
        return dict(data=data, n=n, L=None, off=off, payload=total, algo=2 * total + 8 * (n + 1), xor=True)
    if args.workload == "filter":  # status byte out instead of a CRC word
        return dict(data=data, n=n, L=None, off=off, payload=total, algo=total + n + 8 * (n + 1), filter=True)
    if args.workload == "append":  # the outbound layer: payload || LE32(crc) per datagram into a wire burst
        wire = torch.empty(total + 4 * n, dtype=torch.uint8, device=device)
        return dict(data=data, n=n, L=None, off=off, payload=total, wire=wire, append=True,
                    algo=total + (total + 4 * n) + 4 * n + 8 * (n + 1))
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
    if DRY:
        return
    if w.get("filter_dispatch"):
        if w["fused"]:
            P._lib.check(P.lib().lnl_inbound_filter_dispatch_csr_dev(
                w["data"].data_ptr(), w["off"].data_ptr(), w["n"], w["status"].data_ptr(),
                w["pkt_start"].data_ptr(), w["pkt_len"].data_ptr(), w["pkt_parent"].data_ptr(), w["pkts"],
                w["total"].data_ptr(), stream.cuda_stream), "lnl_inbound_filter_dispatch_csr_dev")
        else:
            P.inbound_filter(w["data"], w["off"], out=w["status"], stream=stream)
            P._lib.check(P.lib().lnl_dispatch_csr_dev(
                w["data"].data_ptr(), w["off"].data_ptr(), w["n"], w["status"].data_ptr(),
                w["pkt_start"].data_ptr(), w["pkt_len"].data_ptr(), w["pkt_parent"].data_ptr(), w["pkts"],
                w["total"].data_ptr(), stream.cuda_stream), "lnl_dispatch_csr_dev")
    elif w.get("dispatch"):
        P._lib.check(P.lib().lnl_dispatch_csr_dev(
            w["data"].data_ptr(), w["off"].data_ptr(), w["n"], w["status"].data_ptr(),
            w["pkt_start"].data_ptr(), w["pkt_len"].data_ptr(), w["pkt_parent"].data_ptr(), w["pkts"],
            w["total"].data_ptr(), stream.cuda_stream), "lnl_dispatch_csr_dev")
    elif w.get("xor") and w["off"] is not None:
        P.xor_layer_csr(w["data"], w["off"], XOR_KEY, stream=stream)
    elif w.get("xor"):
        P.xor_layer_fixed(w["data"], w["L"], w["L"], w["n"], XOR_KEY, stream=stream)
    elif w.get("filter"):
        P.inbound_filter(w["data"], w["off"], out=w["status"], stream=stream)
    elif w.get("append"):  # CRCs into out (checked like csr), wire bytes into w["wire"]
        P._lib.check(P.lib().lnl_crc32c_append_csr_dev(
            w["data"].data_ptr(), w["off"].data_ptr(), w["n"], w["wire"].data_ptr(), out.data_ptr(),
            stream.cuda_stream), "lnl_crc32c_append_csr_dev")
    elif w["off"] is None:
        P.batch_fixed(w["data"], w["L"], w["L"], w["n"], out=out, stream=stream)
    else:
        P.batch_csr(w["data"], w["off"], out=out, stream=stream)


# ------------------------------------------------------------------ context figures
def hbm_probe_peak(data, device):
    """Measured read-only streaming rates over the same buffer (context for
    the nameplate peak; litenetlibpp_amd/csrc/hbm_probe.hip): forms 0 / 1 are
    plain streams (global_load_dwordx4 nt, LDS-DMA nt) over the whole buffer;
    forms 2-4 read it in the shape of a segment-per-lane CSR kernel (48-line
    segments, one round of every resident wave: per-lane lines into VGPRs with
    the default / nt policy, and by LDS-DMA); forms 11-13 are plain streams on
    one-shot grids handed out in buffer order."""
    so = os.path.join(ROOT, "litenetlibpp_amd", "libhbm_probe.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    L.lnl_probe_stream_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int]
    L.lnl_probe_stream_read.restype = ctypes.c_int
    sink = torch.zeros(4, dtype=torch.int32, device=device)
    s = torch.cuda.current_stream()
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    seg_round = cus * 8 * 64 * 48 * 128
    best = {}
    waves = {5: 5, 6: 6}
    for form in (0, 1, 2, 3, 4, 5, 6, 7, 11, 12, 13):
        nbytes = data.numel() // 8192 * 8192 if form < 2 or form > 10 else seg_round * waves.get(form, 8) // 8
        if nbytes > data.numel() or nbytes == 0:
            continue
        rc = 0
        for _ in range(3):
            rc = rc or L.lnl_probe_stream_read(data.data_ptr(), nbytes, sink.data_ptr(), s.cuda_stream, form)
        if rc != 0:  # a form the probe rejects: no figure rather than an empty event pair's
            continue
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            L.lnl_probe_stream_read(data.data_ptr(), nbytes, sink.data_ptr(), s.cuda_stream, form)
        e1.record()
        torch.cuda.synchronize()
        best[form] = nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    return best


def hbm_probe_sectors(data, device, n=1 << 22):
    """Measured rate of independent one-dword reads at n distinct random 64-B
    sectors of the same buffer (hbm_probe.hip sector_read): the ceiling of a
    walk that touches one sector per dependent read, in 64-B sectors' GB/s."""
    so = os.path.join(ROOT, "litenetlibpp_amd", "libhbm_probe.so")
    if not os.path.exists(so):
        return None
    L = ctypes.CDLL(so)
    L.lnl_probe_sector_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_void_p, ctypes.c_void_p]
    L.lnl_probe_sector_read.restype = ctypes.c_int64
    sink = torch.zeros(4, dtype=torch.int32, device=device)
    s = torch.cuda.current_stream()
    for _ in range(3):
        if L.lnl_probe_sector_read(data.data_ptr(), data.numel(), n, 1, sink.data_ptr(), s.cuda_stream) <= 0:
            return None
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        L.lnl_probe_sector_read(data.data_ptr(), data.numel(), n, 1, sink.data_ptr(), s.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    return 64.0 * n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9


def cpu_quota() -> int | None:
    """CPUs the cgroup grants this process (cpu.max quota / period), if capped.
    On the GPU box os.cpu_count() and the affinity mask show the whole machine
    while the job's share is a quota; threads beyond it only time-slice."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, p = f.read().split()[:2]
            if q != "max":
                return max(1, int(int(q) // int(p)))
        except (OSError, ValueError):
            pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        if q > 0:
            return max(1, q // p)
    except (OSError, ValueError):
        pass
    return None


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_copy(w):
    """The rank's batch in host memory (untimed): (bytes, offsets or None)."""
    data = w["data"].cpu().numpy()
    off = None if w["off"] is None else w["off"].cpu().numpy().astype(np.uint64)
    return data, off


def cpu_baseline(w, host):
    """Checker + CPU baseline: the oracle's batch CRC over the WHOLE batch on
    1 core and on every core this process may run on; median of repeats over
    ~2 s per thread count.  Returns (figures, oracle output)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    data, off = host
    if off is None:
        L, n = w["L"], w["n"]
        def run(th):
            return oracle.batch_fixed(data, L, L, n, threads=th)
    else:
        def run(th):
            return oracle.batch_csr(data, off, threads=th)
    cores = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    if quota:
        cores = min(cores, quota)
    res, ref = {}, None
    nproc = os.cpu_count() or cores
    # 1 core, the job's share, and -- for the record -- one thread per CPU the
    # machine reports (beyond the share they only time-slice)
    for th in sorted({1, cores, nproc}):
        times = []
        t_end = time.perf_counter() + 2.0
        while True:
            t0 = time.perf_counter()
            ref = run(th)
            times.append(time.perf_counter() - t0)
            if time.perf_counter() > t_end and len(times) >= 3:
                break
        res[th] = w["payload"] / float(np.median(times)) / 1e9
    return res, cores, ref, quota


def parity_sample(w, out, host):
    """Checker: the rank's GPU output vs the oracle on its first datagrams."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    data, off = host
    k = min(w["n"], 1 << 14)
    got = out[:k].cpu().numpy().view(np.uint32)
    if off is None:
        exp = oracle.batch_fixed(data, w["L"], w["L"], k)
    else:
        exp = oracle.batch_csr(data, off[: k + 1])
    ok = bool(np.array_equal(got, exp))
    if ok and w.get("append"):  # the wire bytes of the same datagrams: payload || LE32(crc)
        o = off[: k + 1].astype(np.int64)
        lens = np.diff(o)
        wire = w["wire"][: int(o[k] - o[0]) + 4 * k].cpu().numpy()
        crcpos = (o[1:] - o[0]) + 4 * np.arange(1, k + 1) - 4
        keep = np.ones(wire.size, dtype=bool)
        for j in range(4):
            keep[crcpos + j] = False
        ok = (np.array_equal(wire[keep], data[o[0]:o[k]]) and
              np.array_equal(wire[crcpos[:, None] + np.arange(4)[None, :]].reshape(-1),
                             exp.astype("<u4").view(np.uint8)) and lens.size == k)
    return ok, k


def _host_timed(fn, reps=3):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        got = fn()
    return (time.perf_counter() - t0) / reps, got


def host_path_rate(P, host, w, device):
    """Config 5: host-resident pinned batch -> lnl_crc32c_batch_host_ex on 2
    HIP streams (BASELINE.json configs[4]), H2D + kernel + D2H, chunks of 64 Ki
    datagrams; the library's default (4 streams) beside it.  PCIe-inclusive;
    never the headline value."""
    data, off = host
    if off is None:
        off = np.arange(0, (w["n"] + 1) * w["L"], w["L"], dtype=np.uint64)
    pinned = torch.from_numpy(data).pin_memory().numpy()
    reps = 3
    dt2, got = _host_timed(lambda: P.batch_host(pinned, off, device, streams=2), reps)
    dt4, got4 = _host_timed(lambda: P.batch_host(pinned, off, device, streams=4), reps)
    return {"value": round(w["payload"] / dt2 / 1e9, 2), "unit": "GB/s", "streams": 2,
            "value_4_streams": round(w["payload"] / dt4 / 1e9, 2),
            "what": "config 5: the same batch in pinned host memory through lnl_crc32c_batch_host_ex "
                    "(H2D + kernel + D2H overlapped on 2 HIP streams, chunks of <= 64 Ki datagrams / 64 MiB), "
                    f"blocking, mean of {reps} calls; value_4_streams: the library default, 4 streams",
            "parity_4_streams": "equal to the 2-stream output" if np.array_equal(got, got4) else "MISMATCH"}, got


def host_append_rate(P, host, w, device):
    """The send side from host memory: the same payload burst, pinned, through
    lnl_crc32c_append_host_ex (H2D + CRC + append + D2H of the wire burst) on
    2 HIP streams (config 5's count) and on 4 (the library default: the D2H of
    a chunk no longer holds up its stream's next H2D), PCIe-inclusive; the
    wire bytes of the first datagrams checked against the device-resident
    call's."""
    data, off = host
    pinned = torch.from_numpy(data).pin_memory().numpy()
    out = torch.empty(int(off[-1] - off[0]) + 4 * w["n"], dtype=torch.uint8).pin_memory().numpy()
    reps = 3
    dt2, (wire, woff) = _host_timed(lambda: P.append_host(pinned, off, device, out=out, streams=2), reps)
    k = min(w["n"], 1 << 14)
    ok = np.array_equal(wire[: int(woff[k])], w["wire"][: int(woff[k])].cpu().numpy())
    dt4, (wire4, _) = _host_timed(lambda: P.append_host(pinned, off, device, out=out, streams=4), reps)
    ok = ok and np.array_equal(wire4[: int(woff[k])], w["wire"][: int(woff[k])].cpu().numpy())
    return {"value": round(w["payload"] / dt2 / 1e9, 2), "unit": "GB/s", "streams": 2,
            "value_4_streams": round(w["payload"] / dt4 / 1e9, 2),
            "what": "the payload burst in pinned host memory through lnl_crc32c_append_host_ex (H2D payload + "
                    "offsets, CRC + append, D2H of the wire burst into pinned memory) on 2 HIP streams, "
                    f"blocking, payload bytes / time, mean of {reps} calls; value_4_streams: 4 streams",
            "parity": "wire bytes equal the device-resident call's" if ok else "MISMATCH"}


# ------------------------------------------------------------------ main
def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(env_world or "1")
    if env_world is not None and world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch one rank per GPU "
                 f"(torchrun --nproc-per-node {args.gpus}) or drop the launcher and let --gpus spawn them")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if DRY and os.environ.get("LNL_BENCH_DRYRUN_FAIL_RANK") == str(rank):
        sys.exit(3)  # dry-run test knob: a rank that dies before rendezvous (spawn_ranks must not hang)
    # Rehearsal knobs (the driver never sets them): LNL_BENCH_BACKEND=gloo and
    # LNL_BENCH_ONE_GPU=1 run N ranks on one GPU to exercise the N > 1 path.
    backend = "gloo" if DRY else os.environ.get("LNL_BENCH_BACKEND", "nccl")
    gpu = 0 if os.environ.get("LNL_BENCH_ONE_GPU") == "1" else local
    if DRY:
        device = torch.device("cpu")
    else:
        torch.cuda.set_device(gpu)
        device = torch.device("cuda", gpu)
    red_dev = device if backend == "nccl" else None
    dist_on = world > 1 or args.force_dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        # bounded rendezvous: a rank that never arrives ends the run, not hangs it
        tmo = datetime.timedelta(seconds=300)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device, timeout=tmo)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=tmo)
    import litenetlibpp_amd as P
    if not DRY:
        P.lib()

    def barrier():
        if dist_on:
            dist.barrier(device_ids=[gpu]) if backend == "nccl" else dist.barrier()

    def sync():
        if not DRY:
            torch.cuda.synchronize()

    w = make_workload(args, rank, world, device)
    out = None if DRY else torch.empty(w["n"], dtype=torch.int32, device=device)
    if w.get("filter") and "status" not in w:
        w["status"] = torch.empty(w["n"], dtype=torch.uint8, device=device)
    stream = None if DRY else torch.cuda.current_stream()
    # settle (untimed): the GPU ramps its clocks up under sustained load; the
    # K timed steps below are exactly K steps of the workload either way
    settle_steps = 0
    if args.settle_ms > 0 and not DRY:
        sync()
        t_settle = time.perf_counter() + args.settle_ms * 1e-3
        while time.perf_counter() < t_settle:
            for _ in range(8):
                launch(P, w, out, stream)
            settle_steps += 8
            sync()
    for _ in range(args.warmup):
        launch(P, w, out, stream)
    sync()

    # K back-to-back launches bracketed by barrier + synchronize; one HIP event
    # pair on the launch stream gives the average launch duration (per-launch
    # event pairs would insert ~11 us of idle between launches)
    if not DRY:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    sync()
    t0 = time.time()
    if not DRY:
        e0.record(stream)
    for _ in range(args.steps):
        launch(P, w, out, stream)
    if not DRY:
        e1.record(stream)
    sync()
    t1 = time.time()
    barrier()
    kern_ms = e0.elapsed_time(e1) / args.steps if not DRY else (t1 - t0) * 1e3 / max(args.steps, 1)
    start = -max_over_ranks(-t0, red_dev)   # the first rank's start
    end = max_over_ranks(t1, red_dev)       # the last rank's finish
    ms_per_step = (end - start) / args.steps * 1e3
    total_payload = sum_over_ranks(w["payload"], red_dev)
    value = total_payload * args.steps / ((end - start) or 1e-9) / 1e9
    kern_all = gather_over_ranks(kern_ms, red_dev)
    kern_max = max(kern_all)
    achieved = w["algo"] / (kern_max * 1e-3) / 1e9

    # checker, outside the timed region: every rank compares its first
    # datagrams with the oracle (rank 0 at N = 1: the whole batch, below)
    crc_workload = not DRY and not (w.get("xor") or w.get("filter") or w.get("dispatch") or w.get("filter_dispatch"))
    host = host_copy(w) if crc_workload else None
    ok_sample = 1.0
    if crc_workload:
        ok, _k = parity_sample(w, out, host)
        ok_sample = 1.0 if ok else 0.0
    if not DRY and w.get("filter_dispatch"):  # every container accepted and cut into its 5 packets
        n, S = w["n"], DISPATCH_STRIDE
        i = torch.arange(n, dtype=torch.int64, device=device)
        j = torch.arange(DISPATCH_SUBS, dtype=torch.int64, device=device)
        exp_start = (i[:, None] * S + 1 + j[None, :] * DISPATCH_SUB + 2).reshape(-1)
        ok = (bool((w["status"] == 1).all()) and int(w["total"].item()) == w["pkts"]
              and torch.equal(w["pkt_start"], exp_start)
              and bool((w["pkt_len"] == DISPATCH_SUB - 2).all())
              and torch.equal(w["pkt_parent"].to(torch.int64), i.repeat_interleave(DISPATCH_SUBS)))
        ok_sample = 1.0 if ok else 0.0
    ok_all = gather_over_ranks(ok_sample, red_dev)

    if rank == 0:
        traffic, traffic_src = None, None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
        if os.path.exists(tf):
            with open(tf) as f:
                tj = json.load(f)
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_src = (f"profiles/traffic_{args.workload}.json: builder's rocprofv3 PMC passes "
                           f"({tj.get('source', 'see file')}), not measured in this run")
        workload_name = {
            "fixed": ("config4: " if world == 8 else "config2: ") +
                     "2^20 x 1400 B datagrams per GPU, fixed stride 1400, device-resident" +
                     (" (8M x 1400 B over 8 GPUs)" if world == 8 else ""),
            "csr": "config3: 2^20 mixed-length datagrams (64..1400 B uniform) per GPU, CSR int64 offsets",
            "filter": "config-3 batch as wire datagrams through lnl_inbound_filter_csr_dev",
            "xor": "XOR layer over the config-2 batch, in place (22-byte key)",
            "xor_csr": "XOR layer over the config-3 batch (CSR, 64..1400 B), in place (22-byte key)",
            "dispatch": "2^20 accepted MERGED containers x 5 UNRELIABLE 256-B messages (1300 B wire), "
                        "lnl_dispatch_csr_dev",
            "filter_dispatch": "2^20 MERGED containers x 5 UNRELIABLE 256-B messages (1300 B wire) through "
                               "lnl_inbound_filter_dispatch_csr_dev (filter + cut in one pass)",
            "filter_then_dispatch": "2^20 MERGED containers x 5 UNRELIABLE 256-B messages (1300 B wire): "
                                    "lnl_inbound_filter_csr_dev, then lnl_dispatch_csr_dev",
            "append": "config-3 batch through lnl_crc32c_append_csr_dev (outbound layer: wire burst of "
                      "payload || LE32(crc))"}[args.workload]
        line = {
            "metric": {"fixed": METRIC,
                       "csr": "CRC32C GB/s (device-resident) over 1M mixed-length (64-1400B) packets; bit-exact",
                       "filter": "inbound filter GB/s (CRC check + verify, device-resident) over 1M mixed-length (64-1400B) datagrams",
                       "xor": "XOR-layer GB/s (device-resident, in place) over 1M x 1400B packets",
                       "xor_csr": "XOR-layer GB/s (device-resident, in place) over 1M mixed-length (64-1400B) packets",
                       "dispatch": "dispatch GB/s (MERGED containers cut on device) over 1M x 1300B datagrams",
                       "filter_dispatch": "filter + dispatch GB/s (CRC check, verify, MERGED cut; device-resident) over 1M x 1300B datagrams",
                       "filter_then_dispatch": "filter + dispatch GB/s (two calls; device-resident) over 1M x 1300B datagrams",
                       "append": "outbound-layer GB/s (CRC + append, device-resident) over 1M mixed-length (64-1400B) payloads"}[args.workload],
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms if not DRY else 0.0,
            "settle_steps": settle_steps,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint on device, seed 42+rank), resident in HBM before timing",
            "config": {
                "workload": workload_name,
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
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": w["algo"],
                "kernel_ms": round(kern_max, 5),
                "kernel_ms_per_rank": [round(k, 5) for k in kern_all],
            },
        }
        line["distributed"] = ({"backend": backend, "world_size": world, "forced": bool(args.force_dist and world == 1),
                                "collectives": "barrier(device_ids), all_reduce MAX/SUM, all_gather on "
                                               + ("device tensors" if red_dev is not None else "CPU tensors")}
                               if dist_on else None)
        if DRY:
            line["dry_run"] = "LNL_BENCH_DRYRUN=1: CPU plumbing test, no kernel ran; figures are meaningless"
        if "line_bytes" in w:  # random narrow reads: HBM moves whole 64-B sectors
            lb = w["line_bytes"] / (kern_max * 1e-3) / 1e9
            line["roofline"]["sector_granular_bytes_per_launch"] = w["line_bytes"]
            line["roofline"]["sector_granular_achieved"] = round(lb, 1)
            line["roofline"]["sector_granular_frac"] = round(lb / HBM_PEAK_GBS, 4)
            if traffic:  # (the walk's FETCH_SIZE factor is calibrated: profiles/fetch_calibration.json)
                line["roofline"]["traffic_over_sector_floor"] = round(traffic / w["line_bytes"], 3)
            if not DRY:
                sec = hbm_probe_sectors(w["data"], device)
                if sec:
                    line["roofline"]["measured_random_sector_gbs"] = round(sec, 1)
                    line["roofline"]["sector_frac_of_measured"] = round(lb / sec, 4)
        if not DRY:
            probe = hbm_probe_peak(w["data"], device)
            if probe:
                peak = max(v for k, v in probe.items() if k in (0, 1, 11, 12, 13))  # whole-buffer streams
                names = {0: "global_load_dwordx4 nt", 1: "global_load_lds_dwordx4 nt",
                         2: "segment lanes, VGPR loads", 3: "segment lanes, VGPR loads nt",
                         4: "segment lanes, LDS-DMA nt", 5: "segment lanes, LDS-DMA nt, 5 waves/CU",
                         6: "segment lanes, LDS-DMA nt, 6 waves/CU",
                         7: "segment lanes, VGPR-staged nt + LDS transpose",
                         11: "one-shot grid, 4 KiB per workgroup, dwordx4 nt",
                         12: "one-shot grid, 16 KiB per workgroup, dwordx4 nt",
                         13: "one-shot grid, 8 KiB per wave, LDS-DMA nt"}
                line["roofline"]["measured_stream_read_peak_gbs"] = round(peak, 1)
                line["roofline"]["measured_stream_read_forms_gbs"] = {names[k]: round(v, 1) for k, v in probe.items()}
                line["roofline"]["frac_of_measured_peak"] = round(achieved / peak, 4)
        if w.get("filter_dispatch"):
            line["parity_whole_batch"] = ("exact" if min(ok_all) == 1.0 else "MISMATCH") + \
                " (every status ACCEPT; every packet's start, length and parent as laid out)"
        if crc_workload:
            line["parity_on_sample"] = ("bit-exact" if min(ok_all) == 1.0 else "MISMATCH") + \
                f" (first {min(w['n'], 1 << 14)} datagrams of each of {world} rank(s) vs the oracle)"
        if world == 1 and crc_workload and not args.no_cpu_baseline:
            res, cores, ref, quota = cpu_baseline(w, host)
            exact = bool(np.array_equal(out.cpu().numpy().view(np.uint32), ref))
            line["cpu_baseline"] = {
                "value": round(res[cores], 3),
                "unit": "GB/s",
                "cores": cores,
                "kind": "port",
                "sample": f"the whole batch ({w['n']} datagrams, {w['payload'] / 1e9:.3f} GB, copied to host "
                          f"memory untimed); oracle SSE4.2 crc32 loop, OpenMP, median of repeats over ~2 s",
                "single_core_value": round(res[1], 3),
                "all_cpus_value": round(res.get(os.cpu_count() or cores, res[cores]), 3),
                "all_cpus_threads": os.cpu_count(),
                "nproc": os.cpu_count(),
                "affinity_cpus": len(os.sched_getaffinity(0)),
                "cgroup_cpu_quota": quota,
                "cores_note": "threads = the CPUs this job may use: the affinity mask, capped by the cgroup "
                              "cpu.max quota when there is one (on the GPU box nproc shows the whole machine "
                              "but the job's share is a quota; more threads than that only time-slice)",
                "cpu_model": cpu_model(),
            }
            line["parity_whole_batch"] = "bit-exact" if exact else "MISMATCH"
        if world == 1 and w.get("append") and not args.no_host_path:  # the send side from host memory
            line["host_append"] = host_append_rate(P, host, w, torch.cuda.current_device())
        if world == 1 and crc_workload and not args.no_host_path:
            hp, got = host_path_rate(P, host, w, torch.cuda.current_device())
            hp["parity"] = "bit-exact vs the device-resident output" if np.array_equal(
                got, out.cpu().numpy().view(np.uint32)) else "MISMATCH"
            line["host_path"] = hp
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
