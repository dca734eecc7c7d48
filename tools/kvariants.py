#!/usr/bin/env python3
"""Kernel-variant experiments (development tool, not the product path).

build:  python tools/kvariants.py build           (here, hipcc cross-compiles)
run:    python tools/kvariants.py run [--rounds R] (on the GPU box)

Each variant is the product library compiled with extra -D flags.  All
variants are timed in ONE process, interleaved over R rounds, on the same
device-resident data (cdna_hip_programming.md section 5.4 rule 24), with HIP
events on the launch stream; the median kernel time per variant is reported.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "litenetlibpp_amd", "build", "variants")

VARIANTS = {
    "base": "",                                     # shipped: lane-run kernel for fixed strides
    "span_nofold": "-DLNL_SPAN_DIAG=1",             # CSR span kernel without its folds (wrong CRCs)
    "span_noev": "-DLNL_SPAN_DIAG=2",               # CSR span kernel: rows + network only (wrong CRCs)
    "span_prev": ("", None, "build/span_prev.hip"),  # A/B: the span kernel source saved in build/ (untracked)
    "span_r3": "-DLNL_SPAN_ROWS_LATE=0 -DLNL_SPAN_FOLD_MASK=0 -DLNL_SPAN_TAIL_REG=0",  # span kernel as in round 3 (first rows with the probe; full-wave partial flushes)
    "span_early": "-DLNL_SPAN_ROWS_LATE=0",         # span kernel: first rows issued with the probe (round 3)
    "span_nofmask": "-DLNL_SPAN_FOLD_MASK=0",       # span kernel: partial flushes look up tables in every lane (round 3)
    "span_ef0": "-DLNL_SPAN_EARLY_FLUSH=0",         # fused walk kernel: no early flush (before round 4)
    "span_ef44": "-DLNL_SPAN_EARLY_FLUSH=44",       # ... fold a stash of >= N entries at a row step's start (product: 50)
    "span_ef56": "-DLNL_SPAN_EARLY_FLUSH=56",
    "span_tstash": "-DLNL_SPAN_TAIL_REG=0",         # span kernel: the segment's tail through the stash (round 3)
    "span_treg1": "-DLNL_SPAN_TAIL_REG=1",          # ... folded in registers after a separate last flush (product: 2)
    "span_ffmask": "-DLNL_SPAN_F_MASK=1",           # span kernel: F(b) read by the boundary lanes only
    "span_ffmask_tl": "-DLNL_SPAN_F_MASK=1 -DLNL_SPAN_DIAG=16",
    "span_finlds": "-DLNL_SPAN_FIN_LDS=1",
    "span_win9": "-DLNL_SPAN_WIN1=9u",              # span setup: 9 x 64 offsets in the first window (default 12)
    "span_win16": "-DLNL_SPAN_WIN1=16u",          # span kernel: heads' final map from the LDS tables
    "span_nob": "-DLNL_SPAN_DIAG=32",               # span kernel, no batch kernel after it (overflow datagrams unwritten)
    "span_noprio": "-DLNL_SPAN_PRIO=2",            # span kernel: no issue-priority balancing
    "span_prio_tl": "-DLNL_SPAN_PRIO=1 -DLNL_SPAN_DIAG=16",
    "span_timeline": "-DLNL_SPAN_DIAG=16",          # span kernel: per-wave timeline into out[] (wrong CRCs)
    "span_r3_tl": "-DLNL_SPAN_ROWS_LATE=0 -DLNL_SPAN_FOLD_MASK=0 -DLNL_SPAN_TAIL_REG=0 -DLNL_SPAN_DIAG=16",
    "run512": "-DLNL_RUN_THREADS=512",              # lane-run kernel: one 512-thread workgroup per CU
    "run512p": "-DLNL_RUN_THREADS=512 -DLNL_RUN_PRIO=1",  # ... with progress-based issue priority
    "noevent": "-DLNL_SCRATCH_EVENTS=0",            # no per-call last-use event on the span / XOR scratch (round 4)
    "ev_always": "-DLNL_SCRATCH_EVENT_FROM=0",      # every call records the last-use event (round 5's first form)
    "ev_sys": "-DLNL_SCRATCH_EVENT_FROM=0 -DLNL_SCRATCH_EVENT_FLAGS=hipEventDisableTiming",  # ... with the system fence
    "app_nobyte": "-DLNL_APPEND_DIAG=1",            # diagnostic (wrong wire): no head / tail byte stores
    "app_aligned": "-DLNL_APPEND_DIAG=2",           # diagnostic (wrong wire): aligned chunk loads only
    "app_diag3": "-DLNL_APPEND_DIAG=3",             # both
    "app_t16": "-DLNL_APPEND_TEAM=16u",             # copy kernel: 16 lanes per datagram (3 chunks in flight each)
    "app_t16u4": "-DLNL_APPEND_TEAM=16u -DLNL_APPEND_COPY_U=4",
    "app_t16u6": "-DLNL_APPEND_TEAM=16u -DLNL_APPEND_COPY_U=6",
    "app_t8u12": "-DLNL_APPEND_TEAM=8u -DLNL_APPEND_COPY_U=12",
    "app_t32u6": "-DLNL_APPEND_COPY_U=6",
    "app_t64u2": "-DLNL_APPEND_TEAM=64u -DLNL_APPEND_COPY_U=2",
    "app_t64u1": "-DLNL_APPEND_TEAM=64u -DLNL_APPEND_COPY_U=1",
    "app_th512": "-DLNL_APPEND_THREADS=512",        # ... 512-thread workgroups
    "app_th128": "-DLNL_APPEND_THREADS=128",
    "app_w16": "-DLNL_APPEND_WGS=16u",              # copy kernel: persistent grid, teams stride (round 4's product)
    "xg_r4": "-DLNL_XOR_GRID_U=4 -DLNL_XOR_GRID_XCD=1 -DLNL_XOR_GRID_PER=0 -DLNL_XOR_GRID_WGS=4u",  # CSR XOR grid, round 4
    "xg_xcd": "-DLNL_XOR_GRID_XCD=1",               # ... XCD-major wave numbering
    "xg_per16": "-DLNL_XOR_GRID_PER=16u",           # ... one workgroup per 16 datagrams
    "xg_per64": "-DLNL_XOR_GRID_PER=64u",
    "app_u1": "-DLNL_APPEND_COPY_U=1",              # outbound layer: round 3's copy kernel (one chunk load in flight per lane)
    "app_u2": "-DLNL_APPEND_COPY_U=2",
    "app_u4": "-DLNL_APPEND_COPY_U=4",
    "app_w8": "-DLNL_APPEND_WGS=8u",                # copy kernel: workgroups per CU (default: no cap)
    "app_w32": "-DLNL_APPEND_WGS=32u",
    "fix64": "-DLNL_SPAN_FIX_WGS=64u",              # batch kernel after the span kernel: 64 workgroups
    "fix8": "-DLNL_SPAN_FIX_WGS=8u",                # ... 8 workgroups
    "fix1": "-DLNL_SPAN_FIX_WGS=1u",                # ... 1 workgroup
    "xcsr_dflt": "-DLNL_XOR_CSR_NT=0",              # flat CSR XOR: default cache policy
    "xcsr_u1": "-DLNL_XOR_CSR_U=1",                 # flat CSR XOR: 1 piece per lane and chunk (1 KiB)
    "xcsr_u4": "-DLNL_XOR_CSR_U=4",                 # flat CSR XOR: 4 pieces per lane and chunk (4 KiB)
    "xcsr_u8": "-DLNL_XOR_CSR_U=8",                 # ... 8 (8 KiB)
    "xcsr_old": "-DLNL_XOR_CSR_FLAT=0",
    "xcsr_flat": "-DLNL_XOR_CSR_FLAT=1",            # flat CSR XOR (round 2's product path)
    "xstr_u2a2w8": "-DLNL_XOR_CSR_FLAT=2 -DLNL_XOR_STREAM_U=2 -DLNL_XOR_STREAM_AHEAD=2 -DLNL_XOR_STREAM_WGS=8",
    "xgrid_u2w5": "-DLNL_XOR_GRID_U=2 -DLNL_XOR_GRID_WGS=5",   # grid-interleaved CSR XOR: pieces per lane x workgroups per CU
    "xgrid_u2w6": "-DLNL_XOR_GRID_U=2 -DLNL_XOR_GRID_WGS=6",
    "xgrid_u3w5": "-DLNL_XOR_GRID_U=3 -DLNL_XOR_GRID_WGS=5",
    "xgrid_u3w4": "-DLNL_XOR_GRID_U=3 -DLNL_XOR_GRID_WGS=4",
    "xgrid_u4w3": "-DLNL_XOR_GRID_U=4 -DLNL_XOR_GRID_WGS=3",
    "xgrid_u8w2": "-DLNL_XOR_GRID_U=8 -DLNL_XOR_GRID_WGS=2",
    "xgrid_u1w8": "-DLNL_XOR_GRID_U=1 -DLNL_XOR_GRID_WGS=8",
    "xgrid_dflt": "-DLNL_XOR_CSR_NT=0",             # ... default cache policy
    "xcsr_prev": "",                                # A/B slot: built from another lnl_xor.hip copied in by hand             # CSR XOR: the per-datagram kernel (before)
    "span_r2": "-DLNL_SPAN_ROUNDS=2u",              # CSR span: segments for two wave-batches per wave (static)
    "span_r3": "-DLNL_SPAN_ROUNDS=3u",
    "span_r4": "-DLNL_SPAN_ROUNDS=4u",
    "disp_scan": "-DLNL_DISPATCH_SCAN=1",           # dispatch passes with the hipCUB scan between them (before: product sums workgroup totals)
    "walk_norow": "-DLNL_WALK_DIAG=1",              # filter + dispatch: no per-row walk (wrong packets)
    "walk_noend": "-DLNL_WALK_DIAG=2",              # ... no walk at datagram ends (wrong packets)
    "walk_notail": "-DLNL_WALK_DIAG=4",             # ... no global-memory finish (wrong packets)
    "walk_none": "-DLNL_WALK_DIAG=7",               # ... none of the three (wrong packets)
    "span_noF": "-DLNL_SPAN_DIAG=4",                # CSR span kernel: boundaries without the F(b) read (wrong CRCs)
    "span_noput": "-DLNL_SPAN_DIAG=8",              # ... without the stash writes (wrong CRCs)
    # (span_pre2, a row's second boundary piece read with the first boundary's F(b): commit 1545e07, measured no gain, removed)
    # (span_cnt / span_st_* / span_stage / span_coalst: the result-store experiments of commit 9db95bb, removed)
    "span_nostore": "-DLNL_SPAN_DIAG=128",           # ... CRC mode without its result stores (wrong results)
    "span_nob2": "-DLNL_SPAN_DIAG=64",              # ... a row's second and later boundaries skipped (wrong CRCs)
    "bucketed": ("", 4),                            # CSR: the bucketed batch kernel (previous default)
    "batch": "-DLNL_NO_RUN",                        # any-layout batch kernel for everything
    "bat_u": "-DLNL_BATCH_UNCAPPED=1",              # batch kernel: one batch per wave, grid in batch order
    "k8c": "-DLNL_RUN_K=8 -DLNL_RUN_UNCAPPED=0",    # lane runs of 8, grid capped at the resident waves (round 4)
    "k2u": "-DLNL_RUN_K=2",                         # lane runs of 2 (one batch per wave, uncapped: the default)
    "k4c": "-DLNL_RUN_UNCAPPED=0",                  # lane runs of 4, capped grid
    "k8": "-DLNL_RUN_K=8",                          # lane runs of 8 / 16 datagrams (uncapped grid)
    "k16": "-DLNL_RUN_K=16",
    "q32": "-DLNL_RUN_QMIN=32",                     # lane runs 32 datagrams apart (default: 16 at S = 1400)
    "q64": "-DLNL_RUN_QMIN=64",
    "k4q32": "-DLNL_RUN_K=4 -DLNL_RUN_QMIN=32",
    "run_dflt": "-DLNL_RUN_AUX=0",                  # default cache policy for the run kernel's loads
    "run_late": "-DLNL_RUN_EARLY_ROWS=0",           # run kernel: first rows issued after the tables land (before round 3)
    # (round 1's uniform / segment / pair CSR paths: tools/experiments/csr_experiment_kernels.patch;
    #  round 4's one-pass append, three-row lane-run kernel and other removed shapes:
    #  tools/experiments/round4_experiments.patch)
    "nobucket": "-DLNL_BUCKET_MIN_N=0xFFFFFFFFu",   # CSR: plain batch kernel, no pre-pass
    "bucket_atomic": "-DLNL_BUCKET_LAYOUT=0",       # CSR: atomic ranks, bucket after bucket (16 runs per bucket)
    "bucket_interleave": "-DLNL_BUCKET_LAYOUT=1",   # CSR: position-ordered buckets, batches interleaved by progress
    "xor_dflt": "-DLNL_XOR_NT=0",                   # XOR layer: default policy loads / stores
    "xor_g64": "-DLNL_XOR_GROUP=64",                # XOR layer: one datagram per wave
    "xor_g64u2": "-DLNL_XOR_GROUP=64 -DLNL_XOR_UNROLL=2",
    "xor_u1": "-DLNL_XOR_UNROLL=1",
    "xor_g64u2d": "-DLNL_XOR_GROUP=64 -DLNL_XOR_UNROLL=2 -DLNL_XOR_NT=0",
    "xor_g64u2d_nocap": "-DLNL_XOR_GROUP=64 -DLNL_XOR_UNROLL=2 -DLNL_XOR_NT=0 -DLNL_XOR_WG_PER_CU=0",
    "xor_g32u4d_nocap": "-DLNL_XOR_GROUP=32 -DLNL_XOR_UNROLL=4 -DLNL_XOR_NT=0 -DLNL_XOR_WG_PER_CU=0",
    "xor_g16u4d_nocap": "-DLNL_XOR_GROUP=16 -DLNL_XOR_UNROLL=4 -DLNL_XOR_NT=0 -DLNL_XOR_WG_PER_CU=0",
    "xor_g64u2_nocap": "-DLNL_XOR_GROUP=64 -DLNL_XOR_UNROLL=2 -DLNL_XOR_WG_PER_CU=0",
    "xor_g32u4_nocap": "-DLNL_XOR_GROUP=32 -DLNL_XOR_UNROLL=4 -DLNL_XOR_WG_PER_CU=0",
    "xor_g32u4d_cap16": "-DLNL_XOR_GROUP=32 -DLNL_XOR_UNROLL=4 -DLNL_XOR_NT=0 -DLNL_XOR_WG_PER_CU=16",
    "xor_g32u3d_nocap": "-DLNL_XOR_GROUP=32 -DLNL_XOR_UNROLL=3 -DLNL_XOR_NT=0 -DLNL_XOR_WG_PER_CU=0",
    "run_sc0": "-DLNL_RUN_AUX=1",
    "run_sc0nt": "-DLNL_RUN_AUX=3",
    "run_sc1": "-DLNL_RUN_AUX=16",
    "run_sc1nt": "-DLNL_RUN_AUX=18",
    "dflt": "-DLNL_GLDS_AUX=0",                     # default cache policy
    "nocomp": "-DLNL_DIAG_NO_COMPUTE",              # memory-pipeline ceiling (wrong CRCs)
    "nocomp_dflt": "-DLNL_DIAG_NO_COMPUTE -DLNL_GLDS_AUX=0",
    "edge2": "-DLNL_EDGE_AUX=2",                    # nt on first/last rows too
    "edge1": "-DLNL_EDGE_AUX=1",                    # sc0 on first/last rows
    "regmask": "-DLNL_MASK_IN_REGS",                # framing masks in registers, not LDS
}


def flags_path(v):
    """VARIANTS entry -> (extra -D flags, CSR path or None)."""
    return (v, None) if isinstance(v, str) else v[:2]


def span_src(v):
    """Optional third field: another span-kernel source (an A/B copy of an
    earlier version, outside the tree's sources), relative to litenetlibpp_amd/."""
    return v[2] if isinstance(v, tuple) and len(v) > 2 else "csrc/crc32c_span.hip"


def build(names):
    for n in names:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "litenetlibpp_amd"), "variant",
                        f"NAME={n}", f"VFLAGS={flags_path(VARIANTS[n])[0]}",
                        f"SPAN_SRC={span_src(VARIANTS[n])}"], check=True)
        print("built", n)


def run(names, rounds, workloads):
    import numpy as np
    import torch
    libs = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(VDIR, n + ".so"))
        L.lnl_crc32c_batch_fixed_dev.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.lnl_crc32c_batch_csr_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p, ctypes.c_void_p]
        L.lnl_xor_layer_fixed_dev.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]
        path = flags_path(VARIANTS[n])[1]
        if path is not None:
            L.lnl_crc32c_set_csr_path(path)
        libs[n] = L
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    results = {}
    for wl in workloads:
        s = torch.cuda.current_stream()
        if wl[0] == "xor":  # ("xor", n, len): XOR layer in place over n x len at stride len
            _, n_pk, L_pk = wl
            data = torch.randint(0, 256, (n_pk * L_pk,), dtype=torch.uint8, device=dev, generator=g)
            algo = 2 * n_pk * L_pk
            wkey = f"xor{n_pk}x{L_pk}"
            key = b"LiteNetLibPP-bench-key"

            def call(L):
                L.lnl_xor_layer_fixed_dev(data.data_ptr(), L_pk, L_pk, n_pk, key, len(key), s.cuda_stream)
        elif wl[0] == "csr":  # ("csr", n, lmin, lmax): config-3-shaped CSR batch
            _, n_pk, lmin, lmax = wl
            lens = torch.randint(lmin, lmax + 1, (n_pk,), device=dev, generator=g, dtype=torch.int64)
            off = torch.zeros(n_pk + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(lens, 0)
            total = int(off[-1])
            data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
            out = torch.empty(n_pk, dtype=torch.int32, device=dev)
            algo = total + 12 * n_pk + 8
            wkey = f"csr{n_pk}x{lmin}-{lmax}"

            def call(L):
                L.lnl_crc32c_batch_csr_dev(data.data_ptr(), off.data_ptr(), n_pk, out.data_ptr(), s.cuda_stream)
        elif wl[0] == "filter":  # ("filter", n, lmin, lmax): inbound filter over a CSR burst (random bytes)
            _, n_pk, lmin, lmax = wl
            lens = torch.randint(lmin, lmax + 1, (n_pk,), device=dev, generator=g, dtype=torch.int64)
            off = torch.zeros(n_pk + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(lens, 0)
            total = int(off[-1])
            data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
            st = torch.empty(n_pk, dtype=torch.uint8, device=dev)
            algo = total + n_pk + 8 * (n_pk + 1)
            wkey = f"filter{n_pk}x{lmin}-{lmax}"

            def call(L):
                L.lnl_inbound_filter_csr_dev(ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()),
                                             ctypes.c_uint32(n_pk), ctypes.c_void_p(st.data_ptr()),
                                             ctypes.c_void_p(s.cuda_stream))
        elif wl[0] == "append":  # ("append", n, lmin, lmax): the outbound layer over a CSR burst
            _, n_pk, lmin, lmax = wl
            lens = torch.randint(lmin, lmax + 1, (n_pk,), device=dev, generator=g, dtype=torch.int64)
            off = torch.zeros(n_pk + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(lens, 0)
            total = int(off[-1])
            data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
            wire = torch.empty(total + 4 * n_pk, dtype=torch.uint8, device=dev)
            out = torch.empty(n_pk, dtype=torch.int32, device=dev)
            algo = 2 * total + 8 * n_pk + 8 * (n_pk + 1)
            wkey = f"append{n_pk}x{lmin}-{lmax}"
            for L in libs.values():
                L.lnl_crc32c_append_csr_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]

            def call(L):
                L.lnl_crc32c_append_csr_dev(data.data_ptr(), off.data_ptr(), n_pk, wire.data_ptr(), out.data_ptr(),
                                            s.cuda_stream)
        elif wl[0] == "xorcsr":  # ("xorcsr", n[, lmin, lmax]): XOR layer in place over a CSR batch (config 3: 64..1400)
            n_pk = wl[1]
            lmin, lmax = (wl[2], wl[3]) if len(wl) > 3 else (64, 1400)
            lens = torch.randint(lmin, lmax + 1, (n_pk,), device=dev, generator=g, dtype=torch.int64)
            off = torch.zeros(n_pk + 1, dtype=torch.int64, device=dev)
            off[1:] = torch.cumsum(lens, 0)
            total = int(off[-1])
            data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
            algo = 2 * total + 8 * (n_pk + 1)
            wkey = f"xorcsr{n_pk}" + (f"x{lmin}-{lmax}" if len(wl) > 3 else "")
            key = b"LiteNetLibPP-bench-key"
            for L in libs.values():
                L.lnl_xor_layer_csr_dev.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                    ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p]

            def call(L):
                L.lnl_xor_layer_csr_dev(data.data_ptr(), off.data_ptr(), n_pk, key, len(key), s.cuda_stream)
        elif wl[0] == "disp":  # ("disp", n): lnl_dispatch_csr_dev over n MERGED containers of 5 x 256-B packets
            n_pk = wl[1]
            S = 1 + 5 * 259 + 4
            data = torch.randint(0, 256, (n_pk * S,), dtype=torch.uint8, device=dev, generator=g)
            d2 = data.view(n_pk, S)
            d2[:, 0] = 0x0C
            for j in range(5):
                d2[:, 1 + 259 * j] = 1
                d2[:, 2 + 259 * j] = 1
                d2[:, 3 + 259 * j] = 0
            off = torch.arange(0, (n_pk + 1) * S, S, dtype=torch.int64, device=dev)
            st = torch.ones(n_pk, dtype=torch.uint8, device=dev)  # every container accepted
            k = 5 * n_pk
            pst = torch.empty(k, dtype=torch.int64, device=dev)
            pl = torch.empty(k, dtype=torch.int32, device=dev)
            pp = torch.empty(k, dtype=torch.int32, device=dev)
            tot = torch.zeros(1, dtype=torch.int32, device=dev)
            algo = n_pk * 10 + 19 * k
            wkey = f"disp{n_pk}"
            outs_ref = {}

            def call(L):
                L.lnl_dispatch_csr_dev(
                    ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), ctypes.c_uint32(n_pk),
                    ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(pst.data_ptr()), ctypes.c_void_p(pl.data_ptr()),
                    ctypes.c_void_p(pp.data_ptr()), ctypes.c_uint32(k), ctypes.c_void_p(tot.data_ptr()),
                    ctypes.c_void_p(s.cuda_stream))
            for name, L in libs.items():  # same packets from every variant
                pst.fill_(-1)
                call(L)
                torch.cuda.synchronize()
                outs_ref[name] = (int(tot.item()), pst.clone(), pl.clone(), pp.clone())
            ref0 = next(iter(outs_ref.values()))
            for name, r in outs_ref.items():
                same = r[0] == ref0[0] and all(torch.equal(x, y) for x, y in zip(r[1:], ref0[1:]))
                print(f"{name}@{wkey} packets {r[0]} same-as-first {same}", flush=True)
        elif wl[0] == "fd":  # ("fd", n): filter + dispatch over n MERGED containers of 5 x 256-B packets
            n_pk = wl[1]
            S = 1 + 5 * 259 + 4
            data = torch.randint(0, 256, (n_pk * S,), dtype=torch.uint8, device=dev, generator=g)
            d2 = data.view(n_pk, S)
            d2[:, 0] = 0x0C
            for j in range(5):
                d2[:, 1 + 259 * j] = 1
                d2[:, 2 + 259 * j] = 1
                d2[:, 3 + 259 * j] = 0
            off = torch.arange(0, (n_pk + 1) * S, S, dtype=torch.int64, device=dev)
            st = torch.empty(n_pk, dtype=torch.uint8, device=dev)
            k = 5 * n_pk
            pst = torch.empty(k, dtype=torch.int64, device=dev)
            pl = torch.empty(k, dtype=torch.int32, device=dev)
            pp = torch.empty(k, dtype=torch.int32, device=dev)
            tot = torch.zeros(1, dtype=torch.int32, device=dev)
            algo = n_pk * S + 8 * (n_pk + 1) + n_pk + 16 * k
            wkey = f"fd{n_pk}"

            def call(L):  # (CRC fields are random: statuses DROP, the walk still runs)
                L.lnl_inbound_filter_dispatch_csr_dev(
                    ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(off.data_ptr()), ctypes.c_uint32(n_pk),
                    ctypes.c_void_p(st.data_ptr()), ctypes.c_void_p(pst.data_ptr()), ctypes.c_void_p(pl.data_ptr()),
                    ctypes.c_void_p(pp.data_ptr()), ctypes.c_uint32(k), ctypes.c_void_p(tot.data_ptr()),
                    ctypes.c_void_p(s.cuda_stream))
        else:
            n_pk, L_pk, stride, shift = wl
            buf = torch.randint(0, 256, (n_pk * stride + 256,), dtype=torch.uint8, device=dev, generator=g)
            data = buf[shift:]
            out = torch.empty(n_pk, dtype=torch.int32, device=dev)
            algo = n_pk * (L_pk + 4)
            wkey = f"{n_pk}x{L_pk}/s{stride}+{shift}"

            def call(L):
                L.lnl_crc32c_batch_fixed_dev(data.data_ptr(), stride, L_pk, n_pk, out.data_ptr(), s.cuda_stream)
        if wl[0] in ("csr", "append") or isinstance(wl[0], int):
            # outputs of every variant against the first (CRC workloads; the
            # diagnostic builds are expected to differ)
            ref_out = None
            for n in names:
                out.fill_(0)
                call(libs[n])
                torch.cuda.synchronize()
                if ref_out is None:
                    ref_out = out.clone()
                print(f"{n}@{wkey} outputs same-as-first {bool(torch.equal(out, ref_out))}", flush=True)
        times = {n: [] for n in names}
        import time as _time
        t_settle = _time.perf_counter() + 0.15  # sustained clocks first (bench.py --settle-ms)
        while _time.perf_counter() < t_settle:
            for n in names:
                call(libs[n])
            torch.cuda.synchronize()
        for r in range(rounds):
            for n in names:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                call(libs[n])
                e0.record(s)
                for _ in range(3):
                    call(libs[n])
                e1.record(s)
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1) / 3)
        for n in names:
            med = float(np.median(times[n]))
            key = f"{n}@{wkey}"
            results[key] = {"us": round(med * 1e3, 2), "min_us": round(min(times[n]) * 1e3, 2),
                            "GBps": round(algo / (med * 1e-3) / 1e9, 1)}
            print(key, results[key], flush=True)
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--names", default=",".join(VARIANTS))
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--workloads", default="1048576:1400:1400:0,csr:1048576:64:1400",
                    help="n:len:stride:byte_shift or csr:n:min_len:max_len, comma-separated")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "kvariants.json"))
    a = ap.parse_args()
    names = a.names.split(",")
    if a.cmd == "build":
        build(names)
    else:
        wl = [(w.split(":")[0],) + tuple(int(v) for v in w.split(":")[1:]) if w.split(":")[0] in ("csr", "xor", "append", "filter", "fd", "xorcsr", "disp")
              else tuple(int(v) for v in w.split(":")) for w in a.workloads.split(",")]
        res = run(names, a.rounds, wl)
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
