"""The product kernels' register discipline around their inline-asm loads (CPU
test, reads the built library; no GPU).

The CRC kernels wait for their own row, table and offset loads with counted
`s_waitcnt vmcnt(N)`.  The compiler does not see those inline-asm
loads: it treats their destination registers as written when the asm
statement ends.  Three things must therefore hold in the code object, and are
checked here:

* no scratch: a spill would put scratch loads and stores -- and the
  compiler's own vmcnt waits for them -- into the middle of that accounting,
  and a spilled in-flight register is stored before it lands;
* no accumulation registers: once the compiler parks values in AGPRs it
  copies registers with v_accvgpr_write, and a copy of an asm-load
  destination taken before its wait is the round-4 three-row fault
  (profiles/bench_r04b/r04ad_span_rows3_fault.log);
* no register of a load in flight is touched before the wait that covers
  it: tests/isa_scan.py, a path-sensitive scan of the disassembly.

The scan is exact on straight-line code and follows the compiler's
correlated scalar branches, but it does not do arithmetic on loop counters.
The span kernel's row pipeline issues row t + 2 when t + 2 < R and waits for
row t with vmcnt(8) when t + 1 < R; that the two bounds agree across the
loop's back edge is arithmetic, so the scan reports the first touch of the
row buffers after that wait (the transposes into the LDS image, and the
compiler's reuse of those registers after the last row).  Those reports are
bounded here to the row-buffer registers, so a hazard on any other asm load
in those kernels still fails; with no AGPR and no scratch, no in-flight
register can be parked or spilled, which is what the round-4 variant did.  The controls
(tests/isa/asm_load_controls.hip, built here for gfx950 and never run) show
that the scan flags a read, an AGPR copy, a short count and a loop-skipped
wait, and passes the correct forms."""
import os
import shutil
import subprocess
import tempfile

import pytest

import isa_scan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "litenetlibpp_amd", "liblnl_crc32c.so")
HIPCC = "/opt/rocm/bin/hipcc"
CONTROLS = os.path.join(ROOT, "tests", "isa", "asm_load_controls.hip")

# The span kernels (crc32c_span.hip) scanned with a smaller path budget (they
# are ~30 K instructions each; their residual reports are bounded by kind)
SPAN = "crc32c_span_kernel"


def _have_tools():
    return os.path.exists(os.path.join(isa_scan.LLVM, "llvm-objdump")) and os.path.exists(LIB)


@pytest.fixture(scope="module")
def code_objects():
    if not _have_tools():
        pytest.skip("ROCm llvm tools or the built library not present")
    d = tempfile.mkdtemp()
    try:
        yield isa_scan.library_code_objects(LIB, d)
    finally:
        shutil.rmtree(d, ignore_errors=True)


@pytest.fixture(scope="module")
def product_scan(code_objects):
    text = isa_scan.disassemble_code_objects(code_objects)
    kernels = {k: v for k, v in isa_scan.parse(text).items() if "lnl" in k}
    return {k: (v, isa_scan.scan_kernel(k, v, 8 if SPAN in k else None)) for k, v in kernels.items()}


def test_product_kernels_have_no_scratch_and_no_agprs(code_objects):
    notes = isa_scan.kernel_notes(code_objects)
    ours = {k: v for k, v in notes.items() if "lnl" in k}
    assert any(SPAN in k for k in ours), sorted(notes)[:10]
    assert any("crc32c_run_kernel" in k for k in ours)
    bad = {k: v for k, v in ours.items()
           if v.get("private_segment_fixed_size", 1) or v.get("vgpr_spill_count", 1) or v.get("agpr_count", 1)}
    assert not bad, bad


def test_no_in_flight_register_touched_outside_the_row_pipeline(product_scan):
    """Every product kernel but the span kernels: no hazard at all (the lane-run
    kernel's table and row loads, the batch, bucket, dispatch, append and XOR
    kernels)."""
    checked = 0
    for k, (_, hazards) in product_scan.items():
        if SPAN in k:
            continue
        assert not hazards, "\n".join(str(h) for h in hazards[:10])
        checked += 1
    assert checked >= 15


def test_span_kernel_reports_are_row_buffer_registers_only(product_scan):
    """The span kernels: what the scan cannot clear touches the row buffers
    only (ra, rb: the destinations of the row loads) -- their transposes
    after the counted wait, and the compiler's reuse of those registers once
    the rows are done.  Every other asm load (the offset window, the probe,
    the tables) is clear, and with no AGPR and no scratch in the kernel
    (above) no in-flight register can be copied or spilled."""
    seen = 0
    for k, (insns, hazards) in product_scan.items():
        if SPAN not in k:
            continue
        seen += 1
        rows = set()
        for x in insns:
            if x.op == "global_load_dwordx4" and x.args.rstrip().endswith("nt"):
                rows |= set(isa_scan.vmem_dest(x))
        # 2 buffers x 8 loads x 4 registers, plus the table loads' (also nt)
        assert 64 <= len(rows) <= 80, len(rows)
        for h in hazards:
            assert set(h.regs) <= rows, str(h)
            assert not h.text.startswith(("v_accvgpr", "scratch_")), str(h)
        assert any(h.text.startswith("ds_write_b128") for h in hazards) or not hazards
    assert seen == 2


@pytest.fixture(scope="module")
def controls():
    if not (os.path.exists(HIPCC) and os.path.exists(os.path.join(isa_scan.LLVM, "llvm-objdump"))):
        pytest.skip("hipcc / llvm tools not present")
    d = tempfile.mkdtemp()
    try:
        co = os.path.join(d, "controls.co")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "--no-gpu-bundle-output",
                        "-c", CONTROLS, "-o", co], check=True, capture_output=True)
        yield isa_scan.scan_code_object(co)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_scan_flags_the_hazard_controls(controls):
    for name in ("bad_read_before_wait", "bad_agpr_copy_before_wait", "bad_count_short", "bad_loop_skipped_wait"):
        assert controls[name], name
    assert any(h.text.startswith("v_accvgpr_write") for h in controls["bad_agpr_copy_before_wait"])


def test_scan_passes_the_correct_controls(controls):
    for name in ("good_wait_then_read", "good_counted_pipeline", "good_flagged_waits"):
        assert not controls[name], (name, [str(h) for h in controls[name]])
