#!/usr/bin/env python3
"""Build the REFERENCE's net_manager with the CRC-32C layer on (test
infrastructure; run in the build container only).

The reference library (/root/reference/src/lnl/**/*.cpp) and its example
server/client are compiled where they lie with g++ (the reference's own
CMakeLists needs only pthread).  Nothing from /root/reference is copied: every
output -- objects and executables -- goes to oracle/_ref/net/<variant>/, which
git ignores.  The three INTEGRATION.md edits are applied without editing any
reference file:

  send_raw / receive_logic   link-time: -Wl,--wrap=sendto,--wrap=recvfrom
                             route the two socket calls through
                             oracle/refnet/refnet_wrap.cpp, which calls the
                             product library's layer (liblnl_crc32c.so)
  POSSIBLE_MTU - 4           compile-time: each translation unit is
                             preprocessed (g++ -E) and the three places that
                             turn an MTU index into an MTU (net_peer.h:171
                             set_mtu, net_peer.cpp:336 the MTU_OK check,
                             net_peer.cpp:689 the probe size) get
                             "- LNL_CRC32C_LAYER_EXTRA", exactly upstream
                             LiteNetLib's ExtraPacketSizeForLayer; the
                             preprocessed text only passes through a pipe into
                             g++ -x c++.  MAX_PACKET_SIZE (the recvfrom
                             buffer, 1432) is unchanged, so the 1428-byte
                             probe plus its CRC still fits.

Variants:
  plain      no layer (the wrappers only observe): the reference as it is
  crc        the layer on, MTU - 4
  crc_nomtu  the layer on, MTU table untouched (negative control: the 1432
             probe no longer fits and the MTU settles one step lower)
  crc_src    the layer on, MTU - 4, and the send_raw / receive_logic edits of
             INTEGRATION.md 2 applied as source text rather than at link
             time: net_manager.cpp is preprocessed with refnet_layer.hpp
             force-included, its sendto in send_raw and its
             "packet->resize(size); on_message_received(packet, addr);" in
             receive_logic are replaced by the INTEGRATION.md snippets
             (m_crc_layer -> refnet_crc_layer(this)), and the wrappers only
             observe (REFNET_CRC=2).  A dropped datagram is then recycled and
             the loop goes back to its poll, exactly as the snippet says.

Usage: python3 oracle/refnet/build.py [--if-stale] [variant ...]   (default: all three)
"""
import os
import re
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("LNL_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "oracle", "_ref", "net")
LIBDIR = os.path.join(REPO, "litenetlibpp_amd")
CXX = os.environ.get("CXX", "g++")
FLAGS = ["-std=c++17", "-O2", "-I" + os.path.join(REF, "include")]

# "net_constants::POSSIBLE_MTU[<mtu index>]" where an index becomes an MTU
MTU_USE = re.compile(r"net_constants\s*::\s*POSSIBLE_MTU\s*\[\s*(mtuIdx|m_mtu_idx\s*\+\s*1)\s*\]")


def layer_extra():
    with open(os.path.join(REPO, "include", "lnl_crc32c.h")) as f:
        m = re.search(r"#define\s+LNL_CRC32C_LAYER_EXTRA\s+(\d+)", f.read())
    return int(m.group(1))


def lib_sources():
    src = []
    for root, _, files in os.walk(os.path.join(REF, "src")):
        src += [os.path.join(root, f) for f in files if f.endswith(".cpp")]
    return sorted(src)


# INTEGRATION.md 2, send_raw (net_manager.cpp:519-521): the sendto of data[offset ..
# offset+length) becomes the layer's scratch copy with the CRC appended
SEND_RAW = re.compile(r"auto\s+result\s*=\s*sendto\s*\(\s*m_socket\s*,\s*\(const char\s*\*\)\s*&data\[offset\]\s*,"
                      r"\s*\(int\)\s*length\s*,\s*0\s*,\s*\(sockaddr\s*\*\)\s*&endpoint\.raw\s*,"
                      r"\s*sizeof\s*\(\s*sockaddr_in\s*\)\s*\)\s*;")
SEND_RAW_NEW = (
    "thread_local uint8_t crc_scratch[net_constants::MAX_PACKET_SIZE + lnl::crc32c_layer::extra_packet_size_for_layer];\n"
    "    const size_t wire_len = refnet_crc_layer(this).process_outbound_packet(&data[offset], length,\n"
    "                                                                        crc_scratch, sizeof crc_scratch);\n"
    "    auto result = sendto(m_socket, (const char*) crc_scratch, (int) wire_len, 0,\n"
    "                         (sockaddr*) &endpoint.raw, sizeof(sockaddr_in));")
# INTEGRATION.md 2, receive_logic (net_manager.cpp:218-222)
RECEIVE = re.compile(r"packet->resize\(size\);\s*on_message_received\(packet,\s*addr\);")
RECEIVE_NEW = (
    "packet->resize(size);\n"
    "        size_t len = packet->size();\n"
    "        if (!refnet_crc_layer(this).process_inbound_packet(packet->data(), len)) {\n"
    "            pool_recycle(packet);\n"
    "            continue;\n"
    "        }\n"
    "        packet->resize(len);\n"
    "        on_message_received(packet, addr);")


def compile_tu(src, obj, mtu_edit, extra, src_edit=False):
    """g++ -c, or (MTU edit) g++ -E | rewrite | g++ -x c++ -c -; returns the
    number of MTU sites rewritten.  src_edit (crc_src, net_manager.cpp): the
    INTEGRATION.md send_raw / receive_logic snippets too, refnet_layer.hpp
    force-included."""
    if not mtu_edit:
        subprocess.run([CXX] + FLAGS + ["-c", src, "-o", obj], check=True)
        return 0
    pre_flags = ["-include", os.path.join(HERE, "refnet_layer.hpp")] if src_edit else []
    pre = subprocess.run([CXX] + FLAGS + pre_flags + ["-E", src], check=True, capture_output=True, text=True).stdout
    text, n = MTU_USE.subn(lambda m: f"(net_constants::POSSIBLE_MTU[{m.group(1)}] - {extra})", pre)
    if src_edit:
        text, ns = SEND_RAW.subn(lambda m: SEND_RAW_NEW, text)
        text, nr = RECEIVE.subn(lambda m: RECEIVE_NEW, text)
        assert ns == 1 and nr == 1, (ns, nr)
    subprocess.run([CXX, "-std=c++17", "-O2", "-x", "c++", "-c", "-", "-o", obj], input=text, text=True,
                   check=True)
    return n


def build(variant):
    crc = variant != "plain"
    mtu_edit = variant in ("crc", "crc_src")
    src_edit = variant == "crc_src"
    extra = layer_extra()
    d = os.path.join(OUT, variant)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    objs, sites = [], {}
    for src in lib_sources():
        obj = os.path.join(d, os.path.basename(src)[:-4] + ".o")
        sites[os.path.basename(src)] = compile_tu(src, obj, mtu_edit, extra,
                                                  src_edit and os.path.basename(src) == "net_manager.cpp")
        objs.append(obj)
    if mtu_edit:
        # set_mtu (inline, net_peer.h) in every unit that includes it, plus the
        # two sites in net_peer.cpp
        assert sites["net_peer.cpp"] == 3, sites
        assert all(v <= 1 for k, v in sites.items() if k != "net_peer.cpp"), sites
    wrap = os.path.join(d, "refnet_wrap.o")
    subprocess.run([CXX, "-std=c++17", "-O2", f"-DREFNET_CRC={2 if src_edit else (1 if crc else 0)}", "-c",
                    os.path.join(HERE, "refnet_wrap.cpp"), "-o", wrap], check=True)
    link = [wrap, "-Wl,--wrap=sendto", "-Wl,--wrap=recvfrom", "-L" + LIBDIR, "-llnl_crc32c",
            "-Wl,-rpath," + LIBDIR, "-lpthread"]
    exes = {"refnet_driver": os.path.join(HERE, "refnet_driver.cpp"),
            "lnl_example_server": os.path.join(REF, "example", "server.cpp"),
            "lnl_example_client": os.path.join(REF, "example", "client.cpp")}
    for name, src in exes.items():
        obj = os.path.join(d, name + ".o")
        compile_tu(src, obj, mtu_edit, extra)
        subprocess.run([CXX, "-o", os.path.join(d, name), obj] + objs + link, check=True)
    return sites


def stale(variant):
    """True when a variant's driver is missing or older than anything it is built from."""
    exe = os.path.join(OUT, variant, "refnet_driver")
    if not os.path.exists(exe):
        return True
    t = os.path.getmtime(exe)
    deps = lib_sources() + [os.path.join(HERE, f)
                            for f in ("build.py", "refnet_wrap.cpp", "refnet_driver.cpp", "refnet_layer.hpp")]
    deps += [os.path.join(LIBDIR, "liblnl_crc32c.so"), os.path.join(REPO, "include", "lnl_crc32c.h")]
    return any(os.path.getmtime(f) > t for f in deps)


def main():
    args = [a for a in sys.argv[1:] if a != "--if-stale"]
    only_stale = "--if-stale" in sys.argv[1:]
    if not os.path.isdir(os.path.join(REF, "src")):
        print(f"no reference at {REF}: nothing to build", file=sys.stderr)
        return 1
    if not os.path.exists(os.path.join(LIBDIR, "liblnl_crc32c.so")):
        print("build litenetlibpp_amd/liblnl_crc32c.so first (make -C litenetlibpp_amd)", file=sys.stderr)
        return 1
    for v in args or ["plain", "crc", "crc_nomtu", "crc_src"]:
        if only_stale and not stale(v):
            print(v, "up to date")
            continue
        sites = build(v)
        print(v, "built; MTU sites rewritten:", sum(sites.values()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
