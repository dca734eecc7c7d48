"""The C++ packet-layer mirror (include/lnl_crc32c_layer.hpp) compiled with
g++ against the in-tree library and run on the CPU."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_layer(tmp_path):
    libdir = os.path.join(ROOT, "litenetlibpp_amd")
    if not os.path.exists(os.path.join(libdir, "liblnl_crc32c.so")):
        subprocess.run(["make", "-C", libdir], check=True, capture_output=True)
    exe = tmp_path / "test_layer"
    subprocess.run(["g++", "-O1", "-std=c++17", "-o", str(exe),
                    os.path.join(ROOT, "tests", "cpp", "test_layer.cpp"),
                    f"-L{libdir}", "-llnl_crc32c", f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")
