"""The C++ mirrors of the reference interfaces (include/h3c_checksum_info.hpp,
include/h3c_storage.hpp) compiled against the C ABI and run as programs."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
LIBDIR = os.path.join(ROOT, "3fs_amd", "_lib")
ORADIR = os.path.join(ROOT, "oracle", "build")
HEADERS = [os.path.join(ROOT, "include", h) for h in ("h3c_crc.h", "h3c_checksum_info.hpp", "h3c_storage.hpp")]
PROGRAMS = ["checksum_info_test", "storage_path_test"]


def build(name):
    src = os.path.join(CPP, name + ".cpp")
    exe = os.path.join(CPP, "build", name)
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(p) for p in [src] + HEADERS):
        return exe
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o", exe, src,
           f"-L{LIBDIR}", "-lh3c_crc", f"-L{ORADIR}", "-loracle", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{LIBDIR}", f"-Wl,-rpath,{ORADIR}", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return exe


@pytest.mark.parametrize("name", PROGRAMS)
def test_cpp_mirror_cpu(name):
    r = subprocess.run([build(name), "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", PROGRAMS)
def test_cpp_mirror_gpu(name):
    r = subprocess.run([build(name), "gpu"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
