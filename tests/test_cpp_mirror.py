"""The C++ ChecksumInfo mirror (include/h3c_checksum_info.hpp) compiled and run as a program."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "checksum_info_test.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "build", "checksum_info_test")
LIBDIR = os.path.join(ROOT, "3fs_amd", "_lib")
ORADIR = os.path.join(ROOT, "oracle", "build")


def build():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    if os.path.exists(EXE) and os.path.getmtime(EXE) > max(os.path.getmtime(SRC), os.path.getmtime(
            os.path.join(ROOT, "include", "h3c_checksum_info.hpp"))):
        return EXE
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    cmd = ["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o", EXE, SRC,
           f"-L{LIBDIR}", "-lh3c_crc", f"-L{ORADIR}", "-loracle", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{LIBDIR}", f"-Wl,-rpath,{ORADIR}", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return EXE


def test_cpp_mirror_cpu():
    r = subprocess.run([build(), "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_gpu():
    r = subprocess.run([build(), "gpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
