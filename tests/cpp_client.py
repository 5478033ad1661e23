"""Build helper for tests/cpp/abi_client.cpp: the C++ host side (include/mgmc_sampler.hh) linked
against the in-tree libmgmc_hip.so with g++, as a reference maintainer would link it."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_client(tmpdir, asan=False):
    """asan: the client (include/mgmc_sampler.hh and its caller) with AddressSanitizer + UBSan; the
    library itself stays uninstrumented (no device sanitizers on this pool)."""
    exe = os.path.join(str(tmpdir), "abi_client_asan" if asan else "abi_client")
    libdir = os.path.join(ROOT, "multigridmc_amd")
    san = ["-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"] \
        if asan else []
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", *san, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "abi_client.cpp"), "-L", libdir, "-lmgmc_hip",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    return exe
