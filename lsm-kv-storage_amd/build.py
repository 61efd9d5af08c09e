"""Build the in-tree native libraries of the SST block codec.

    python lsm-kv-storage_amd/build.py          # libsstcodec.so (gfx950)

Outputs go to lsm-kv-storage_amd/lib/ (git-ignored, shipped to the GPU box with
the repo snapshot).  hipcc cross-compiles for gfx950 without a GPU.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
ARCH = os.environ.get("SSTC_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["sstc_kernels.hip", "sstc_compact.hip", "sstc_get.hip", "sstc_api.hip"]
HOST_SOURCES = ["host/sst_table.cpp", "host/compact_files.cpp"]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the codec has no CPU build")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False):
    os.makedirs(os.path.join(LIB, "obj"), exist_ok=True)
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, h) for h in ("sstc_device.h", "sstc_launch.h")]
    headers.append(os.path.join(ROOT, "include", "sstcodec.h"))
    host_headers = [os.path.join(CSRC, "host", "sst_table.h"), os.path.join(ROOT, "include", "sstc_table.h")]
    objs = []
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result"]
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(LIB, "obj", os.path.basename(src) + ".o")
        if _newer(o, [s] + headers):
            cmd = [hipcc] + flags + ["-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
        objs.append(o)
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        if not os.path.exists(s):
            continue
        o = os.path.join(LIB, "obj", os.path.basename(src) + ".o")
        if _newer(o, [s] + headers + [h for h in host_headers if os.path.exists(h)]):
            rocm = os.path.dirname(os.path.dirname(os.path.realpath(hipcc)))
            cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-Wall", "-D__HIP_PLATFORM_AMD__",
                   "-I" + os.path.join(rocm, "include"), "-I" + os.path.join(ROOT, "include"), "-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
        objs.append(o)
    so = os.path.join(LIB, "libsstcodec.so")
    if _newer(so, objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    # a C++ caller compiled against include/sstc_table.h (the drop-in surface):
    # the DoCompactJob loop over sstc::TableBuilder / TableReaderIterator
    tu = os.path.join(ROOT, "tests", "cpp", "compact_loop.cc")
    exe = os.path.join(LIB, "sstc_compact_loop")
    if os.path.exists(tu) and _newer(exe, [tu, so, os.path.join(ROOT, "include", "sstc_table.h")]):
        cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"), tu,
               "-o", exe, "-L" + LIB, "-lsstcodec", "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return so


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
