"""Builds tempme_amd/lib/_dropin_ext*.so (csrc/dropin_ext.cpp: the drop-in fast path's host side on torch's
C++ API) in-tree with g++ against the installed torch; run by __graft_entry__.build() (on the CPU; the
built .so travels to the GPU box with the tree).  Rebuilt when the source is newer than the library."""
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "dropin_ext.cpp")


def target():
    return os.path.join(HERE, "lib", "_dropin_ext" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force=False):
    import torch
    out = target()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(SRC):
        return out
    tdir = os.path.dirname(torch.__file__)
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = out + ".tmp"
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__=1",
           "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_dropin_ext", f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-I" + os.path.join(tdir, "include"), "-I" + os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           "-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(rocm, "include"), SRC, "-o", tmp,
           "-L" + os.path.join(tdir, "lib"), "-ltorch_python", "-ltorch", "-lc10", "-lc10_hip",
           "-Wl,-rpath," + os.path.join(tdir, "lib")]
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
