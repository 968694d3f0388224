"""In-tree native build: HIP kernels (hipcc, gfx950) + C++ runtime -> ``multidisttorch_amd/_C.so``.

No JIT cache, no hipify: ``csrc/kernels/*.hip`` are CDNA4 sources compiled with
``hipcc --offload-arch=gfx950``; ``csrc/runtime/*.cpp`` and ``csrc/bindings.cpp``
are host C++ against torch's headers. The shared object links torch's bundled
``libamdhip64`` (same SONAME as the system one, and already loaded by
``import torch``) so only one HIP runtime ever lives in the process.

Usage: ``python -m multidisttorch_amd._build [-j N] [--force]``.

``MDT_SANITIZE=1`` builds a second, host-sanitized copy
(``build/san/_C.so``, objects in ``build/native_san``): the C++ runtime
(reducers, stream/event bookkeeping, planners, bindings) is compiled with
``-fsanitize=address,undefined``; the gfx950 kernels are unchanged (GPU
sanitizers are not available on the pool). Load it with
``MDT_NATIVE_SO=build/san/_C.so`` under ``LD_PRELOAD=<libasan.so>`` on a CPU
host (``scripts/sanitize_host.sh``).
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "multidisttorch_amd")
CSRC = os.path.join(ROOT, "csrc")
SANITIZE = os.getenv("MDT_SANITIZE", "0") == "1"
# MDT_BUILD_TAG=name: an A/B variant (e.g. with MDT_HIP_EXTRA_FLAGS=-D...) built
# into variants/<name>/_C.so (objects in build/native_<name>); load it on the
# GPU box with MDT_NATIVE_SO=variants/<name>/_C.so. The default build is untouched.
TAG = os.getenv("MDT_BUILD_TAG", "")
BUILD = os.path.join(ROOT, "build", "native_san" if SANITIZE else ("native_" + TAG if TAG else "native"))
OUT = (os.path.join(ROOT, "build", "san", "_C.so") if SANITIZE else
       os.path.join(ROOT, "variants", TAG, "_C.so") if TAG else os.path.join(PKG, "_C.so"))
SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
ARCH = os.environ.get("MDT_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _sources():
    kern = sorted(os.path.join(CSRC, "kernels", f) for f in os.listdir(os.path.join(CSRC, "kernels"))
                  if f.endswith(".hip"))
    host = sorted(os.path.join(CSRC, "runtime", f) for f in os.listdir(os.path.join(CSRC, "runtime"))
                  if f.endswith(".cpp"))
    host.append(os.path.join(CSRC, "bindings.cpp"))
    return kern, host


def _headers():
    hs = []
    for d, _, fs in os.walk(CSRC):
        hs += [os.path.join(d, f) for f in fs if f.endswith((".h", ".hpp"))]
    return sorted(hs)


def _stamp(paths, flags):
    h = hashlib.sha1(" ".join(flags).encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _compile(cmd, src, obj, stamp):
    sfile = obj + ".stamp"
    if os.path.exists(obj) and os.path.exists(sfile) and open(sfile).read() == stamp:
        return obj, False, ""
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(sfile, "w") as f:
        f.write(stamp)
    return obj, True, r.stderr


def hip_flags():
    # MDT_HIP_EXTRA_FLAGS: compile-time A/B switches (e.g. -DNAME=1)
    extra = os.getenv("MDT_HIP_EXTRA_FLAGS", "").split()
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
            "-Wno-unused-result", "-I" + os.path.join(CSRC, "kernels")] + extra


# Per-file code-generation flags. -amdgpu-mfma-vgpr-form: MFMA accumulators in
# the VGPR file. With the default AGPR form the compiler copied every loop-
# carried accumulator AGPR -> VGPR -> AGPR around the k-loop back edge of the
# conv GEMM kernels (3-4 thousand v_accvgpr moves per file; none in the fused
# 28x28 / MLP kernels, which keep the default).
FILE_FLAGS = {
    "conv_igemm.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
    "conv_jobs.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
    "conv_thin.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


# Host files with their own flags: the native CPU step (config #1) vectorises
# its fused elementwise loops (sqrt/div for Adam under IEEE rules; exp/log via
# glibc's libmvec in the fast-math loss file only: under -ffast-math GCC's
# vectorised Adam produced NaN for zero gradients); AVX2 + FMA only, which
# every x86-64 host of an MI355X node has.
HOST_FILE_FLAGS = {
    "cpu_mlp.cpp": ["-O3", "-mavx2", "-mfma", "-fno-math-errno"],
    "cpu_mlp_bce.cpp": ["-O3", "-mavx2", "-mfma", "-ffast-math"],
}


def build(jobs: int = 8, force: bool = False, verbose: bool = False) -> str:
    inc, tlib, abi = _torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    kern, host = _sources()
    hdrs = _headers()
    pyinc = sysconfig.get_paths()["include"]
    host_flags = ["-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                  "-DHIPBLAS_V2", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C",
                  f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-Wno-deprecated-declarations",
                  "-I" + CSRC, "-I" + pyinc] + ["-I" + p for p in inc] + ["-I" + os.path.join(ROCM, "include")]
    if SANITIZE:
        host_flags = ["-O1" if f == "-O2" else f for f in host_flags] + SAN_FLAGS
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    jobsl = []
    for s in kern:
        obj = os.path.join(BUILD, os.path.basename(s) + ".o")
        flags = hip_flags()
        if os.getenv("MDT_MFMA_VGPR", "1") != "0":
            flags = flags + FILE_FLAGS.get(os.path.basename(s), [])
        cmd = [hipcc] + flags + ["-c", s, "-o", obj]
        jobsl.append((cmd, s, obj, _stamp([s] + hdrs, flags + ["force" if force else ""])))
    for s in host:
        obj = os.path.join(BUILD, os.path.basename(s) + ".o")
        flags = host_flags + HOST_FILE_FLAGS.get(os.path.basename(s), [])
        cmd = ["g++"] + flags + ["-c", s, "-o", obj]
        jobsl.append((cmd, s, obj, _stamp([s] + hdrs, flags + ["force" if force else ""])))
    objs, changed = [], False
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_compile, *j) for j in jobsl]
        for f in futs:
            obj, ch, err = f.result()
            objs.append(obj)
            changed |= ch
            if verbose and err:
                print(err, file=sys.stderr)
    if changed or force or not os.path.exists(OUT):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        link = ["g++", "-shared", "-o", OUT + ".tmp"] + (SAN_FLAGS if SANITIZE else []) + objs + [
            "-L" + tlib, "-Wl,-rpath," + tlib,
            "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
            "-lamdhip64", "-lrccl"]  # torch's bundled librccl: the same runtime ProcessGroupNCCL uses
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
        os.replace(OUT + ".tmp", OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args(argv)
    out = build(a.j, a.force, a.v)
    print(out)


if __name__ == "__main__":
    main()
