"""Build the gfx950 kernel library in-tree: ``induction_network_on_fewrel_amd/_ina_kernels.so``.

* every ``csrc/kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` (device + host stub),
* ``csrc/bindings.cpp`` (torch op registrations, host only) by ``g++`` against torch's headers,
* everything is linked by ``hipcc -shared`` against torch's libs (the process's single HIP runtime).

Incremental: an object is rebuilt when its source or any header is newer. ``python csrc/build.py``
or ``from csrc.build import build; build()``. Works without a GPU (cross-compilation).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
# Experiment variants: INA_BUILD_TAG=<tag> INA_VARIANT_FLAGS="-DX=1" builds variants/_ina_kernels_<tag>.so
# (load it with INA_KERNEL_LIB=<path>); the default build is the in-tree package library.
# Host AddressSanitizer build: `python csrc/build.py --asan` (or INA_ASAN=1) ->
# variants/_ina_kernels_asan.so, host code only (bindings + the kernels' host launch stubs;
# `-fsanitize=address` goes after -Xarch_host on the hipcc lines, GPU code is never instrumented).  Load it
# in a CPU process with LD_PRELOAD=$(gcc -print-file-name=libasan.so) (tests/test_native_build.py).
_ASAN = os.environ.get("INA_ASAN") == "1" or "--asan" in sys.argv
if _ASAN:
    os.environ.setdefault("INA_BUILD_TAG", "asan")
_TAG = os.environ.get("INA_BUILD_TAG", "")
_VFLAGS = os.environ.get("INA_VARIANT_FLAGS", "").split()
# per-file variant flags: INA_VARIANT_FILE_FLAGS="rec_attn.hip:-fno-slp-vectorize;lstm.hip:-DX=1"
_VFILE = {f: fl.split(",") for f, fl in (e.split(":", 1) for e in os.environ.get("INA_VARIANT_FILE_FLAGS", "").split(";")
                                          if ":" in e)}
OUT_DIR = os.path.join(ROOT, "build", "obj" + (f"_{_TAG}" if _TAG else ""))
LIB = (os.path.join(ROOT, "variants", f"_ina_kernels_{_TAG}.so") if _TAG
       else os.path.join(ROOT, "induction_network_on_fewrel_amd", "_ina_kernels.so"))
HOST_LIB = os.path.join(ROOT, "induction_network_on_fewrel_amd", "_ina_host" + sysconfig.get_config_var("EXT_SUFFIX"))
ARCH = os.environ.get("INA_OFFLOAD_ARCH", "gfx950")
# Per-file code generation flags.  rec_attn.hip: MFMA results in VGPRs (gfx950's unified register
# file allows it); the default AGPR form cost 12 v_accvgpr_read per token step of the attention
# forward, whose tanh / softmax epilogue reads every accumulator back on the VALU.  No SLP
# vectoriser there: its v_pk_fma_f32 broadcasts pair a scalar with whatever register sits next to it,
# and the wait-count pass then treats a prefetch landing in that neighbour as a dependency (a
# vmcnt(0) in the middle of the backward's step); 444 vs 464 us forward, 746 vs 756 us backward.
# lstm.hip: no SLP vectoriser either -- its packed v_pk_mul / v_pk_fma f32 next to the recurrences' MFMAs
# cost more issue cycles than the scalar forms (MI355X_MICROARCH: packed f32 beside MFMAs is an
# anti-lever): 1,925,812 / 1,897,512 vs 1,886,461 / 1,885,572 episodes/s same box (profiles/r4_noslp).
# routing.hip likewise (fwd 31 -> 26 us, bwd 87 -> 80 us; ntn.hip measured mixed: fwd -8, bwd +16 us, kept;
# profiles/r4_noslp/noslp2).
FILE_FLAGS = {"rec_attn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"],
              "lstm.hip": ["-fno-slp-vectorize"], "routing.hip": ["-fno-slp-vectorize"],
              "bert.hip": ["-fno-slp-vectorize"]}   # BERT 108.75 / 108.75 vs 108.37 / 108.29 (r4_noslp/noslp3)


def _torch_paths():
    import torch  # noqa: F401
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths()
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    return inc, lib


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_host() -> str:
    """The host-only CPython extension (no torch / HIP: checkpoint CRC32C on any host, csrc/host/ina_host.c).
    Built FIRST by build() and on its own by ``python csrc/build.py --host`` (a CPU-only host without hipcc)."""
    hsrc = os.path.join(CSRC, "host", "ina_host.c")
    if _newer(HOST_LIB, [hsrc, __file__]):
        _run([shutil.which("gcc") or "cc", "-O2", "-fPIC", "-shared", "-I" + sysconfig.get_paths()["include"], hsrc,
              "-o", HOST_LIB])
    return HOST_LIB


def build(verbose: bool = False, jobs: int = 0) -> str:
    build_host()
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "include", "*.h"))
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    inc, tlib = _torch_paths()
    jobs = jobs or min(8, os.cpu_count() or 4)
    tasks = []
    objs = []
    for src in kernels:
        obj = os.path.join(OUT_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(obj, [src, *headers, __file__]):
            tasks.append([hipcc, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", *_VFLAGS,
                          *(["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
                            if _ASAN else []),
                          *FILE_FLAGS.get(os.path.basename(src), []),
                          *_VFILE.get(os.path.basename(src), []), "-I" + os.path.join(CSRC, "include"), "-c", src,
                          "-o", obj])
    for bsrc in sorted(glob.glob(os.path.join(CSRC, "*.cpp"))):   # host-only torch bindings (g++)
        bobj = os.path.join(OUT_DIR, os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if _newer(bobj, [bsrc, *headers, __file__]):
            cxx = shutil.which("g++") or "c++"
            cmd = [cxx, "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                   "-D_GLIBCXX_USE_CXX11_ABI=1", "-I/opt/rocm/include"]
            if _ASAN:
                cmd += ["-fsanitize=address", "-fno-omit-frame-pointer", "-g"]
            cmd += ["-I" + p for p in inc]
            cmd += ["-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(CSRC, "include"), "-c", bsrc, "-o",
                    bobj]
            tasks.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for out in ex.map(_run, tasks):
            if verbose and out.strip():
                print(out)
    if tasks or not os.path.exists(LIB) or _newer(LIB, objs):
        cmd = [hipcc, "-shared", "-fPIC", "-o", LIB, *objs, f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-lc10",
               "-lc10_hip", "-ltorch_hip", "-lrccl", f"-Wl,-rpath,{tlib}"]
        if _ASAN:   # the host ASan runtime (gcc's; the process preloads it)
            cmd += [subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                                   text=True).stdout.strip()]
        _run(cmd)
    return LIB


if __name__ == "__main__":
    print(build_host() if "--host" in sys.argv else build(verbose="-v" in sys.argv))
