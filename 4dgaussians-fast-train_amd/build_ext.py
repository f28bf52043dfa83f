"""In-tree build of the MI355X rasterizer and kNN initialiser.

  diff_gaussian_rasterization/libgs4d.so -- HIP kernels + C ABI (include/gs4d.h), hipcc --offload-arch=gfx950
  diff_gaussian_rasterization/_C.*.so    -- PyTorch-ROCm binding of the rasterizer (csrc/torch_glue.cpp)
  simple_knn/_C.*.so                     -- PyTorch-ROCm binding of distCUDA2 (csrc/knn_glue.cpp)
  gs4d_train/_C.*.so                     -- PyTorch-ROCm binding of the train-step kernels (csrc/train_glue.cpp)

The modules link libgs4d.so by rpath, so both packages load from the tree (never from site-packages
or a JIT cache).  Usage: python build_ext.py [--force] [-v]
"""
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "diff_gaussian_rasterization")
OBJ = os.path.join(HERE, "build", "obj")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("GS4D_ARCH", "gfx950")
HIP_SOURCES = ["preprocess.hip", "binning.hip", "render.hip", "preprocess_backward.hip", "knn.hip", "train_tail.hip", "hexplane.hip", "capi.hip"]
# Per-Gaussian math (K1, K8/K9) is compiled without FMA contraction: it costs nothing measurable
# (those kernels are tiny) and keeps radii / tile rects -- discrete decisions -- bit-identical to the
# oracle.  The per-pixel blend kernels keep contraction for throughput.
# (package, pybind glue) pairs: each package gets an in-tree `_C` module over libgs4d
BINDINGS = [("diff_gaussian_rasterization", "torch_glue.cpp"), ("simple_knn", "knn_glue.cpp"), ("gs4d_train", "train_glue.cpp")]
NO_CONTRACT = {"preprocess.hip", "preprocess_backward.hip", "binning.hip", "knn.hip", "train_tail.hip", "hexplane.hip"}
# The blend kernels pack pixel pairs explicitly (ext_vector_type(2) -> v_pk_*_f32); the SLP vectorizer
# would also pack their scalar horizontal adds, paying register moves for a v_pk_add_f32 (4 issue cycles)
# where two v_add_f32 cost about 5 (tools/bench/valu_rates.hip), so it is off for render.hip.
NO_SLP = {"render.hip"}
# The blend kernels and the binning take LLVM's iterative ILP scheduler: measured on one box, render forward
# 104.5 -> 103.3 us, backward 162.9 -> 161.2 us, the train-like tile sort 43.4 -> 42.5 us (tools/ab_lib.sh,
# tools/ab_train_kernels.sh); the HexPlane backward got slower with it (+4 us) and train_tail.hip crashes the
# register allocator under it, so the other files keep the default.
SCHED_ILP = {"render.hip", "binning.hip"}
HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-Wall",
               "-Wno-unused-result", "-I" + INCLUDE]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def lib_path():
    return os.path.join(OUT, "libgs4d.so")


def module_path(pkg="diff_gaussian_rasterization"):
    return os.path.join(HERE, pkg, "_C" + ext_suffix())


def build(force=False, verbose=False, report=True):
    """Compile what is out of date; report=True prints one line per object / library / module saying whether it
    was compiled or reused (mtimes of its sources, the headers and this script)."""
    os.makedirs(OBJ, exist_ok=True)
    done = []  # (artifact, "compiled" | "reused")
    headers = [os.path.join(CSRC, h) for h in ("gs4d_math.h", "gs4d_internal.h", "radix_sort.h")] + [os.path.join(INCLUDE, h) for h in ("gs4d.h", "gs4d_train.h")]
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

    def compile_one(src):
        s = os.path.join(CSRC, src)
        o = os.path.join(OBJ, src + ".o")
        if force or _newer(o, [s, os.path.abspath(__file__)] + headers):
            extra = (["-ffp-contract=off"] if src in NO_CONTRACT else []) + (["-fno-slp-vectorize"] if src in NO_SLP else []) \
                + (["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"] if src in SCHED_ILP else [])
            _run([hipcc, *HIPCC_FLAGS, *extra, "-c", s, "-o", o], verbose)
            return o, "compiled"
        return o, "reused"

    with cf.ThreadPoolExecutor(max_workers=min(8, len(HIP_SOURCES))) as ex:
        res = list(ex.map(compile_one, HIP_SOURCES))
    objs = [o for o, _ in res]
    done += res
    lib = lib_path()
    if force or _newer(lib, objs):
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", lib], verbose)
        done.append((lib, "compiled"))
    else:
        done.append((lib, "reused"))

    # torch bindings: (package dir, glue source); each links libgs4d from diff_gaussian_rasterization/
    import torch
    from torch.utils import cpp_extension as ce
    tdir = os.path.dirname(torch.__file__)
    incs = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames \
        else ce.include_paths(cuda=True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    mods = []
    for pkg, glue_src in BINDINGS:
        mod = module_path(pkg)
        glue = os.path.join(CSRC, glue_src)
        rel = os.path.relpath(OUT, os.path.join(HERE, pkg))
        if force or _newer(mod, [glue, lib, os.path.join(INCLUDE, "gs4d.h"), os.path.join(INCLUDE, "gs4d_train.h")]):
            cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", glue, "-o", mod,
                   f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                   "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2",
                   "-I" + sysconfig.get_paths()["include"]] + ["-I" + p for p in incs] + [
                "-L" + os.path.join(tdir, "lib"), "-L/opt/rocm/lib", "-L" + OUT,
                "-lgs4d", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64",
                "-lrocblas",
                "-Wl,-rpath,$ORIGIN" + ("" if rel == "." else "/" + rel), "-Wl,-rpath," + os.path.join(tdir, "lib"),
                "-Wl,-rpath,/opt/rocm/lib"]
            _run(cmd, verbose)
            done.append((mod, "compiled"))
        else:
            done.append((mod, "reused"))
        mods.append(mod)
    if report:
        for path, how in done:
            print(f"gs4d build: {how:8s} {os.path.relpath(path, HERE)}", flush=True)
    return lib, mods


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose="-v" in sys.argv)
    print("built", lib_path(), *[module_path(p) for p, _ in BINDINGS])
