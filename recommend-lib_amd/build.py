"""Build libbprmf_amd.so in-tree for gfx950 with hipcc (no torch JIT cache, no pip install).

The shared library is the product: the gfx950 kernels (kernels.hip, segment.hip, step.hip,
dist.hip) + the C ABI of include/bprmf.h (capi.cpp, dist.cpp; RCCL for the sharded runner).
It is placed next to this file so it travels to the GPU box with the repo.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libbprmf_amd.so")
SOURCES = [os.path.join(HERE, "csrc", n) for n in ("kernels.hip", "segment.hip", "step.hip", "dist.hip", "topk.hip", "ncf.hip", "capi.cpp", "dist.cpp", "ncf_capi.cpp", "ingest.cpp", "mf.hip", "mf_capi.cpp", "bprfm.hip", "bprfm_capi.cpp", "sgns.hip", "sgns_capi.cpp")]
HEADERS = [os.path.join(HERE, "csrc", n) for n in ("kernels.h", "device_common.h", "handle.h", "ncf_kernels.h", "mf_kernels.h", "bprfm_kernels.h", "sgns_kernels.h")] + [os.path.join(ROOT, "include", n) for n in ("bprmf.h", "ncf.h", "mf.h", "bprfm.h", "sgns.h")]
ARCH = os.environ.get("BPRMF_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def is_stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(s) > t for s in SOURCES + HEADERS)


def _compile(args):
    cmd, src = args
    r = subprocess.run(cmd, capture_output=True, text=True)
    return src, r.returncode, r.stdout + r.stderr


def build(force=False, verbose=False, defines=(), out=None):
    """Compile every source to an object in parallel (objects outside the tree), then link.
    defines/out: a diagnostic variant (e.g. tools/ubench_build.py) with its own objects."""
    out = out or LIB
    if not force and out == LIB and not is_stale():
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    obj_dir = os.environ.get("BPRMF_OBJ_DIR", os.path.join("/tmp", "bprmf_amd_obj"))
    if defines:
        obj_dir += "_" + "_".join(d.lower() for d in defines)
    os.makedirs(obj_dir, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in HEADERS)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function", "-I", os.path.join(ROOT, "include")] + [f"-D{d}" for d in defines]
    jobs, objs = [], []
    for src in SOURCES:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            jobs.append(([hipcc()] + flags + ["-c", src, "-o", obj], src))
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8))
    with ThreadPoolExecutor(workers) as ex:
        for src, rc, log in ex.map(_compile, jobs):
            if verbose:
                print(f"compiled {src}", file=sys.stderr)
            if rc != 0:
                raise RuntimeError(f"hipcc failed on {src} ({rc}):\n{log}")
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp] + objs + \
          ["-L/opt/rocm/lib", "-lrccl", "-lrocblas"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
