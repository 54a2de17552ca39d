"""Build libbprmf_amd.so in-tree for gfx950 with hipcc (no torch JIT cache, no pip install).

The shared library is the product: the gfx950 kernels (kernels.hip, segment.hip, step.hip,
dist.hip) + the C ABI of include/bprmf.h (capi.cpp, dist.cpp; RCCL for the sharded runner).
It is placed next to this file so it travels to the GPU box with the repo.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libbprmf_amd.so")
SOURCES = [os.path.join(HERE, "csrc", n) for n in ("kernels.hip", "segment.hip", "step.hip", "hogwild.hip", "dist.hip", "topk.hip", "ncf.hip", "capi.cpp", "dist.cpp", "ncf_capi.cpp", "ingest.cpp", "status.cpp", "host_plan.cpp", "node_barrier.cpp", "mf.hip", "mf_capi.cpp", "bprfm.hip", "bprfm_capi.cpp", "sgns.hip", "sgns_capi.cpp")]
HEADERS = [os.path.join(HERE, "csrc", n) for n in ("kernels.h", "device_common.h", "handle.h", "ncf_kernels.h", "mf_kernels.h", "bprfm_kernels.h", "sgns_kernels.h", "status.h", "dist_body.h", "host_plan.h")] + [os.path.join(ROOT, "include", n) for n in ("bprmf.h", "ncf.h", "mf.h", "bprfm.h", "sgns.h")]
ARCH = os.environ.get("BPRMF_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def _flags(defines=()):
    return [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
            "-Wno-unused-function", "-I", os.path.join(ROOT, "include")] + [f"-D{d}" for d in defines]


def _link_cmd(out):
    return [hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", out]


def _stamp_path(out):
    return out + ".cmd"


def _stamp_text(defines=()):
    # everything that decides the objects: the tree they come from, the compiler, arch and flags
    return "\n".join([ROOT, hipcc()] + _flags(defines) + ["link:"] + _link_cmd("<out>")[1:]) + "\n"


def is_stale(out=LIB, defines=()):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    if any(os.path.getmtime(s) > t for s in SOURCES + HEADERS):
        return True
    try:
        with open(_stamp_path(out)) as f:
            return f.read() != _stamp_text(defines)
    except OSError:
        return True


def _compile(args):
    cmd, src = args
    r = subprocess.run(cmd, capture_output=True, text=True)
    return src, r.returncode, r.stdout + r.stderr


def build(force=False, verbose=False, defines=(), out=None):
    """Compile every source to an object in parallel (objects outside the tree), then link.
    defines/out: a diagnostic variant (e.g. tools/ubench_build.py) with its own objects."""
    out = out or LIB
    if not force and out == LIB and not is_stale(out, defines):
        return LIB
    from concurrent.futures import ThreadPoolExecutor
    # objects are keyed on the source tree, compiler, arch and flags: another checkout, another
    # arch or other defines never link these objects
    key = hashlib.sha1(_stamp_text(defines).encode()).hexdigest()[:16]
    obj_dir = os.environ.get("BPRMF_OBJ_DIR", os.path.join("/tmp", "bprmf_amd_obj_" + key))
    os.makedirs(obj_dir, exist_ok=True)
    hdr_t = max(os.path.getmtime(h) for h in HEADERS)
    flags = _flags(defines)
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
    cmd = _link_cmd(tmp) + objs + ["-L/opt/rocm/lib", "-lrccl", "-lrocblas"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    with open(_stamp_path(out), "w") as f:
        f.write(_stamp_text(defines))
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
