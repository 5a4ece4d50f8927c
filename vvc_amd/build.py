"""Builds libvvcr (HIP, gfx950) and the oracle's C restatement. No JIT caches: everything is built
in-tree so the shared objects travel with the repository snapshot to the GPU box."""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "vvc_amd", "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(ROOT, "vvc_amd", "libvvcr.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# host code for x86-64-v3 (AVX2 / BMI2 / LZCNT: both this container's Xeon and the GPU box's EPYC 9575F have
# them): the CABAC pass -3.5 %, motion derivation -2.5 % on the box (tools/host_ab_time.py, single thread)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + os.path.join(ROOT, "include"),
         "-Wno-unused-result", "-munsafe-fp-atomics", "-Xarch_host", "-march=x86-64-v3"]


def _compile(src, extra=(), obj_dir=OBJ):
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + \
        [os.path.join(ROOT, "include", h) for h in ("vvcr.h", "vvcp.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [HIPCC] + FLAGS + list(extra) + ["-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + FLAGS + list(extra) + ["-x", "hip", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return obj


def build_lib(jobs=8, extra=(), obj_dir=OBJ, lib=LIB):
    """extra/obj_dir/lib: diagnostics variants (e.g. tools/intra_prof.py's -DVVCR_INTRA_PROF build)."""
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, extra, obj_dir), srcs))
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-pthread", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return lib


APP = os.path.join(ROOT, "vvc_amd", "vvcdec")


def build_app(lib=LIB):
    """vvc_amd/vvcdec: the DecoderApp-compatible command-line decoder (vvc_amd/app/vvcdec.cpp) over the
    C-ABI of libvvcr.so (found next to it at run time)."""
    src = os.path.join(ROOT, "vvc_amd", "app", "vvcdec.cpp")
    deps = [src, lib] + [os.path.join(ROOT, "include", h) for h in ("vvcr.h", "vvcp.h")]
    if os.path.exists(APP) and os.path.getmtime(APP) >= max(os.path.getmtime(d) for d in deps):
        return APP
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-pthread", "-I" + os.path.join(ROOT, "include"), "-o", APP, src,
           lib, "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("vvcdec build failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return APP


def build_oracle():
    """oracle/ C restatement -> oracle/_build/liboracle.so (test infrastructure)."""
    src_dir = os.path.join(ROOT, "oracle")
    out_dir = os.path.join(src_dir, "_build")
    os.makedirs(out_dir, exist_ok=True)
    srcs = sorted(os.path.join(src_dir, f) for f in os.listdir(src_dir) if f.endswith(".c"))
    out = os.path.join(out_dir, "liboracle.so")
    if not srcs:
        return None
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(s) for s in srcs + [os.path.join(src_dir, "oracle.h")]):
        cmd = ["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-Wall", "-o", out] + srcs + ["-lm"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("oracle build failed:\n%s%s" % (r.stdout, r.stderr))
    return out


def build_reference(jobs=8):
    """oracle/_ref: the reference (VTM 7.3) built from /root/reference's own sources by oracle/ref.mk —
    DecoderApp (CPU baseline), EncoderApp (test streams), vtm_capture (golden fixtures). Test
    infrastructure; skipped where the reference is absent (the GPU box uses the prebuilt files)."""
    if not os.path.isdir("/root/reference/source"):
        return None
    r = subprocess.run(["make", "-f", os.path.join(ROOT, "oracle", "ref.mk"), "-j%d" % jobs, "all"],
                       cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("reference build failed:\n%s%s" % (r.stdout[-4000:], r.stderr[-4000:]))
    return os.path.join(ROOT, "oracle", "_ref")


if __name__ == "__main__":
    print(build_lib())
    print(build_app())
    print(build_oracle())
