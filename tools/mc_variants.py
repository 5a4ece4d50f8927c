"""Builds k_mc A/B variants of libvvcr (vvc_amd/libvvcr_<name>.so, run with VVCR_LIB=...; tools/gpu_kt_ab.sh).
  python tools/mc_variants.py name=-DDEF1=1,-DDEF2=3 [name2=...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vvc_amd import build as B  # noqa: E402

for arg in sys.argv[1:]:
    name, defs = arg.split("=", 1)
    extra = [d for d in defs.split(",") if d]
    lib = os.path.join(ROOT, "vvc_amd", "libvvcr_%s.so" % name)
    print(B.build_lib(extra=extra, obj_dir=os.path.join(ROOT, "build", "var_" + name), lib=lib))
