"""C-ABI surface: libvvcr exports every entry point include/vvcr.h declares (no GPU needed)."""
import os
import re
import subprocess

from vvc_amd import native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_and_library_agree():
    hdr = open(os.path.join(ROOT, "include", "vvcr.h")).read()
    declared = set(re.findall(r"^(?:int|int64_t|const char \*|void \*)\s*(vvcr_\w+)\(", hdr, re.M))
    assert declared == set(N.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (vvcr_\w+)", out))
    missing = declared - exported
    assert not missing, missing


def test_parser_header_and_library_agree():
    """include/vvcp.h (the host parser's entry points) is exported by the same library"""
    hdr = open(os.path.join(ROOT, "include", "vvcp.h")).read()
    declared = set(re.findall(r"^(?:int|int64_t|const char \*|void \*)\s*(vvcp_\w+)\(", hdr, re.M))
    assert len(declared) > 10
    out = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    missing = declared - set(re.findall(r" T (vvcp_\w+)", out))
    assert not missing, missing


def test_library_loads_without_gpu():
    L = N.lib()
    assert L.vvcr_last_error(None) is not None
