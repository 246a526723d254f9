"""The reference's own test driver compiles and links UNCHANGED against the drop-in headers.

INTEGRATION.md promises that code written against the reference's API switches by changing the
include path and adding -lseqalib_hip.  This pins it: /root/reference/test/Test.cpp is compiled
in place (read by absolute path, as oracle/Makefile reads the reference; nothing of it is copied
into this tree or travels to the GPU box) with test/Makefile:2's own command
(`$(CXX) Test.cpp -o Test -std=c++14 -O2 -I../include/`), the include path pointed at
include/seqalib, and linked against libseqalib_hip.so.  Our headers must not add a single warning
under those flags.  Skipped where the reference tree is absent (the GPU box).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_TEST = "/root/reference/test/Test.cpp"
LIBDIR = os.path.join(ROOT, "seqalib_amd", "lib")


@pytest.mark.skipif(not os.path.exists(REF_TEST), reason="reference tree absent (GPU box)")
@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_reference_test_driver_compiles_unchanged(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libseqalib_hip.so")):
        pytest.skip("libseqalib_hip.so not built (make lib)")
    exe = tmp_path / "Test"
    cmd = ["g++", REF_TEST, "-o", str(exe), "-std=c++14", "-O2", "-I" + os.path.join(ROOT, "include", "seqalib"),
           "-L" + LIBDIR, "-lseqalib_hip", "-Wl,-rpath," + LIBDIR, "-pthread"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    ours = [ln for ln in p.stderr.splitlines() if "include/seqalib" in ln and "warning" in ln]
    assert not ours, ours
    assert exe.exists()
