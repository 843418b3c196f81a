"""CPU: the library's host C++ (host BM25, RRF, the Snowball stemmer, the
native index file and its streaming writer) built with
-fsanitize=address,undefined by g++ and driven by tests/asan/asan_driver.cpp
("a -fsanitize=address host build").  No GPU code is
instrumented: the file's device entry points only link against the HIP
runtime."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hybrid-rag-colbertv2_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not found")
def test_host_cpp_under_asan_and_ubsan(tmp_path):
    exe = str(tmp_path / "asan_driver")
    srcs = [os.path.join(ROOT, "tests", "asan", "asan_driver.cpp")] + [
        os.path.join(CSRC, f) for f in ("host_bm25.cpp", "host_rrf.cpp", "text_en.cpp", "index_file.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-fno-sanitize-recover=undefined", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
           "-I", "/opt/rocm/include", *srcs, "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64",
           "-pthread", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failed checks" in r.stdout
