"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer.

Compiles tests/sanitize/host_check.cpp with the product's host-only codec half
(zs3server_amd/csrc/codec_host.hpp: coding matrix, permute and dyadic tables,
per-erasure-pattern reconstruct plans, XXH64), the scalar oracle (oracle/zs3_oracle.c)
and the CPU baseline (oracle/cpu_ref.cpp), all with -fsanitize=address,undefined and
halt-on-error, and runs the 60 erasureSelfTest KATs, every erasure pattern of every
(k, m) with k + m <= 8 against the oracle, the dyadic tables and cpu_ref on ragged
blocks.  CPU only.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_host_code_asan_ubsan(tmp_path):
    obj = tmp_path / "zs3_oracle.o"
    exe = tmp_path / "host_check"
    subprocess.check_call(["gcc", "-std=c99", *SAN, "-c", os.path.join(ROOT, "oracle", "zs3_oracle.c"), "-o", str(obj)])
    subprocess.check_call(["g++", "-std=c++17", *SAN, "-pthread",
                           os.path.join(ROOT, "tests", "sanitize", "host_check.cpp"),
                           os.path.join(ROOT, "oracle", "cpu_ref.cpp"), str(obj), "-o", str(exe)])
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_check: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sanitizer_is_live(tmp_path):
    """Negative control: the same flags catch a one-byte heap overflow."""
    src = tmp_path / "oob.cpp"
    src.write_text("#include <cstdlib>\nint main(){volatile char* p=(char*)std::malloc(8); p[8]=1; return 0;}\n")
    exe = tmp_path / "oob"
    subprocess.check_call(["g++", *SAN, str(src), "-o", str(exe)])
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:verify_asan_link_order=0")
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and ("heap-buffer-overflow" in r.stderr or "runtime error" in r.stderr), r.stderr
