"""Host code under AddressSanitizer + UBSan: liblfm's host-only logic
(dis_project_amd/csrc/lfm_host.cpp: x-layout detection, the factorisation's step plan, the
host mirror of the trailing update's unit enumeration, the side-CU helper's sizing and lead
clamp, the device tenancy lock: mutual exclusion, shared admission, cross-process waits and the
turnstile) and the C++ oracle (oracle/lfm_cpu.cpp), built by tests/native/Makefile and run by
tests/native/host_check.cpp. CPU only."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan")
def test_host_code_under_asan_and_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "asan"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "host_check: all passed" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
