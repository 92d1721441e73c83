"""Runs the C++ C-ABI test program (tests/cpp/rbc_test.cpp: Test_shard,
Test_validateMessage, Test_interpolate named after rbc/rbc_internal_test.go,
klauspost TestOneEncode, reconstruct, concurrent batcher) on the GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_cpp_abi_suite():
    exe = os.path.join(HERE, "cpp", "rbc_test")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(HERE, "cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("PASS") == 8


def test_cpp_abi_builds():
    """The C++ client compiles against include/rbc_gpu.h and links the .so."""
    r = subprocess.run(["make", "-C", os.path.join(HERE, "cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
