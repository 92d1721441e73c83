"""ASan + UBSan over the host C++ that parses untrusted network input
(SURVEY 5, row "race detection / sanitizers"): csrc/rbc_node.cpp -- the
pb.Message / Go-JSON codec (rbc_pb_decode_rbc, rbc_json_decode_val/ready,
rbc_pb_encode_rbc) and the RBC state machine's message handling -- built
with -fsanitize=address,undefined against stub batcher symbols and driven by
tests/cpp/codec_fuzz.cpp: round trips, the malformed cases of
tests/test_protocol_codec.py, a libFuzzer-style loop of random bytes and
mutated valid messages, and 200 four-node rounds over mutated traffic.

The request batcher (csrc/batcher.cpp) is built unchanged under
ThreadSanitizer and under ASan + UBSan against an oracle-backed stand-in for
the context's asynchronous batch API (tests/cpp/batcher_race.cpp): client
threads submit random shard / validate / interpolate requests and complete
them by wait or poll, every result checked against the C oracle.

The host runtime behind the C ABI (csrc/capi.cpp: argument checks, pinned
staging and slots, tickets, rbc_acs_*, the reedsolomon.Encoder mirror, the
receive step's batch checks) is built with ASan + UBSan against a host-memory
stand-in for HIP, RCCL and the kernel launchers (tests/cpp/hip_stub.cpp: the
stub kernels touch exactly what the real ones write) and driven with random
arguments by tests/cpp/capi_fuzz.cpp.
CPU only; no GPU code is built or run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


@pytest.fixture(scope="module")
def fuzz_exe(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("san") / "codec_fuzz_san")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-Wall", "-o", exe, os.path.join(CPP, "codec_fuzz.cpp"),
           os.path.join(ROOT, "cleisthenes_amd", "csrc", "rbc_node.cpp")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_codec_and_state_machine_clean_under_asan_ubsan(fuzz_exe):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([fuzz_exe, "60000"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.stdout.startswith("ok"), r.stdout


CLANG = "/opt/rocm/lib/llvm/bin/clang"


def _build_batcher_race(tmp, san):
    ref = os.path.join(ROOT, "oracle", "c", "rbc_ref.c")
    srcs = [os.path.join(CPP, "batcher_race.cpp"), os.path.join(ROOT, "cleisthenes_amd", "csrc", "batcher.cpp")]
    # ThreadSanitizer from ROCm's clang: gcc 11's runtime does not intercept
    # pthread_cond_clockwait and reports condition_variable::wait_until as a
    # double lock
    cc, cxx = (CLANG, CLANG + "++") if san == "thread" else ("gcc", "g++")
    if not shutil.which(cc) or not shutil.which(cxx):
        pytest.skip(f"{cxx} not available")
    obj, exe = str(tmp / f"ref_{san}.o"), str(tmp / f"batcher_race_{san}")
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}"]
    if san != "thread":
        flags.append("-fno-sanitize-recover=all")
    for cmd in ([cc, *flags, "-c", ref, "-o", obj],
                [cxx, "-std=c++17", *flags, "-Wall", "-o", exe, *srcs, obj, "-lpthread"]):
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    return exe


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_batcher_clean_under_sanitizers(tmp_path, san):
    exe = _build_batcher_race(tmp_path, san)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, "8", "50"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    for bad in ("ThreadSanitizer", "AddressSanitizer", "runtime error", "FAIL"):
        assert bad not in r.stderr, r.stderr[-4000:]
    assert r.stdout.rstrip().endswith("ok"), r.stdout


def test_capi_host_runtime_clean_under_asan_ubsan(tmp_path):
    """Random arguments through every host-side entry point of the C ABI;
    caller buffers are exactly as large as the contract asks, so a read or
    write past them, or past a buffer the runtime sized itself, is reported."""
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    for h in ("hip/hip_runtime_api.h", "rccl/rccl.h"):  # capi.cpp's own includes (types only: hip_stub links)
        if not os.path.exists(os.path.join("/opt/rocm/include", h)):
            pytest.skip(f"/opt/rocm/include/{h} not available")
    exe = str(tmp_path / "capi_fuzz")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-o", exe,
           os.path.join(CPP, "capi_fuzz.cpp"), os.path.join(CPP, "hip_stub.cpp"),
           os.path.join(ROOT, "cleisthenes_amd", "csrc", "capi.cpp"), "-ldl", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    for seed in ("1", "20261017", "77"):
        r = subprocess.run([exe, "30000", seed], capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        for bad in ("AddressSanitizer", "runtime error", "FAIL"):
            assert bad not in r.stderr, r.stderr[-4000:]
        assert r.stdout.startswith("ok"), r.stdout
