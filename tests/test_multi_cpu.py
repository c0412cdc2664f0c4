"""CPU: the C-ABI multi-GPU extension (rsm_multi.cpp, product code) exchanging data
between G = 2, 4, 8 ranks -- on host "devices": rsm_multi.cpp and the product host
runtime are built against a stubbed HIP runtime whose encode launches compute the
real parity with the C oracle (tests/native/hip_stub.cpp, RSM_STUB_ORACLE) and a
stubbed RCCL whose grouped all-gather and send/recv move the bytes between the
ranks' buffers with RCCL's semantics (tests/native/rccl_stub.cpp).  Checks, for
k in {8, 64} (GF(2^8)) and k = 256 (GF(2^16)), both schedules: the whole EDS of
rsm_multi_extend_square and every GPU's rows / column slice / all-gathered top half
of rsm_multi_extend_dev, bit-exact against the oracle's 2D extension
(extendeddatasquare.go:50-77 at G = 1 vs sharded).  The same
executable also runs under ThreadSanitizer with threads sharing one clique and
owning cliques of their own."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rsmt2d_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
CXX = "/opt/rocm/lib/llvm/bin/clang++"
CPP = [os.path.join(CSRC, f) for f in ("rsm_multi.cpp", "rsm_runtime.cpp", "eds.cpp", "merkle.cpp", "gf16_tables.cpp")] + [
    os.path.join(NATIVE, f) for f in ("hip_stub.cpp", "rccl_stub.cpp", "multi_check.cpp")]
ORACLE_C = os.path.join(ROOT, "oracle", "leopard_oracle.c")


def _build(tmp, san):
    extra = ["-fsanitize=thread"] if san else []
    flags = ["-O1", "-g", *extra, "-D__HIP_PLATFORM_AMD__", "-DRSM_STUB_ORACLE", "-I/opt/rocm/include"]
    procs, objs = [], []
    for s in CPP + [ORACLE_C]:
        o = os.path.join(tmp, os.path.basename(s) + (".tsan" if san else "") + ".o")
        lang = ["-x", "c", "-std=c11"] if s.endswith(".c") else ["-x", "c++", "-std=c++20"]
        procs.append((s, subprocess.Popen([CXX, *flags, *lang, "-c", s, "-o", o], stdout=subprocess.PIPE,
                                          stderr=subprocess.STDOUT)))
        objs.append(o)
    for s, p in procs:
        out = p.communicate(timeout=600)[0].decode(errors="replace")
        assert p.returncode == 0, f"{s}:\n{out[-3000:]}"
    exe = os.path.join(tmp, "multi_check" + ("_tsan" if san else ""))
    subprocess.run([CXX, *extra, *objs, "-o", exe, "-lpthread"], check=True, timeout=300)
    return exe


@pytest.fixture(scope="module")
def tmp(tmp_path_factory):
    if not os.path.exists(CXX):
        pytest.skip("ROCm clang++ not present")
    return str(tmp_path_factory.mktemp("multi"))


def test_multi_gpu_exchange_bit_exact(tmp):
    exe = _build(tmp, san=False)
    r = subprocess.run([exe], capture_output=True, timeout=600)
    assert r.returncode == 0, r.stderr.decode(errors="replace")[-6000:]
    assert b"multi_check: ok" in r.stdout


def test_multi_gpu_exchange_under_tsan(tmp):
    exe = _build(tmp, san=True)
    r = subprocess.run([exe, "quick"], capture_output=True, timeout=900,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1"))
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-6000:]
    assert "ThreadSanitizer" not in err, err[-6000:]
    assert b"multi_check: ok" in r.stdout
