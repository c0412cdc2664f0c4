"""CPU: ThreadSanitizer build of the product's host code (rsm_runtime.cpp, eds.cpp,
merkle.cpp, gf16_tables.cpp) against a stubbed HIP runtime (tests/native/hip_stub.cpp),
hammered by 85 threads on one context (tests/native/tsan_hammer.cpp): concurrent
Encode/Decode (GF(2^8) and GF(2^16)), host-memory and device-resident extensions,
device roots on caller streams, stream create/destroy and the EDS layer.  The
reference runs its Codec from up to 2k goroutines under `go test -race`
(.github/workflows/ci.yml:41-44); this is that check for the C ABI.  The stub's
"kernels" compute nothing, so results are not checked here (tests/test_gpu_runtime.py
checks them on the GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rsmt2d_amd", "csrc")
NATIVE = os.path.join(ROOT, "tests", "native")
CXX = "/opt/rocm/lib/llvm/bin/clang++"
FLAGS = ["-std=c++20", "-O1", "-g", "-fsanitize=thread", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-x", "c++"]
SOURCES = [os.path.join(CSRC, f) for f in ("rsm_runtime.cpp", "eds.cpp", "merkle.cpp", "gf16_tables.cpp")] + [
    os.path.join(NATIVE, "hip_stub.cpp"), os.path.join(NATIVE, "tsan_hammer.cpp")]

RACY = r"""
#include <thread>
int g;
int main() { std::thread a([] { for (int i = 0; i < 100000; ++i) g++; }); for (int i = 0; i < 100000; ++i) g++; a.join(); }
"""


def _build(tmp, srcs, out):
    objs = []
    procs = []
    for s in srcs:
        o = os.path.join(tmp, os.path.basename(s) + ".o")
        procs.append(subprocess.Popen([CXX, *FLAGS, "-c", s, "-o", o], stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        objs.append(o)
    for p, s in zip(procs, srcs):
        out_txt = p.communicate(timeout=600)[0].decode(errors="replace")
        assert p.returncode == 0, f"{s}:\n{out_txt[-3000:]}"
    exe = os.path.join(tmp, out)
    subprocess.run([CXX, "-fsanitize=thread", *objs, "-o", exe, "-lpthread"], check=True, timeout=300)
    return exe


@pytest.fixture(scope="module")
def tmp(tmp_path_factory):
    if not os.path.exists(CXX):
        pytest.skip("ROCm clang++ not present")
    return str(tmp_path_factory.mktemp("tsan"))


def test_sanitizer_is_live(tmp):
    """The detector itself fires on a deliberate race (so a clean run means something)."""
    src = os.path.join(tmp, "racy.cpp")
    open(src, "w").write(RACY)
    exe = os.path.join(tmp, "racy")
    subprocess.run([CXX, "-std=c++20", "-O1", "-fsanitize=thread", src, "-o", exe, "-lpthread"], check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, timeout=120, env=dict(os.environ, TSAN_OPTIONS="exitcode=66"))
    assert r.returncode == 66 and b"data race" in r.stderr


def test_host_runtime_has_no_data_races(tmp):
    exe = _build(tmp, SOURCES, "hammer")
    r = subprocess.run([exe], capture_output=True, timeout=600,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1"))
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-6000:]
    assert "ThreadSanitizer" not in err, err[-6000:]
    assert b"hammer: ok" in r.stdout
