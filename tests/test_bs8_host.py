"""CPU check of the bit-sliced GF(2^8) encode arithmetic (rsmt2d_amd/csrc/bs8.hpp).

tests/native/bs8_host.cpp runs the kernel's templates (bytes -> bit-planes, the
per-wave small layers, the LDS layout exchange as an index relabelling, the
shared large layers, planes -> bytes) on the host and compares every parity byte
with the oracle's leo_encode (klauspost leopard8 restatement)."""
import os
import shutil
import subprocess

import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def bs8_host(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    oracle.build()
    exe = str(tmp_path_factory.mktemp("bs8") / "bs8_host")
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["g++", "-O1", "-std=c++20", "-o", exe, os.path.join(HERE, "native", "bs8_host.cpp"),
                    "-L" + odir, "-lleopard_oracle", "-Wl,-rpath," + odir], check=True)
    return exe


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("k,S", [(128, 512), (65, 64), (100, 192), (127, 1024)])
def test_bitsliced_encode_matches_oracle(bs8_host, k, S, split):
    """split 0: the two-launch kernel's schedule (small layout e = 16A + j); split 1:
    the half-split schedule of the queue kernel (layout S', e = (j & 7) + 8A + 64 (j >> 3),
    per-half small / large layers, transpose exchange per half)."""
    r = subprocess.run([bs8_host, str(k), str(S), str(k * 7919 + S), str(split)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
