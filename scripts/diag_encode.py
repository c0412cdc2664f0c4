"""Diagnostic: which parity symbols / byte ranges of a single k=128 codeword encode
differ from the oracle (used to localise a bit-sliced kernel fault)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle
import rsmt2d_amd as R

k = 128
S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
rng = np.random.default_rng(1)
data = [rng.integers(0, 256, S, dtype=np.uint8).tobytes() for _ in range(k)]
got = np.frombuffer(b"".join(R.NewLeoRSCodec().Encode(data)), np.uint8).reshape(k, S)
want = np.frombuffer(b"".join(oracle.encode(data)), np.uint8).reshape(k, S)
bad = got != want
print("S=%d bad bytes %d of %d" % (S, bad.sum(), bad.size))
syms = np.nonzero(bad.any(axis=1))[0]
print("bad parity symbols:", syms.tolist())
# per 16-byte piece (lane piece), over all bad symbols
pieces = np.nonzero(bad.reshape(k, S // 16, 16).any(axis=(0, 2)))[0]
print("bad 16-byte pieces:", pieces.tolist()[:80])
for e in syms[:4]:
    print("sym", e, "bad pieces", np.nonzero(bad[e].reshape(S // 16, 16).any(axis=1))[0].tolist()[:40])
